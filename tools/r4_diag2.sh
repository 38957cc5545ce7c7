#!/bin/bash
# timing diagnostics (wrong results): no check pass (diag3), no check pass + no decision stores (diag4), one iteration
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$1; mkdir -p $OUT
for i in 1 2; do
  for v in cur diag3 diag4; do
    if [ $v = cur ]; then L=; else L=srsue_amd/libsrsue_amd_$v.so; fi
    SRSUE_AMD_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --plan-steps 0 --streams 1 --steps 40 --max-its 1 --iterating-snr 0 > $OUT/${v}_$i.json 2>$OUT/diag.err || exit 12
    echo -n "$v its1: "; python3 tools/bj.py $OUT/${v}_$i.json
  done
done
