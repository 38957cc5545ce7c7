#!/bin/bash
# A/B of rate de-matching variants (make -C srsue_amd/csrc variant VNAME=<v> VFLAGS=...): ./tools/ab_rm.sh <tag> <v>...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > $OUT/base_$i.json 2> $OUT/base.err || exit 20
  for v in "$@"; do
    SRSUE_AMD_LIB=srsue_amd/libsrsue_amd_$v.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > $OUT/${v}_$i.json 2> $OUT/$v.err || exit 21
  done
done
echo done
