#!/bin/bash
# check-pass diagnostics (wrong results: diag3 = no check pass, diag4 = + no decision stores; one iteration) and the
# A/B of the check pass's load ring (chk1 = one chunk ahead, the round-3 form)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$1; mkdir -p $OUT
for i in 1 2; do
  for v in cur diag3 diag4; do
    if [ $v = cur ]; then L=; else L=srsue_amd/libsrsue_amd_$v.so; fi
    SRSUE_AMD_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --plan-steps 0 --streams 1 --steps 40 --max-its 1 --iterating-snr 0 > $OUT/d_${v}_$i.json 2>$OUT/diag.err || exit 12
    echo -n "$v its1: "; python3 tools/bj.py $OUT/d_${v}_$i.json
  done
done
./tools/ab_serial.sh $1/s1 chk1 || exit 13
./tools/ab_round.sh $1/s4 chk1 --plan-steps 0 || exit 14
for f in gpurun_out/$1/s4/*.json; do python3 tools/bj.py $f; done
