#!/bin/bash
# (record of a measurement: the knob is not in the tree -- apply profiles/r4/ab_cont_half/half_density.patch first)
# half-density continuation pairs (MI_TDEC_CONT_HALF: 1 = rounds after the first, 2 = every round): GPU suite on the
# default build, the bench-configuration tests in both half modes, then the same-box A/B (one stream, four streams)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 10; }
tail -1 $OUT/gpu_tests.log
for hm in 1 2; do
  MI_TDEC_CONT_HALF=$hm timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bench_config.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_half$hm.log 2>&1 || { tail -30 $OUT/gpu_half$hm.log; exit 11; }
  echo -n "half $hm: "; tail -1 $OUT/gpu_half$hm.log
done
for S in 1 4; do
  for i in 1 2; do
    for hm in 0 1 2; do
      MI_TDEC_CONT_HALF=$hm timeout -k 10 240 python3 bench.py --no-cpu-baseline --plan-steps 0 --streams $S --steps 60 > $OUT/s${S}_h${hm}_$i.json 2> $OUT/bench.err || exit 12
      echo -n "streams $S half $hm: "; python3 tools/bj.py $OUT/s${S}_h${hm}_$i.json
    done
  done
done
