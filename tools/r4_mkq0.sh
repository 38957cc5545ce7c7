#!/bin/bash
# (record of a measurement: the knob is not in the tree -- apply profiles/r4/ab_mkq0/mkq0.patch first)
# q rows created by the waterfall's first launch and copied by the gather (MI_TDEC_MKQ0=1) vs re-quantised from the
# softbuffer (0): the bench-configuration tests, then same-box A/B (one stream, four streams)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_replan.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_cfg.log 2>&1 || { tail -30 $OUT/gpu_cfg.log; exit 10; }
tail -1 $OUT/gpu_cfg.log
for S in 1 4; do
  for i in 1 2; do
    for m in 0 1; do
      MI_TDEC_MKQ0=$m timeout -k 10 240 python3 bench.py --no-cpu-baseline --plan-steps 0 --streams $S --steps 60 > $OUT/s${S}_m${m}_$i.json 2> $OUT/bench.err || exit 12
      echo -n "streams $S mkq0 $m: "; python3 tools/bj.py $OUT/s${S}_m${m}_$i.json
    done
  done
done
