#!/bin/bash
# rate de-matching XCD queues: GPU suite, then same-box A/B (one stream and four streams) and request counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
BENCH_ARGS="--streams 1 --plan-steps 0 --steps 60" ./tools/ab_env.sh $1/s1 MI_RM_XCDQ=1 MI_RM_XCDQ=0 || exit 2
BENCH_ARGS="--plan-steps 0" ./tools/ab_env.sh $1/s4 MI_RM_XCDQ=1 MI_RM_XCDQ=0 || exit 3
cd /tmp && export TMPDIR=/tmp
for x in 1 0; do
  MI_RM_XCDQ=$x timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/pmc_x$x/bench -o run -- python3 $R/bench.py --streams 1 --steps 20 --iterating-snr 0 --plan-steps 0 --no-cpu-baseline > $OUT/pmc_x$x.log 2>&1 || exit 4
  python3 $R/tools/rdreq_summary.py $OUT/pmc_x$x | grep -E "rm_combine|tdec_kernel_p2x|ofdm|chest"
done
