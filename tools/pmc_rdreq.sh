#!/bin/bash
# Read requests by size (TCC_EA0_RDREQ_{32B,64B,128B} + total) for the calibration kernels and the default bench on one
# stream, so read bytes can be counted per request size instead of FETCH_SIZE's 64-B tally:  ./tools/pmc_rdreq.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/calib -o run -- $R/tools/calib/pmc_calib > $OUT/calib.log 2>&1 || exit 41
timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $OUT/bench -o run -- python3 $R/bench.py --streams 1 --steps 20 --iterating-snr 0 --plan-steps 0 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 42
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/bench_hit -o run -- python3 $R/bench.py --streams 1 --steps 20 --iterating-snr 0 --plan-steps 0 --no-cpu-baseline > $OUT/bench_hit.log 2>&1 || exit 43
python3 $R/tools/rdreq_summary.py $OUT
