#!/bin/bash
# 4-stream kernel timeline, QPP-table diagnostic (wrong results, timing only) and SQ counters of the turbo kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl -o run -- python3 $R/bench.py --steps 20 --plan-steps 0 --iterating-snr 0 --no-cpu-baseline > $OUT/tl.log 2>&1 || exit 11
python3 $R/tools/timeline.py $OUT/tl/run_kernel_trace.csv
{ timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cal -o run -- $R/tools/calib/pmc_calib > $OUT/cal.log 2>&1 && python3 $R/tools/calib/bw.py $OUT/cal/run_kernel_stats.csv; } || exit 14
cd $R
for i in 1 2; do
  for v in cur nopi piid; do
    if [ $v = cur ]; then L=; else L=srsue_amd/libsrsue_amd_$v.so; fi
    SRSUE_AMD_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --plan-steps 0 --streams 1 --steps 40 --max-its 1 --iterating-snr 0 > $OUT/diag_${v}_$i.json 2>$OUT/diag.err || exit 12
    echo -n "$v its1: "; python3 tools/bj.py $OUT/diag_${v}_$i.json
  done
done
./tools/pmc_tdec.sh $1/sq --streams 1 --plan-steps 0 || exit 13
python3 tools/summarize_sq.py gpurun_out/$1/sq
