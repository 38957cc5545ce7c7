#!/bin/bash
# waterfall kernel trace (one stream) and the payload-store diagnostic (wrong results) of the check pass
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
for i in 1 2; do
  for v in cur diag5; do
    if [ $v = cur ]; then L=; else L=srsue_amd/libsrsue_amd_$v.so; fi
    SRSUE_AMD_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --plan-steps 0 --streams 1 --steps 40 --max-its 1 --iterating-snr 0 > $OUT/d_${v}_$i.json 2>$OUT/diag.err || exit 12
    echo -n "$v its1: "; python3 tools/bj.py $OUT/d_${v}_$i.json
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/wf -o run -- python3 $R/bench.py --snr 21.5 --streams 1 --steps 10 --plan-steps 0 --iterating-snr 0 --no-cpu-baseline > $OUT/wf.log 2>&1 || exit 11
python3 - $OUT/wf/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-40s calls %5s  avg %.3f ms  total %.1f ms" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
