#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration by access width (tools/calib/pmc_calib.hip): ./tools/calib/run.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $R/tools/calib/pmc_calib > $OUT/trace.log 2>&1 || exit 31
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $R/tools/calib/pmc_calib > $OUT/fetch.log 2>&1 || exit 32
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $R/tools/calib/pmc_calib > $OUT/write.log 2>&1 || exit 33
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
B = 2 << 30
for kind in ("fetch", "write"):
    f = glob.glob(out + "/" + kind + "/**/*counter_collection.csv", recursive=True)
    if not f: print(kind, "no csv"); continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        agg[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        kib = sum(v) / len(v)
        print("%-5s %-60s %14.0f KiB = %.3f x bytes" % (kind, k, kib, kib * 1024 / B))
PY
