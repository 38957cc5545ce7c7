#!/bin/bash
# GPU measurement recipe (run through gpurun): default bench, rocprofv3 kernel trace + stats, and
# separate PMC passes for HBM traffic (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in own passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 11
SMALL="--sf-per-gpu 2000 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $SMALL > $OUT/prof_trace.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $SMALL > $OUT/prof_fetch.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $SMALL > $OUT/prof_write.log 2>&1 || exit 14
echo done
