#!/bin/bash
# copy a tools/profile.sh result from gpurun_out/<tag> into profiles/<tag> (the judged record) and make its
# traffic.json the one bench.py reads:  ./tools/save_profile.sh <tag>
set -e
S=gpurun_out/$1; D=profiles/$1
mkdir -p $D
cp $S/bench.json $S/summary.json $S/summary.md $D/
cp $S/trace/run_kernel_stats.csv $D/rocprof_kernel_stats.csv
cp $S/pmc_fetch/run_counter_collection.csv $D/rocprof_pmc_fetch.csv
cp $S/pmc_write/run_counter_collection.csv $D/rocprof_pmc_write.csv
[ -f $S/pmc_valu/run_counter_collection.csv ] && cp $S/pmc_valu/run_counter_collection.csv $D/rocprof_pmc_valu.csv
[ -f $S/traffic.json ] && cp $S/traffic.json profiles/traffic.json
echo saved $D
