#!/bin/bash
# round 5: counters of the wide-layout writer diagnostic and of configs[0]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
PMC_SET=traffic ./tools/pmc_ab.sh $1/pmc cur sbw || exit 3
python3 tools/pmc_summary.py $OUT/pmc rm_ tdec_kernel_p2x
BENCH_ARGS="--config 1" ./tools/pmc_ab.sh $1/pmc_c1 cur ck16 || exit 4
python3 tools/pmc_summary.py $OUT/pmc_c1 tdec
