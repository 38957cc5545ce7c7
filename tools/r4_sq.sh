#!/bin/bash
# SQ counters of the final build (one stream, no planning block) and their summary
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
./tools/pmc_tdec.sh $1 --plan-steps 0 --streams 1 || exit 11
python3 tools/summarize_sq.py gpurun_out/$1 > gpurun_out/$1/summary.md || exit 12
cat gpurun_out/$1/summary.md
