#!/bin/bash
# round-end record: GPU suite, smoke(), the profile recipe (tools/profile.sh) on the final build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$1/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$1/gpu_tests.log; exit 10; }
tail -2 gpurun_out/$1/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$1/smoke.log 2>&1 || { tail -20 gpurun_out/$1/smoke.log; exit 11; }
tail -1 gpurun_out/$1/smoke.log
./tools/profile.sh $1_prof || exit 12
cat gpurun_out/$1_prof/summary.md | head -30
