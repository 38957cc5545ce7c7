#!/bin/bash
# split check pass + waterfall re-compaction rounds: GPU suite, then same-box A/Bs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$1/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/$1/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$1/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$1/smoke.log 2>&1 || { echo SMOKE FAILED; tail -5 gpurun_out/$1/smoke.log; exit 2; }
tail -1 gpurun_out/$1/smoke.log
./tools/ab_serial.sh $1/s1 nosplit || exit 3
BENCH_ARGS="--snr 21.5 --plan-steps 0" ./tools/ab_env.sh $1/wf MI_TDEC_ROUNDS=0 - || exit 4
./tools/ab_round.sh $1/s4 nosplit --plan-steps 0 || exit 5
for f in gpurun_out/$1/s4/*.json; do python3 tools/bj.py $f; done
