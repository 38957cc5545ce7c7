#!/bin/bash
# tree maxima / continuation checkpoints / stored w rows: GPU suite, then same-box A/Bs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$1/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/$1/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$1/gpu_tests.log
./tools/ab_serial.sh $1/s1 "notree p2cck8" || exit 2
BENCH_ARGS="--snr 21.5 --plan-steps 0" ./tools/ab_env.sh $1/wf MI_TDEC_STORE_W=0 - || exit 3
./tools/ab_round.sh $1/s4 "notree p2cck8" --plan-steps 0 || exit 4
for f in gpurun_out/$1/s4/*.json; do python3 tools/bj.py $f; done
