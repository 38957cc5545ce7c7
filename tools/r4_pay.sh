#!/bin/bash
# GPU suite on the dword payload stores, then serial A/B (pay8 = byte stores; pay2 = dword stores in the first launch only)
# and the 4-stream A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$1/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$1/gpu_tests.log; exit 10; }
tail -2 gpurun_out/$1/gpu_tests.log
./tools/ab_serial.sh $1/s1i "pay8 pay2" --max-its 1 --iterating-snr 0 || exit 11
./tools/ab_serial.sh $1/s1 "pay8 pay2" || exit 12
./tools/ab_round.sh $1/s4 "pay8 pay2" --plan-steps 0 || exit 14
for f in gpurun_out/$1/s4/*.json; do python3 tools/bj.py $f; done
