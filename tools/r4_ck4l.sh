#!/bin/bash
# 4-step checkpoints in the re-compaction rounds after the first (ck4l, MI_TDEC_P2C_CK_LATE=1) vs the current build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
./tools/ab_serial.sh $1/s1 ck4l || exit 11
./tools/ab_round.sh $1/s4 ck4l --plan-steps 0 || exit 12
for f in gpurun_out/$1/s4/*.json; do python3 tools/bj.py $f; done
