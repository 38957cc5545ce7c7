#!/bin/bash
# round-end record: the profile recipe on the final build, then the BASELINE configs sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
./tools/profile.sh $1_prof || exit 12
head -20 gpurun_out/$1_prof/summary.md
./tools/configs.sh $1_cfg || exit 13
for f in gpurun_out/$1_cfg/*.json; do echo -n "$(basename $f) "; python3 tools/bj.py $f; done
