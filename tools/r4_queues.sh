#!/bin/bash
# hardware queues per process (GPU_MAX_HW_QUEUES, 4 by default) x streams in flight, default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$1; mkdir -p $OUT
for i in 1 2 3; do
  for qs in "4 4" "8 4" "16 4"; do
    set -- $qs
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 240 python3 bench.py --no-cpu-baseline --plan-steps 0 --steps 100 --streams $2 --iterating-streams $2 > $OUT/q$1_s$2_$i.json 2> $OUT/q.err || exit 11
    echo -n "queues $1 streams $2: "; python3 tools/bj.py $OUT/q$1_s$2_$i.json
  done
done
