#!/bin/bash
# A/B of the lane-per-code-block turbo schedules (one vs two wavefronts per group) on configs[0],
# configs[2] and the headline: ./tools/ab_x.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
run() { name=$1; shift; timeout -k 10 240 python3 bench.py "$@" --no-cpu-baseline > $OUT/$name.json 2> $OUT/$name.err || exit 20; }
for s in lane lanex; do
  run c1_$s --config 1 --sched $s
  run c3_$s --config 3 --sched $s
  run c4_$s --sched $s --steps 5
done
echo done
