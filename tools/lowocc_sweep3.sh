#!/bin/bash
# Low-occupancy configs, more streams (through gpurun): ./tools/lowocc_sweep3.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
run() { name=$1; shift; timeout -k 10 240 python3 bench.py --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 20; echo -n "$name: "; python3 tools/bj.py $OUT/$name.json; }
run c3_s16_p2_h16 --config 3 --streams 16 --sched p2 --hw-queues 16
run c3_s24_p2_h32 --config 3 --streams 24 --sched p2 --hw-queues 32
run c3_s32_p2_h32 --config 3 --streams 32 --sched p2 --hw-queues 32
run c5_s16_h16 --config 5 --streams 16 --hw-queues 16
run c1_s12_h16 --config 1 --streams 12 --hw-queues 16
echo done
