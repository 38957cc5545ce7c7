#!/bin/bash
# Low-occupancy configs at 16 hardware queues: streams x turbo form (through gpurun): ./tools/lowocc_sweep2.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
run() { name=$1; shift; timeout -k 10 240 python3 bench.py --no-cpu-baseline --hw-queues 16 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 20; echo -n "$name: "; python3 tools/bj.py $OUT/$name.json; }
run c3_s8 --config 3 --streams 8
run c3_s8_p2 --config 3 --streams 8 --sched p2
run c3_s12_p2 --config 3 --streams 12 --sched p2
run c3_s16_p2 --config 3 --streams 16 --sched p2
run c3_s16 --config 3 --streams 16
run c5_s8 --config 5 --streams 8
run c5_s12 --config 5 --streams 12
run c1_s4 --config 1 --streams 4
run c1_s8 --config 1 --streams 8
echo done
