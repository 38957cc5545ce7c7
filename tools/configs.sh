#!/bin/bash
# BASELINE configs measured one after the other (through gpurun): ./tools/configs.sh <tag>
# each line is bench.py's JSON for one configuration (CPU baselines included, bounded samples)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
run() { name=$1; shift; timeout -k 10 240 python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 20; }
run c2 --config 2 --cpu-seconds 6
run c2_lane --config 2 --sched lane --no-cpu-baseline
run c3 --config 3 --cpu-seconds 6
run c3_s1 --config 3 --streams 1 --no-cpu-baseline
run c1 --config 1 --cpu-seconds 9
run c5 --config 5 --cpu-seconds 6
run c5_s1 --config 5 --streams 1 --no-cpu-baseline
run c4 --cpu-seconds 9
run c4_s1 --streams 1 --no-cpu-baseline
run c4_gen --tdec gen --cpu-seconds 6 --iterating-snr 0
run ul --ul --cpu-seconds 6 --steps 5 --iterating-snr 0
echo done
