#!/bin/bash
# Low-occupancy configs: streams and turbo form sweep (through gpurun): ./tools/lowocc_sweep.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
run() { name=$1; shift; timeout -k 10 240 python3 bench.py --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 20; echo -n "$name: "; python3 tools/bj.py $OUT/$name.json; }
run c3_s4 --config 3 --streams 4
run c3_s8 --config 3 --streams 8
MI_TDEC_X=3 run c3_s4_p2 --config 3 --streams 4
MI_TDEC_X=3 run c3_s8_p2 --config 3 --streams 8
run c5_s4 --config 5 --streams 4
run c5_s8 --config 5 --streams 8
run c1_s3 --config 1 --streams 3
run c1_s6 --config 1 --streams 6
echo done
