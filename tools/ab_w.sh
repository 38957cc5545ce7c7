set -o pipefail
OUT=gpurun_out/ab_w; mkdir -p $OUT
run() { name=$1; shift; timeout -k 10 240 python3 bench.py "$@" --no-cpu-baseline > $OUT/$name.json 2> $OUT/$name.err || exit 20; }
run c3_auto --config 3
run c3_win --config 3 --sched win
run c1_auto --config 1
run c1_win --config 1 --sched win
run c5_auto --config 5
run c5_lane --config 5 --sched lane
echo done
