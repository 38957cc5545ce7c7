#!/bin/bash
# Same-box A/B of the library's creation-time environment knobs (engine.h Engine::Opts) on the bench:
#   ./tools/ab_env.sh <tag> "<ENV=..>" "<ENV=..>" ...     ("-" = no extra variable); each setting runs twice,
# interleaved (A B A B), one bench line per run (tools/bj.py).  Bench arguments: BENCH_ARGS (default: no CPU baseline,
# no waterfall block, no planning / PCIe blocks; e.g. BENCH_ARGS="--no-cpu-baseline --plan-steps 0 --h2d-steps 0"
# keeps the waterfall block).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --iterating-snr 0 --plan-steps 0 --h2d-steps 0 --tti-ttis 0"}
for rep in 1 2; do
  for e in "$@"; do
    tag=$(echo "$e r$rep" | tr ' =/.-' '_____')
    if [ "$e" = "-" ]; then envs=(); else envs=($e); fi
    env "${envs[@]}" timeout -k 10 240 python3 $R/bench.py $ARGS > $OUT/$tag.json 2> $OUT/$tag.err || exit 1
    echo -n "$e: "; python3 $R/tools/bj.py $OUT/$tag.json
  done
done
