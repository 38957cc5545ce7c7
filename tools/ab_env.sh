#!/bin/bash
# Same-box A/B of environment knobs on the default bench (no CPU baseline, no waterfall block):
#   ./tools/ab_env.sh <tag> "<ENV=..>" "<ENV=..>" ...     ("-" = no extra variable); each setting runs twice,
# interleaved (A B A B), one compact line per run.  Extra bench arguments: BENCH_ARGS.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
for rep in 1 2; do
  for e in "$@"; do
    tag=$(echo "$e r$rep" | tr ' =/.-' '_____')
    if [ "$e" = "-" ]; then envs=(); else envs=($e); fi
    env "${envs[@]}" timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --iterating-snr 0 ${BENCH_ARGS:-} \
      > $OUT/$tag.json 2> $OUT/$tag.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stage_ms_per_step']; print('%-34s %10.1f %s  ms/step %.3f  tdec %.3f  rm %.3f' % (sys.argv[2], d['value'], d['unit'], d['ms_per_step'], s['tdec'], s['rm']))" $OUT/$tag.json "$e r$rep"
  done
done
