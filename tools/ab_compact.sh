#!/bin/bash
# same-box A/B of the waterfall compaction (MI_TDEC_COMPACT=0 disables it): ./tools/ab_compact.sh <tag> [bench args...]
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for i in 1 2; do
  for c in 1 0; do
    MI_TDEC_COMPACT=$c timeout -k 10 240 python3 bench.py --no-cpu-baseline "$@" > $OUT/c${c}_$i.json 2> $OUT/c$c.err || exit 20
  done
done
echo done
