#!/bin/bash
# same-box A/B of bench argument sets (same build): ./tools/ab_args.sh <tag> "<args A>" "<args B>" ... -- two rounds each
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for i in 1 2; do
  j=0
  for a in "$@"; do
    j=$((j+1))
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --iterating-snr 0 $a > $OUT/v${j}_$i.json 2> $OUT/v$j.err || exit 20
  done
done
echo done
