#!/bin/bash
# one same-box A/B round: the current build vs variant libraries (srsue_amd/libsrsue_amd_<v>.so), each with the
# default bench (headline + iterating block), alternating: ./tools/ab_round.sh <tag> "<v1> <v2> ..." [bench args...]
set -o pipefail
OUT=gpurun_out/$1; VS="cur $2"; shift 2
mkdir -p $OUT
for i in 1 2; do
  for v in $VS; do
    if [ $v = cur ]; then L=; else L=srsue_amd/libsrsue_amd_$v.so; fi
    SRSUE_AMD_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline "$@" > $OUT/${v}_$i.json 2> $OUT/$v.err || exit 20
  done
done
echo done
