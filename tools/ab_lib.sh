#!/bin/bash
# same-box A/B of the current build against another build's library (srsue_amd/libsrsue_amd_<v>.so, e.g.
# the previous commit built in a git worktree): ./tools/ab_lib.sh <tag> <v> [bench args...]
set -o pipefail
OUT=gpurun_out/$1; V=$2; shift 2
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > $OUT/cur_$i.json 2> $OUT/cur.err || exit 20
  SRSUE_AMD_LIB=srsue_amd/libsrsue_amd_$V.so timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > $OUT/${V}_$i.json 2> $OUT/$V.err || exit 21
done
echo done
