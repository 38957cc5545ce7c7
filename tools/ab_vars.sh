#!/bin/bash
# same-box A/B of the current build against variant libraries srsue_amd/libsrsue_amd_<v>.so (make variant):
#   ./tools/ab_vars.sh <tag> "<v1> <v2> ..." [bench args...]   -- two headline rounds + one configs[0] run each
set -o pipefail
OUT=gpurun_out/$1; VS="cur $2"; shift 2
mkdir -p $OUT
for i in 1 2; do
  for v in $VS; do
    if [ $v = cur ]; then L=; else L=srsue_amd/libsrsue_amd_$v.so; fi
    SRSUE_AMD_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --iterating-snr 0 "$@" > $OUT/hd_${v}_$i.json 2> $OUT/hd_$v.err || exit 20
  done
done
for v in $VS; do
  if [ $v = cur ]; then L=; else L=srsue_amd/libsrsue_amd_$v.so; fi
  SRSUE_AMD_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --config 1 --iterating-snr 0 > $OUT/c0_$v.json 2> $OUT/c0_$v.err || exit 21
done
echo done
