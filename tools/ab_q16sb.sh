#!/bin/bash
# timing diagnostic: one-iteration decode with fp32 vs int16-wide softbuffer reads (results wrong in the variant)
set -o pipefail
OUT=gpurun_out/ab_q16sb; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 --max-its 1 > $OUT/base_$i.json 2> $OUT/base.err || exit 20
  SRSUE_AMD_LIB=srsue_amd/libsrsue_amd_q16sb.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 --max-its 1 > $OUT/q16sb_$i.json 2> $OUT/q16sb.err || exit 21
done
echo done
