#!/bin/bash
# same-box A/B of library variants over chosen bench configurations:
#   ./tools/abv.sh <tag> "<config args>;<config args>;..." lib1 [lib2 ...]
# one JSON per (config, library) under gpurun_out/<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
CFGS=$2
shift 2
mkdir -p $OUT
IFS=';' read -ra CA <<< "$CFGS"
for i in "${!CA[@]}"; do
  for lib in "$@"; do
    SRSUE_AMD_LIB=$R/srsue_amd/$lib timeout -k 10 240 python3 $R/bench.py --no-cpu-baseline --iterating-snr 0 ${CA[$i]} > $OUT/c${i}_${lib%.so}.json 2> $OUT/c${i}_${lib%.so}.err || exit 20
  done
done
echo done
