#!/bin/bash
# Interleaved A/B of library builds on one box (no test suite): ./tools/ab_libs.sh <tag> <reps> <lib-suffix...> [-- bench args]
#   each suffix v selects srsue_amd/libsrsue_amd_<v>.so ("cur" = srsue_amd/libsrsue_amd.so); every rep runs each build
#   once with bench.py --no-cpu-baseline and the given args, in the listed order
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
REPS=$2
shift 2
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p $OUT
cd $R
for i in $(seq 1 $REPS); do
  for v in "${LIBS[@]}"; do
    if [ "$v" == "cur" ]; then lib=srsue_amd/libsrsue_amd.so; else lib=srsue_amd/libsrsue_amd_$v.so; fi
    SRSUE_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $OUT/${v}_$i.json 2> $OUT/$v.err || exit 21
    echo -n "$v: "; python3 tools/bj.py $OUT/${v}_$i.json
  done
done
echo done
