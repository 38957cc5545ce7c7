#!/bin/bash
# Same-box A/B of library variants on the default bench only (one line per library, repeated):
#   ./tools/ab1.sh <tag> <reps> <lib> [<lib> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
REPS=$2
shift 2
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    tag=${lib}_$rep
    SRSUE_AMD_LIB=$R/srsue_amd/$lib timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline $AB_ARGS > $OUT/$tag.json 2> $OUT/$tag.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stage_ms_per_step']; print('%-28s %10.1f %s  ms/step %.3f  ' % (sys.argv[2], d['value'], d['unit'], d['ms_per_step']) + ' '.join('%s %.3f' % kv for kv in s.items()))" $OUT/$tag.json "$lib"
  done
done
