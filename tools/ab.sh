#!/bin/bash
# Same-box A/B of library variants (make -C srsue_amd/csrc variant VNAME=.. VFLAGS=..):
#   ./tools/ab.sh <tag> <lib> [<lib> ...]      e.g. ./tools/ab.sh r1q libsrsue_amd.so libsrsue_amd_v1.so
# For each library: the default bench (int16), config 1 and config 2; one compact line per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
for lib in "$@"; do
  for cfg in "" "--config 1" "--config 2" "--tdec gen"; do
    tag=$(echo "$lib $cfg" | tr ' -' '__')
    SRSUE_AMD_LIB=$R/srsue_amd/$lib timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline $cfg > $OUT/$tag.json 2> $OUT/$tag.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stage_ms_per_step']; print('%-40s %10.1f %s  ms/step %.3f  tdec %.3f  rm %.3f' % (sys.argv[2], d['value'], d['unit'], d['ms_per_step'], s['tdec'], s['rm']))" $OUT/$tag.json "$lib $cfg"
  done
done
