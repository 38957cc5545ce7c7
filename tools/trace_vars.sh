#!/bin/bash
# per-kernel average durations (rocprofv3 --kernel-trace --stats) of the current build and variant libraries,
# alternating, default bench without the iterating block:  ./tools/trace_vars.sh <tag> "<v1> ..." [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; VS="cur $2"; shift 2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  for v in $VS; do
    if [ $v = cur ]; then L=; else L=$R/srsue_amd/libsrsue_amd_$v.so; fi
    SRSUE_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${v}_$i -o run -- python3 $R/bench.py --no-cpu-baseline --iterating-snr 0 "$@" > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err || exit 20
  done
done
echo done
