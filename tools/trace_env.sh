#!/bin/bash
# per-kernel average durations (rocprofv3 --kernel-trace --stats) of the current build under alternating
# environment settings, default bench without the iterating block:
#   ./tools/trace_env.sh <tag> "<NAME=VALUE|cur> ..." [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; VS="$2"; shift 2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  for v in $VS; do
    n=${v//=/_}
    if [ $v = cur ]; then E=; else E=$v; fi
    env $E true || exit 21
    ( [ -n "$E" ] && export "$E"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${n}_$i -o run -- python3 $R/bench.py --no-cpu-baseline --iterating-snr 0 "$@" > $OUT/${n}_$i.json 2> $OUT/${n}_$i.err ) || exit 20
  done
done
echo done
