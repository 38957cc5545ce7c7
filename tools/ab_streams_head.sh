#!/bin/bash
# Same-box A/B of --streams at the default bench (headline + waterfall block), interleaved twice:
#   ./tools/ab_streams_head.sh <tag> 1 2 3 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
for rep in 1 2; do
  for s in "$@"; do
    timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --streams $s ${BENCH_ARGS:-} > $OUT/s${s}_r$rep.json 2> $OUT/s${s}_r$rep.err || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); s=d['stage_ms_per_step']; it=d.get('iterating',{}); r=d['roofline']
print('streams %s r%s  %9.1f Mbps ms/step %.3f tdec %.3f (iso %s) | waterfall %s Mbps ms/step %s' % (sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], s['tdec'], r['avg_launch_ms'], it.get('Mbps'), it.get('ms_per_step')))" $OUT/s${s}_r$rep.json $s $rep
  done
done
