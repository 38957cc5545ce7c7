#!/bin/bash
# Same-box A/B of (--streams, --iterating-streams) pairs at the default bench, interleaved twice:
#   ./tools/ab_streams2.sh <tag> 3:2 4:3 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
for rep in 1 2; do
  for p in "$@"; do
    s=${p%%:*}; i=${p##*:}
    timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --streams $s --iterating-streams $i ${BENCH_ARGS:-} \
      > $OUT/s${s}_i${i}_r$rep.json 2> $OUT/s${s}_i${i}_r$rep.err || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); s=d['stage_ms_per_step']; it=d.get('iterating',{}); r=d['roofline']
print('streams %s r%s  %9.1f Mbps ms/step %.3f tdec iso %s | waterfall %s Mbps ms/step %s iso %s' % (sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], r['avg_launch_ms'], it.get('Mbps'), it.get('ms_per_step'), it.get('tdec_roofline',{}).get('avg_launch_ms')))" $OUT/s${s}_i${i}_r$rep.json $p $rep
  done
done
