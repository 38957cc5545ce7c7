#!/bin/bash
# same-box A/B of variant libraries on ONE stream (per-kernel stage times are then each kernel's own):
#   ./tools/ab_serial.sh <tag> "<v1> <v2> ..." [bench args...]      (cur = the current build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; VS="cur $2"; shift 2
mkdir -p $OUT
cd $R
for i in 1 2; do
  for v in $VS; do
    if [ $v = cur ]; then L=; else L=srsue_amd/libsrsue_amd_$v.so; fi
    SRSUE_AMD_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline --plan-steps 0 --steps 60 --streams 1 "$@" > $OUT/${v}_$i.json 2> $OUT/$v.err || exit 20
    echo -n "$v: "; python3 tools/bj.py $OUT/${v}_$i.json
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('   stages', d['stage_ms_per_step'], 'iter', (d.get('iterating') or {}).get('stage_ms_per_step'))" $OUT/${v}_$i.json
  done
done
echo done
