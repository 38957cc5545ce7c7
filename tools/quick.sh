#!/bin/bash
# quick GPU check of a decoder change: ./tools/quick.sh <tag> [pytest files...]; bench line summary in <tag>/bench.json
set -o pipefail
T=$1; shift
mkdir -p gpurun_out/$T
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/t.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/$T/t.log; exit 1; }
  tail -1 gpurun_out/$T/t.log
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/$T/bench.err; exit 2; }
python - "$T" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/{sys.argv[1]}/bench.json").read().strip().splitlines()[-1])
it = d.get("iterating", {})
print("value", d["value"], "ms", d["ms_per_step"], "stages", d.get("stage_ms_per_step"), "frac", d["roofline"]["frac"])
print("iterating", it.get("Mbps"), it.get("stage_ms_per_step"))
PY
