#!/bin/bash
# One GPU check of the tree (through gpurun): ./tools/gpu_round.sh <tag> [bench args...]
#   1. the full GPU suite (python -m pytest -m gpu), 2. smoke(), 3. the default bench line (+ extra args)
# Each step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 3; }
python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "tdec", d["roofline"]["avg_launch_ms"])
it = d.get("iterating", {})
print("iterating", it.get("Mbps"), it.get("tdec_roofline", {}).get("avg_launch_ms"))
print("planning", json.dumps(d.get("planning")))
print("cpu", d.get("cpu_baseline", {}).get("value"), "devices", d.get("rank_devices"))
PY
