#!/bin/bash
# round-end record on the final build: GPU suite, smoke(), the profile recipe, the default bench line (the driver's
# command) and its one-stream form
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 10; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 11; }
tail -1 $OUT/smoke.log
./tools/profile.sh $1_prof || exit 12
head -14 gpurun_out/$1_prof/summary.md
timeout -k 10 400 python3 bench.py > $OUT/c4.json 2> $OUT/c4.err || exit 13
echo -n "default: "; python3 tools/bj.py $OUT/c4.json
timeout -k 10 300 python3 bench.py --streams 1 --no-cpu-baseline --plan-steps 0 > $OUT/c4_s1.json 2> $OUT/c4_s1.err || exit 14
echo -n "one stream: "; python3 tools/bj.py $OUT/c4_s1.json
