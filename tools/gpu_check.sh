#!/bin/bash
# One GPU check of the tree without stopping at the first failing test: ./tools/gpu_check.sh <tag> [variant ...]
#   1. the full GPU suite (every failure listed), 2. smoke(), 3. the default bench line,
#   4. for each variant library srsue_amd/libsrsue_amd_<v>.so: the default bench without CPU baseline, A/B interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log; grep -E "^(FAILED|ERROR)" $OUT/gpu_tests.log
# a timeout / abort / segfault ends the call here (no further GPU work after a fault)
case $rc in 0|1) ;; *) echo "TESTS rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 3; }
python3 tools/bj.py $OUT/bench.json; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps(d.get(\"planning\")))" $OUT/bench.json
for v in "$@"; do
  for i in 1 2; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/cur_$i.json 2> $OUT/cur.err || exit 20
    python3 tools/bj.py $OUT/cur_$i.json
    SRSUE_AMD_LIB=srsue_amd/libsrsue_amd_$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/${v}_$i.json 2> $OUT/$v.err || exit 21
    echo -n "$v: "; python3 tools/bj.py $OUT/${v}_$i.json
  done
done
echo done
