#!/bin/bash
# the driver's default bench command with the bench's 8 hardware queues, then the bench's own GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 400 python3 bench.py > $OUT/c4.json 2> $OUT/c4.err || exit 11
echo -n "default: "; python3 tools/bj.py $OUT/c4.json
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['config'])" $OUT/c4.json
timeout -k 10 400 python3 -u -m pytest tests/test_dist.py tests/test_bench_host.py tests/test_gpu_bench_config.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/gpu_bench_tests.log 2>&1 || { tail -30 $OUT/gpu_bench_tests.log; exit 12; }
tail -1 $OUT/gpu_bench_tests.log
