set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tdec.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x.log 2>&1 || { tail -30 gpurun_out/t_x.log; exit 1; }
tail -3 gpurun_out/t_x.log
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --sched lane > gpurun_out/b_lane.json 2> gpurun_out/b_lane.err
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --sched lanex > gpurun_out/b_lanex.json 2> gpurun_out/b_lanex.err
for f in gpurun_out/b_lane.json gpurun_out/b_lanex.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('stage_ms'))"; done
