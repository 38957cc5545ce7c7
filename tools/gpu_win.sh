set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tdec.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_win.log 2>&1
timeout -k 10 120 python bench.py --config 2 --no-cpu-baseline > gpurun_out/c2_win.json 2>/dev/null
timeout -k 10 120 python bench.py --config 2 --no-cpu-baseline --sched lane > gpurun_out/c2_lane.json 2>/dev/null
timeout -k 10 120 python bench.py --config 3 --no-cpu-baseline --sched win > gpurun_out/c3_win.json 2>/dev/null
timeout -k 10 120 python bench.py --config 1 --no-cpu-baseline --sched win --cb-per-gpu 16384 > gpurun_out/c1_win.json 2>/dev/null
timeout -k 10 120 python bench.py --no-cpu-baseline --sched win > gpurun_out/c4_win.json 2>/dev/null
