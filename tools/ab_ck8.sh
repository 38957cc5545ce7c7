set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tdec.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ck8.log 2>&1
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ck8_$i.json 2>/dev/null
SRSUE_AMD_LIB=srsue_amd/libsrsue_amd_ck4.so timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ck4_$i.json 2>/dev/null
done
timeout -k 10 200 python bench.py --config 1 --no-cpu-baseline > gpurun_out/ck8_c1.json 2>/dev/null
SRSUE_AMD_LIB=srsue_amd/libsrsue_amd_ck4.so timeout -k 10 200 python bench.py --config 1 --no-cpu-baseline > gpurun_out/ck4_c1.json 2>/dev/null
