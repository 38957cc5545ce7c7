#!/bin/bash
# packed decoder checkpoint spacing A/B (same box): the current build (8-step checkpoints, row deltas in
# soffset) against libsrsue_amd_ck4.so (-DMI_TDEC_P2_CK8=0) and libsrsue_amd_base.so (also
# -DMI_ROW_CROW_SOFF=0); decoder + parity GPU tests first.   ./tools/ab_ck8.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_tdec.py tests/test_gpu_parity.py tests/test_gpu_alloc.py -x -q \
  --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 10
for i in 1 2; do
  for v in cur ck4 base; do
    if [ $v = cur ]; then L=; else L=srsue_amd/libsrsue_amd_$v.so; fi
    SRSUE_AMD_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --iterating-snr 0 > $OUT/hd_${v}_$i.json 2> $OUT/hd_$v.err || exit 20
  done
done
for v in cur ck4 base; do
  if [ $v = cur ]; then L=; else L=srsue_amd/libsrsue_amd_$v.so; fi
  SRSUE_AMD_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --config 1 --iterating-snr 0 > $OUT/c0_$v.json 2> $OUT/c0_$v.err || exit 21
done
echo done
