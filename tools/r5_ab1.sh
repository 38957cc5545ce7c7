#!/bin/bash
# round 5: checkpoint spacing on configs[0], writer side of an interleaved softbuffer, new GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_replan.py tests/test_gpu_golden.py -v --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log; case $rc in 0|1) ;; *) exit 1;; esac
for i in 1 2; do
  for v in cur ck16; do
    if [ $v = cur ]; then unset SRSUE_AMD_LIB; else export SRSUE_AMD_LIB=$R/srsue_amd/libsrsue_amd_$v.so; fi
    timeout -k 10 300 python3 bench.py --config 1 --no-cpu-baseline > $OUT/c1_${v}_$i.json 2> $OUT/c1_$v.err || exit 2
    echo -n "$v "; python3 tools/bj.py $OUT/c1_${v}_$i.json
  done
done
unset SRSUE_AMD_LIB
PMC_SET=traffic ./tools/pmc_ab.sh $1/pmc cur sbw || exit 3
python3 tools/pmc_summary.py $OUT/pmc rm_ tdec_kernel_p2x
