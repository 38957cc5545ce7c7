#!/bin/bash
# SQ counters of the turbo kernel (VALU / memory issue, wave cycles), one rocprofv3 --pmc pass per
# counter group, no tracing domains combined with --pmc:  ./tools/pmc_tdec.sh <tag> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --iterating-snr 0 "$@" > $OUT/pmc$i.log 2>&1 || exit 1$i
done
echo done
