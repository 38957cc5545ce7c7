#!/bin/bash
# Counter A/B of library builds at the headline, one stream (every launch alone on the GPU):
#   ./tools/pmc_ab.sh <tag> <v> [<v> ...]     v = cur (srsue_amd/libsrsue_amd.so) or a variant suffix
#                                              (srsue_amd/libsrsue_amd_<v>.so, make -C srsue_amd/csrc variant VNAME=<v>)
# Per build, each in a rocprofv3 run of its own: a kernel trace (--kernel-trace --stats), FETCH_SIZE, WRITE_SIZE and
# three SQ counter groups (no tracing domain beside --pmc); PMC_SET=traffic: the trace and the two traffic passes only;
# PMC_GROUPS: the trace and the given groups.
# Extra bench arguments: BENCH_ARGS.  Summary: python3 tools/pmc_summary.py gpurun_out/<tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
ARGS="--no-cpu-baseline --steps 3 --warmup 1 --iterating-snr 0 --plan-steps 0 --h2d-steps 0 --tti-ttis 0 --streams 1 ${BENCH_ARGS:-}"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = cur ]; then unset SRSUE_AMD_LIB; else export SRSUE_AMD_LIB=$R/srsue_amd/libsrsue_amd_$v.so; fi
  D=$OUT/$v
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/bench.py $ARGS > $D/trace.log 2>&1 || exit 10
  i=0
  PASSES=("FETCH_SIZE" "WRITE_SIZE")
  # PMC_GROUPS="A B;C D": these counter groups instead, one pass each (<= 8 SQ / 4 TCC counters per pass)
  if [ -n "${PMC_GROUPS:-}" ]; then IFS=';' read -ra PASSES <<< "$PMC_GROUPS"; PMC_SET=custom; fi
  [ "${PMC_SET:-all}" = traffic ] || [ "${PMC_SET:-all}" = custom ] || PASSES+=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU" \
             "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
             "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE")
  for grp in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $D/pmc$i -o run -- python3 $R/bench.py $ARGS > $D/pmc$i.log 2>&1 || exit 1$i
  done
  echo "$v done"
done
