#!/bin/bash
# GPU measurement recipe, run through gpurun:  ./tools/profile.sh <tag>
#  1. the default bench line (python3 bench.py)
#  2. rocprofv3 --kernel-trace --stats of the SAME command (per-kernel average durations)
#  3. separate PMC passes FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md: TCC slots do not fit both),
#     and one SQ pass (VALU instructions, waves, GPU-active cycles) for the turbo kernel's VALU busy
#  4. tools/summarize_profile.py -> summary.json / summary.md (traffic per launch, agreement check)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
ARGS="--iterating-snr 0 --plan-steps 0 --h2d-steps 0 --tti-ttis 0 --steps 20 --streams 1 $@"   # one operating point per profile, every tdec launch alone on the GPU (rocprof durations = per-kernel)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || exit 11
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/prof_trace.log 2>&1 || exit 12
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS --no-cpu-baseline > $OUT/prof_fetch.log 2>&1 || exit 13
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS --no-cpu-baseline > $OUT/prof_write.log 2>&1 || exit 14
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_valu -o run -- python3 $R/bench.py $ARGS --no-cpu-baseline > $OUT/prof_valu.log 2>&1 || exit 14
python3 $R/tools/summarize_profile.py $OUT || exit 15
echo done
