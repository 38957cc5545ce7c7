#!/bin/bash
# instruction / scalar-cache counters of the turbo kernel: ./tools/pmc_ic.sh <tag> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH" "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/ic$i -o run -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --iterating-snr 0 "$@" > $OUT/ic$i.log 2>&1 || exit 1$i
done
echo done
