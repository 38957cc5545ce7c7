#!/bin/bash
# same-box A/B of the packed int16 decoder (two code blocks per lane) against the default crossed schedule:
#   ./tools/ab_p2.sh <tag> [configs...]   (config names below; default: all)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd $R
run() { name=$1; shift; timeout -k 10 240 python3 bench.py --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 20; }
SEL=${@:-hd c1 c3 c5}
for c in $SEL; do
  case $c in
    hd) run hd_def; run hd_p2 --sched p2 ;;
    c1) run c1_def --config 1; run c1_p2 --config 1 --sched p2 ;;
    c3) run c3_def --config 3 --iterating-snr 0; run c3_p2 --config 3 --sched p2 --iterating-snr 0 ;;
    c5) run c5_def --config 5 --iterating-snr 0; run c5_p2 --config 5 --sched p2 --iterating-snr 0 ;;
  esac
done
echo done
