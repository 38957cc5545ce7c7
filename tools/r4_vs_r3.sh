#!/bin/bash
# (ab_r3/ is made with: mkdir ab_r3 && git archive 54cb33e bench.py srsue_amd oracle include profiles/traffic.json | tar -x -C ab_r3, then make in ab_r3/srsue_amd/csrc)
# same-box A/B of the round-3 final build (ab_r3/: bench.py + package of commit 54cb33e with its library, not
# committed) and the current build: configs[0] (3 streams and one stream), then the default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p $OUT
one() {   # one <version> <name> <bench args...>
  v=$1; n=$2; shift 2
  if [ $v = cur ]; then D=$R; else D=$R/ab_r3; fi
  (cd $D && timeout -k 10 240 python3 bench.py --no-cpu-baseline "$@") > $OUT/${n}_$v.json 2> $OUT/$v.err || exit 11
  echo -n "$n $v: "; python3 $R/tools/bj.py $OUT/${n}_$v.json
}
for i in 1 2; do
  for v in cur r3; do
    one $v c1_$i --config 1 || exit 11
    one $v c1s1_$i --config 1 --streams 1 || exit 12
  done
done
for i in 1 2; do
  for v in r3 cur; do
    one $v head_$i --steps 100 --plan-steps 0 || exit 13
  done
done
