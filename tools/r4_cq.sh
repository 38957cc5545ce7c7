#!/bin/bash
# waterfall continuation with a 2-waves-per-SIMD register budget and q-row loads 2 (cq2) or 3 (cq3) windows ahead,
# vs the current build: one stream, then four; then the round-3 build vs the current one
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
./tools/ab_serial.sh $1/s1 "cq2 cq3" || exit 11
./tools/ab_round.sh $1/s4 "cq2 cq3" --plan-steps 0 || exit 12
for f in gpurun_out/$1/s4/*.json; do python3 tools/bj.py $f; done
# the round-3 final build (ab_r3/, not committed; its bench has no planning block) vs the current one, default bench
mkdir -p gpurun_out/$1/h
for i in 1 2; do
  (cd ab_r3 && timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 100) > gpurun_out/$1/h/r3_$i.json 2> gpurun_out/$1/h/r3.err || exit 13
  echo -n "r3: "; python3 tools/bj.py gpurun_out/$1/h/r3_$i.json
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 100 --plan-steps 0 > gpurun_out/$1/h/cur_$i.json 2> gpurun_out/$1/h/cur.err || exit 14
  echo -n "cur: "; python3 tools/bj.py gpurun_out/$1/h/cur_$i.json
done
