set -o pipefail
O=gpurun_out/str
mkdir -p $O
for c in 4 3 5; do for s in 1 2 3 4; do
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --iterating-snr 0 --config $c --streams $s > $O/c${c}_s$s.json 2> $O/c${c}_s$s.err || exit 20
done; done
echo done
