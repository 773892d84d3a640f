# sustained 4-slice headline: 1000 timed steps per slice (~14 s)
set -o pipefail
out=gpurun_out/sustained; mkdir -p $out
timeout -k 10 500 python -u bench.py --mode shim --steps 1000 --warmup 20 --out $out/s4_1000.json > $out/s4_1000.log 2>&1 || exit 1
