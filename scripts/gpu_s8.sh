# 8-slice fairness investigation: queue counts, masks, per-slice logs
set -o pipefail
out=gpurun_out/s8; mkdir -p $out
run() { tag=$1; shift; MIVGPU_BENCH_LOGS=$out/logs_$tag timeout -k 10 200 python -u bench.py --slices 8 --mode shim --steps 60 --out $out/$tag.json "$@" > $out/$tag.log 2>&1; }
run q2 || exit 1
run q1 --hw-queues 1 || exit 1
run q2_nomask --no-spatial --policy disable || exit 1
run q2_b16 --batch 16 || exit 1
run q2_again || exit 1
