# 8-slice mode=all with the shim round first; per-slice logs
set -o pipefail
out=gpurun_out/s8b; mkdir -p $out
MIVGPU_BENCH_LOGS=$out/logs8 timeout -k 10 300 python -u bench.py --slices 8 --out $out/s8.json > $out/s8.log 2>&1 || exit 1
MIVGPU_BENCH_LOGS=$out/logs2 timeout -k 10 300 python -u bench.py --slices 2 --out $out/s2.json > $out/s2.log 2>&1 || exit 1
