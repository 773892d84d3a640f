# governor at 50 %, one bench slice: 100 vs 400 timed steps
set -o pipefail
out=gpurun_out/govbench; mkdir -p $out
for n in 100 400; do
  timeout -k 10 300 python -u bench.py --slices 1 --mode shim --steps $n --child-env HIP_DEVICE_CORE_LIMIT=50 --child-env GPU_CORE_UTILIZATION_POLICY=force --child-env MIVGPU_LOG_LEVEL=3 --out $out/s1_50_$n.json > $out/s1_50_$n.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --slices 1 --mode shim --steps 100 --out $out/s1_full.json > $out/s1_full.log 2>&1 || exit 1
