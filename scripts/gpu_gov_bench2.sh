# governor after the in-launch fix: GPU governor tests, one bench slice at 25/50 % with 100 and 400 steps, 4 x 25 % temporal
set -o pipefail
out=gpurun_out/govbench2; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_shim_gpu.py -x -v -s --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for n in 100 400; do for l in 25 50; do
  timeout -k 10 300 python -u bench.py --slices 1 --mode shim --steps $n --child-env HIP_DEVICE_CORE_LIMIT=$l --child-env GPU_CORE_UTILIZATION_POLICY=force --out $out/s1_${l}_$n.json > $out/s1_${l}_$n.log 2>&1 || exit 1
done; done
timeout -k 10 400 python -u bench.py --slices 4 --no-spatial --policy force --mode shim --out $out/s4_board.json > $out/s4_board.log 2>&1 || exit 1
