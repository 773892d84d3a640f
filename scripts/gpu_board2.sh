# governor: gate per graph launch; duty cycle on decode alone at 25/50/75 %, board A/B test
set -o pipefail
out=gpurun_out/board2; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_shim_gpu.py -x -v -s --timeout 300 --timeout-method thread -k "governor" > $out/tests.log 2>&1 || exit 1
for l in 25 50 75; do
  timeout -k 10 300 python -u bench.py --slices 1 --mode shim --child-env HIP_DEVICE_CORE_LIMIT=$l --child-env GPU_CORE_UTILIZATION_POLICY=force --out $out/s1_$l.json > $out/s1_$l.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --slices 1 --mode shim --out $out/s1_100.json > $out/s1_100.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --slices 4 --no-spatial --policy force --mode shim --out $out/s4_board.json > $out/s4_board.log 2>&1 || exit 1
