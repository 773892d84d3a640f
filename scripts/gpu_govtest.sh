set -o pipefail
out=gpurun_out/govtest; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_shim_gpu.py -x -v -s --timeout 300 --timeout-method thread -k "governor" > $out/tests.log 2>&1 || exit 1
