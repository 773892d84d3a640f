# shim GPU tests after the context-accounting changes
set -o pipefail
out=gpurun_out/shim; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_shim_gpu.py tests/test_e2e_gpu.py -x -v -s --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 1
