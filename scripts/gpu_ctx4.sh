set -o pipefail
out=gpurun_out/ctx4; mkdir -p $out
timeout -k 10 300 python -u bench.py --mode shim --out $out/s4.json > $out/s4.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_shim_gpu.py -x -q --timeout 200 --timeout-method thread -k "context or two_processes" > $out/tests.log 2>&1 || exit 1
