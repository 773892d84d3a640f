# round check: full GPU suite, smoke, default bench
set -o pipefail
out=gpurun_out/full; mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --out $out/bench.json > $out/bench.log 2>&1 || exit 1
