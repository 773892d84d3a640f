# round 2: occupancy-weighted governor checks (governor GPU tests + default bench with the temporal round)
set -o pipefail
out=gpurun_out/r2_gov; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_shim_gpu.py -v -s --timeout 300 --timeout-method thread -k "governor or temporal or masked or heavy or launch" > $out/shim_tests.log 2>&1
rc=$?
timeout -k 10 400 python -u bench.py --out $out/bench.json > $out/bench.log 2>&1 || exit 1
exit $rc
