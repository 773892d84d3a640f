# round 2: governor busy share in rocprofv3 kernel traces + the loadgen duty cycle
set -o pipefail
out=gpurun_out/r2_busy; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_loadgen_gpu.py -v -s --timeout 200 --timeout-method thread > $out/loadgen.log 2>&1 || exit 1
timeout -k 10 500 python -u scripts/probe/governor_busyshare.py > $out/busyshare.jsonl 2> $out/busyshare.err || exit 1
