# round 2: full GPU suite + smoke, then the governor busy-share traces
set -o pipefail
out=gpurun_out/r2_full; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/probe/governor_busyshare.py > $out/busyshare.jsonl 2> $out/busyshare.err || exit 1
exit $rc
