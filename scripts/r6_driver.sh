#!/bin/bash
# Round 6: what the driver runs at round end -- smoke(), pytest -x -q -m gpu, bench.py -- on one fresh box.
set -o pipefail
O=${O:-gpurun_out/r6drv}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1100 python -u -m pytest tests/ -x -q -m gpu > $O/gpu_tests.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 60; echo "$(date +%T) $(tail -c 120 $O/gpu_tests.log | tr '\n' ' ')"; done
wait $pid; rc=$?
echo "pytest rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-400
