#!/bin/bash
# The whole GPU suite with a heartbeat (one line a minute, and who holds the
# GPU) and the benches' slice logs under gpurun_out.
set -o pipefail
O=${O:-gpurun_out/r6m}
mkdir -p $O
export MIVGPU_TEST_BENCH_LOGS=$PWD/$O/benchlogs
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do
  sleep 60
  echo "$(date +%T) $(grep -c PASSED $O/gpu_tests.log) passed, last: $(grep -o 'tests/[a-z_0-9]*\.py::[A-Za-z_0-9]*' $O/gpu_tests.log | tail -1)"
  (rocm-smi --showpids 2>/dev/null | grep -E "^[0-9]+ " | head -20) >> $O/gpu_pids.log
done
wait $pid
rc=$?
echo "suite rc=$rc"
grep -E "^(FAILED|ERROR)" $O/gpu_tests.log | head -20
tail -1 $O/gpu_tests.log
exit $rc
