#!/bin/bash
# Round 6: no bucket debt while ungoverned -- governor tests, then eight pooled slices at 100 / 20 steps.
set -o pipefail
O=gpurun_out/r6ng
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_a8_tenants_gpu.py tests/test_shim_gpu.py -v --timeout 300 --timeout-method thread \
  -k "eight or temporal or unequal or masked or symmetric or held or share" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
run() {
  local n=$1; shift
  MIVGPU_GATE_TRACE=1 timeout -k 10 400 python -u bench.py "$@" --out $O/$n.json > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d.get('native_value'),d.get('slice_fairness_min_over_max'),[g.get('held_ms') for g in d.get('governor_rank0',[])])"
}
run s8_100a --slices 8 --rounds shim,native --steps 100 --warmup 5
run s8_100b --slices 8 --rounds shim,native --steps 100 --warmup 5
run s8_20 --slices 8 --rounds shim,native --steps 20 --warmup 5
