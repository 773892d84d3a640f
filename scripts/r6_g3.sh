#!/bin/bash
# Round 6: pooled 8 slices after the bucket start credit; governor + e2e tests; FA priority A/B.
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --out $O/$n.json > $O/$n.log 2>&1 || { echo "$n failed rc=$?"; tail -20 $O/$n.log; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d.get('native_value'),d.get('slice_fairness_min_over_max'),d.get('temporal_value'),d.get('temporal_fairness_min_over_max'),d.get('shim_overhead_pct'),[g.get('held_ms') for g in d.get('governor_rank0',[])])"
}
run s8_mon20a --slices 8 --rounds shim,native --steps 20 --warmup 5
run s8_mon20b --slices 8 --rounds shim,native --steps 20 --warmup 5
run s8_mon100 --slices 8 --rounds shim,native --steps 100 --warmup 5
timeout -k 10 900 python -u -m pytest tests/test_shim_gpu.py tests/test_e2e_gpu.py -v -s --timeout 300 --timeout-method thread \
  > $O/gov_tests.log 2>&1 || echo "tests rc=$?"
grep -E "passed|failed" $O/gov_tests.log | tail -3
grep -E "FAILED" $O/gov_tests.log | head
for p in 0 1; do
  MIVGPU_FA_PRIO=$p timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.prefill_attention --lens 2048,8192 --reps 30 --eager-max 0 > $O/fa_prio$p.json 2>&1 || exit 1
  cat $O/fa_prio$p.json
done
