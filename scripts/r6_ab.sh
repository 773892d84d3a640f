#!/bin/bash
# Round 6: where the shim's ~1 % in the masked headline round comes from (A/B,
# 4 interleaved pairs each at 100 steps), and 8 pooled slices with the monitor.
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --out $O/$n.json > $O/$n.log 2>&1 || { echo "$n failed rc=$?"; tail -20 $O/$n.log; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d.get('native_value'),d.get('slice_fairness_min_over_max'),d.get('shim_overhead_pct'),(d.get('shim_overhead') or {}).get('per_pair_pct'),d.get('isolation_overhead_pct'))"
}
run ab_default --rounds shim,masked_noshim --steps 100 --warmup 5
run ab_boardoff --rounds shim,masked_noshim --steps 100 --warmup 5 --board off
run ab_noocc --rounds shim,masked_noshim --steps 100 --warmup 5 --child-env MIVGPU_OCCUPANCY=0
run ab_nomon --rounds shim,masked_noshim --steps 100 --warmup 5 --monitor 0
run s8_mon100 --slices 8 --rounds shim,native --steps 100 --warmup 5
run s8_mon20 --slices 8 --rounds shim,native --steps 20 --warmup 5
