#!/bin/bash
# Round 6 verification: pooled / temporal 8 slices at 20 and 100 steps, the
# driver's bench config, then the whole GPU suite.
set -o pipefail
O=${O:-gpurun_out/r6l}
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --out $O/$n.json > $O/$n.log 2>&1 || { echo "$n failed rc=$?"; tail -20 $O/$n.log; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d.get('native_value'),d.get('slice_fairness_min_over_max'),d.get('temporal_value'),d.get('temporal_fairness_min_over_max'),d.get('shim_overhead_pct'),[g.get('held_ms') for g in d.get('governor_rank0',[])])"
}
run s8_20a --slices 8 --rounds shim,native --steps 20 --warmup 5
run s8_20b --slices 8 --rounds shim,native --steps 20 --warmup 5
run s8_100 --slices 8 --rounds shim,native --steps 100 --warmup 5
run t8_20 --slices 8 --rounds temporal,native --steps 20 --warmup 5 --no-spatial --policy force
run bench_driver --gpus 1 --steps 20 --warmup 5
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "suite rc=$?"
grep -E "^(FAILED|ERROR)" $O/gpu_tests.log | head -20
tail -1 $O/gpu_tests.log
