#!/bin/bash
set -o pipefail
export O=${O:-gpurun_out/r6n}
bash scripts/r6_suite.sh; src=$?
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --out $O/$n.json > $O/$n.log 2>&1 || { echo "$n failed rc=$?"; tail -20 $O/$n.log; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d.get('native_value'),d.get('slice_fairness_min_over_max'),d.get('temporal_value'),d.get('temporal_fairness_min_over_max'),d.get('shim_overhead_pct'),[g.get('held_ms') for g in d.get('governor_rank0',[])])"
}
[ $src -eq 0 ] || [ $src -eq 1 ] || exit $src
run s8_20 --slices 8 --rounds shim,native --steps 20 --warmup 5
run s8_100 --slices 8 --rounds shim,native --steps 100 --warmup 5
run bench_driver --gpus 1 --steps 20 --warmup 5
