#!/bin/bash
# Round 6: eight pooled slices on the final commit, 100 and 20 steps.
set -o pipefail
O=gpurun_out/r6s8f
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --out $O/$n.json > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d.get('native_value'),round(d['value']/d['native_value'],4),d.get('slice_fairness_min_over_max'),[g.get('held_ms') for g in d.get('governor_rank0',[])])"
}
run s8_100a --slices 8 --rounds shim,native --steps 100 --warmup 5
run s8_100b --slices 8 --rounds shim,native --steps 100 --warmup 5
run s8_20a --slices 8 --rounds shim,native --steps 20 --warmup 5
run t8_100 --slices 8 --rounds temporal,native --steps 100 --warmup 5
