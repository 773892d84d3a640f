#!/bin/bash
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
for n in a b; do
timeout -k 10 400 python -u bench.py --slices 8 --rounds shim,native --steps 20 --warmup 5 --child-env MIVGPU_GATE_TRACE=1 --out $O/s8_$n.json > $O/s8_$n.log 2>&1 || exit 1
python - <<PY
import json
d=json.load(open("$O/s8_$n.json"))
print("s8_$n", d["value"], d["native_value"], d["slice_fairness_min_over_max"])
for g in d["governor_rank0"]:
    print(g["held_ms"], g["at_go"], g["at_end"], g["hold_trace"], g["fair_samples"], g["board_fair_passes"], g["board_passes"])
PY
done
