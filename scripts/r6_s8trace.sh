#!/bin/bash
# Round 6: eight pooled slices over 100 steps with the gate trace (where the holds fall).
set -o pipefail
O=gpurun_out/r6t8
mkdir -p $O
MIVGPU_GATE_TRACE=1 timeout -k 10 400 python -u bench.py --slices 8 --rounds shim,native --steps 100 --warmup 5 --out $O/s8_100.json > $O/s8_100.log 2>&1 || { echo "failed"; tail -20 $O/s8_100.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r6t8/s8_100.json"))
print(d["value"], d.get("native_value"), d.get("slice_fairness_min_over_max"))
print(sorted(d.keys()))
for k in ("slices", "per_slice", "slice_rows"):
    if k in d:
        print(k, json.dumps(d[k])[:3000])
for g in d.get("governor_rank0", []):
    print(g["held_ms"], g.get("at_end"), g.get("hold_trace"))
PY
