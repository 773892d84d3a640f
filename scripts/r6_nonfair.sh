#!/bin/bash
# Round 6: eight pooled slices, 100 steps, with the gate trace and the non-fair sample record.
set -o pipefail
O=gpurun_out/r6nf
mkdir -p $O
for r in a b; do
MIVGPU_GATE_TRACE=1 timeout -k 10 400 python -u bench.py --slices 8 --rounds shim --steps 100 --warmup 5 --out $O/s8_$r.json > $O/s8_$r.log 2>&1 || { echo "failed"; tail -20 $O/s8_$r.log; exit 1; }
python - "$O/s8_$r.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["value"], d.get("slice_fairness_min_over_max"))
for g in d.get("governor_rank0", []):
    if g["held_ms"]:
        print("held", g["held_ms"], "trace", g.get("hold_trace"))
        for e in (g.get("nonfair") or []):
            print("   ", e)
PY
done
