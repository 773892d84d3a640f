#!/bin/bash
# Round 6: governor tests + 8-tenant fairness A/B of the presence window.
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_shim_gpu.py -v -s --timeout 300 --timeout-method thread \
  -k "temporal or unequal or symmetric" > $O/gov_tests.log 2>&1 || echo "gov tests rc=$?"
grep -E "passed|failed" $O/gov_tests.log | tail -1
timeout -k 10 300 python -u bench.py --slices 8 --rounds temporal,native --steps 100 --warmup 5 \
  --presence-window-us 0 --out $O/t8_w0.json > $O/t8_w0.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --slices 8 --rounds temporal,native --steps 100 --warmup 5 \
  --out $O/t8_w20.json > $O/t8_w20.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --slices 8 --rounds shim,native --steps 100 --warmup 5 \
  --out $O/s8_mon.json > $O/s8_mon.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/bench_driver.json > $O/bench_driver.log 2>&1 || exit 1
python - <<'PY'
import json
O="gpurun_out/r6c"
for n in ("t8_w0","t8_w20","s8_mon","bench_driver"):
    d=json.load(open(f"{O}/{n}.json"))
    keys=("value","native_value","temporal_value","temporal_fairness_min_over_max","slice_fairness_min_over_max",
          "shim_overhead_pct","isolation_overhead_pct","temporal_overhead_pct")
    print(n, {k:d.get(k) for k in keys if k in d})
PY
