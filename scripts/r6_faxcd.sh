#!/bin/bash
# Round 6: flash attention with kv head = block mod 8 (each XCD's L2 one head's K/V) -- numerics, A/B, 8k prefill.
set -o pipefail
O=gpurun_out/r6fx
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -v --timeout 300 --timeout-method thread \
  -k "prefill_flash or prefill_matches or long_prefill" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for rep in 1 2; do for d in 0 1; do
  MIVGPU_FA_XCD=$d timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.prefill_attention --lens 2048,8192 --reps 30 --eager-max 0 > $O/fa_x${d}_$rep.json 2>&1 || exit 1
  echo "x$d rep$rep $(grep -o '"L": [0-9]*\|"flash_ms": [0-9.]*\|"flash_tflops": [0-9.]*' $O/fa_x${d}_$rep.json | tr '\n' ' ')"
done; done
for rep in 1 2 3; do for d in 0 1; do
  MIVGPU_FA_XCD=$d timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 8448 --iters 20 > $O/pf8k_x${d}_$rep.json 2>$O/pf8k_x${d}_$rep.err || exit 1
  echo "x$d rep$rep $(python -c "import json;print(json.loads(open('$O/pf8k_x${d}_$rep.json').read().strip().splitlines()[-1])['ms_per_prefill'])")"
done; done
