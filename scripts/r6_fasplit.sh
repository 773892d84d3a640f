#!/bin/bash
# Round 6: flash attention, second half exponentials after the first half P.V (MIVGPU_FA_SPLIT=1) -- numerics, A/B, 8k prefill.
set -o pipefail
O=gpurun_out/r6fs
mkdir -p $O
MIVGPU_FA_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -v --timeout 300 --timeout-method thread \
  -k "prefill_flash" > $O/fa_d2_tests.log 2>&1 || { echo "split tests failed"; grep -E "FAILED|Error" $O/fa_d2_tests.log | head; exit 1; }
grep -E "passed|failed" $O/fa_d2_tests.log | tail -1
for rep in 1 2; do for d in 0 1; do
  MIVGPU_FA_SPLIT=$d timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.prefill_attention --lens 2048,8192 --reps 30 --eager-max 0 > $O/fa_d${d}_$rep.json 2>&1 || exit 1
  echo "d$d rep$rep $(grep -o '"L": [0-9]*\|"flash_ms": [0-9.]*\|"flash_tflops": [0-9.]*' $O/fa_d${d}_$rep.json | tr '\n' ' ')"
done; done
for d in 0 1; do
  MIVGPU_FA_SPLIT=$d timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 8448 --iters 10 > $O/pf8k_d$d.json 2>$O/pf8k_d$d.err || exit 1
  echo "d$d $(cat $O/pf8k_d$d.json)"
done
