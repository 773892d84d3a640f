#!/bin/bash
# Round 6: software-pipelined flash attention (MIVGPU_FA_KERNEL=9) -- numerics, microbench A/B, 8k prefill.
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
MIVGPU_FA_KERNEL=9 timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -v --timeout 300 --timeout-method thread \
  -k "prefill_flash" > $O/fa9_tests.log 2>&1 || { echo "fa9 tests failed"; grep -E "FAILED|Error" $O/fa9_tests.log | head; tail -30 $O/fa9_tests.log; exit 1; }
grep -E "passed|failed" $O/fa9_tests.log | tail -1
for kern in 8 9; do for p in 0 1; do
  MIVGPU_FA_KERNEL=$kern MIVGPU_FA_PRIO=$p timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.prefill_attention --lens 2048,8192 --reps 30 --eager-max 0 > $O/fa_k${kern}_p$p.json 2>&1 || exit 1
  echo "k$kern p$p $(grep -o '"L": [0-9]*\|"flash_ms": [0-9.]*\|"flash_tflops": [0-9.]*' $O/fa_k${kern}_p$p.json | tr '\n' ' ')"
done; done
for kern in 8 9; do
  MIVGPU_FA_KERNEL=$kern timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 8448 --iters 10 > $O/pf8k_k$kern.json 2>$O/pf8k_k$kern.err || exit 1
  echo "k$kern $(cat $O/pf8k_k$kern.json)"
done
