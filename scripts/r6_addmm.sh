#!/bin/bash
# Round 6: prefill residual add inside the library GEMM (beta = 1) -- numerics + 8k A/B.
set -o pipefail
O=gpurun_out/r6am
mkdir -p $O
[ -n "$SKIP_TESTS" ] || MIVGPU_PREFILL_ADDMM=1 timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -v --timeout 200 --timeout-method thread \
  -k "prefill_matches or long_prefill or packed_only_long" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
[ -n "$SKIP_TESTS" ] || grep -E "passed|failed" $O/tests.log | tail -1
pf() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 8448 --iters 20 > $O/pf_$tag.json 2>$O/pf_$tag.err || { echo "$tag failed"; tail -5 $O/pf_$tag.err; exit 1; }
  echo "$tag $(tail -1 $O/pf_$tag.json)"
}
for rep in 1 2 3 4 5; do
  pf a0_$rep MIVGPU_PREFILL_ADDMM=0
  pf a1_$rep MIVGPU_PREFILL_ADDMM=1
done
