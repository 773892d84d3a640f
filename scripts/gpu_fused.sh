# fused attention: numerics, decode step per fusion mode, 4-slice bench
set -o pipefail
out=gpurun_out/fused2; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > $out/ops_tests.log 2>&1 || exit 1
MIVGPU_ATTN_FUSED=1 timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k fused > $out/ops_tests_f1.log 2>&1 || exit 1
for f in 2 1 0; do for m in "" "0:0-63"; do
  tag=f${f}_$(echo "$m" | tr -d ':-'); [ -z "$m" ] && tag=f${f}_full
  if [ -n "$m" ]; then export HSA_CU_MASK="$m"; else unset HSA_CU_MASK; fi
  MIVGPU_ATTN_FUSED=$f timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 30 > $out/decode_$tag.log 2>&1 || exit 1
done; done
