# decode-attention A/B: numerics, microbench over partitions, decode step
set -o pipefail
mkdir -p gpurun_out/attn2
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn2/ops_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u -m k8s_vgpu_scheduler_amd.bench.attention --variants mfma,mfma:nt,mfma8,mfma8:nt,valu:auto --masks ",0:0-63,0:0-31" --out gpurun_out/attn2/attention.json > gpurun_out/attn2/attention.log 2>&1 || exit 1
for m in "" "0:0-63"; do
  tag=$(echo "$m" | tr -d ':-'); [ -z "$m" ] && tag=full
  if [ -n "$m" ]; then export HSA_CU_MASK="$m"; else unset HSA_CU_MASK; fi
  timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 30 > gpurun_out/attn2/decode_mfma_$tag.log 2>&1 || exit 1
done
