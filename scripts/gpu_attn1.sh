set -o pipefail
mkdir -p gpurun_out/attn1
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn1/ops_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m k8s_vgpu_scheduler_amd.bench.attention --variants mfma,mfma8,valu:auto --masks ",0:0-63,0:0-31" --out gpurun_out/attn1/attention.json > gpurun_out/attn1/attention.log 2>&1 || exit 1
for k in mfma valu; do for m in "" "0:0-63"; do
  tag=${k}_$(echo "$m" | tr -d ':' | tr -d '-'); [ -z "$m" ] && tag=${k}_full
  if [ -n "$m" ]; then export HSA_CU_MASK="$m"; else unset HSA_CU_MASK; fi
  MIVGPU_ATTN_KERNEL=$k timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 30 > gpurun_out/attn1/decode_$tag.log 2>&1 || exit 1
done; done
