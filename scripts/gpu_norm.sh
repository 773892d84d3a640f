# row-norm fusion: numerics, decode step fused vs unfused
set -o pipefail
out=gpurun_out/norm; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_skinny_gemm_gpu.py tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for f in 1 0; do for m in "" "0:0-63"; do
  tag=n${f}_$(echo "$m" | tr -d ':-'); [ -z "$m" ] && tag=n${f}_full
  if [ -n "$m" ]; then export HSA_CU_MASK="$m"; else unset HSA_CU_MASK; fi
  MIVGPU_NORM_FUSED=$f timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 30 > $out/decode_$tag.log 2>&1 || exit 1
done; done
