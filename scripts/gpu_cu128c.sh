# mid-partition (128-CU) wide plans: numerics, decode step A/B, 2-slice bench
set -o pipefail
out=gpurun_out/cu128c; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_skinny_gemm_gpu.py -x -v --timeout 200 --timeout-method thread -k "half_gpu" > $out/tests.log 2>&1 || exit 1
for m in 1 0 1 0; do
  HSA_CU_MASK=0:0-127 MIVGPU_WIDE_MID_PLAN=$m timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 50 >> $out/decode_cu128_mid$m.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --slices 2 --mode shim --out $out/s2_shim.json > $out/s2_shim.log 2>&1 || exit 1
