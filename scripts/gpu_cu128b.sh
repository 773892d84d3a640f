# 128-CU slices: wide-kernel plan sweep, qkv plan A/B on the decode step, 2-slice bench
set -o pipefail
out=gpurun_out/cu128b; mkdir -p $out
HSA_CU_MASK=0:0-127 timeout -k 10 500 python -u -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --shapes gate_up,down,lm_head --sweep --out $out/sweep_cu128.json > $out/sweep_cu128.log 2>&1 || exit 1
for q in 160 0; do
  HSA_CU_MASK=0:0-127 MIVGPU_QKV_WIDE_CUS=$q timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 30 > $out/decode_cu128_q$q.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --slices 2 --mode shim --out $out/s2_shim.json > $out/s2_shim.log 2>&1 || exit 1
