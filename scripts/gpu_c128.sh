# 128-CU slices: full-chip vs slice GEMM plans; 2-slice bench both ways
set -o pipefail
out=gpurun_out/c128; mkdir -p $out
for lim in 96 128; do
  HSA_CU_MASK=0:0-127 MIVGPU_SLICE_PLAN_CUS=$lim timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 30 > $out/decode_lim$lim.log 2>&1 || exit 1
done
for lim in 96 128; do
  timeout -k 10 300 python -u bench.py --slices 2 --mode shim --child-env MIVGPU_SLICE_PLAN_CUS=$lim --out $out/s2_lim$lim.json > $out/s2_lim$lim.log 2>&1 || exit 1
done
