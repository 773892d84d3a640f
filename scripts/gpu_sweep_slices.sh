# wide-kernel plan sweeps in the 64-CU (4-slice) and 32-CU (8-slice) partitions
set -o pipefail
out=gpurun_out/sweeps; mkdir -p $out
for m in 0:0-63 0:0-31; do
  tag=$(echo $m | tr -d ':-')
  HSA_CU_MASK=$m timeout -k 10 550 python -u -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --sweep --out $out/sweep_$tag.json > $out/sweep_$tag.log 2>&1 || exit 1
done
