# 8 x 32-CU shared read ceiling vs blocks per CU (20 GiB working set each)
set -o pipefail
out=gpurun_out/membw8; mkdir -p $out
for b in 2 4 8 16; do
  timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.membw --gib 20 --shared-only 8 --shared-bpc $b --out $out/membw8_b$b.json > $out/membw8_b$b.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.membw --gib 20 --shared-only 4 --shared-bpc 4 --out $out/membw4_b4.json > $out/membw4_b4.log 2>&1 || exit 1
