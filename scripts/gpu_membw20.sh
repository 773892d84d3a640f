# HBM read ceiling with a decode-sized working set (20 GiB per process) at 4 and 8 partitions
set -o pipefail
out=gpurun_out/membw20; mkdir -p $out
timeout -k 10 500 python -u -m k8s_vgpu_scheduler_amd.bench.membw --gib 20 --shared-only 4,8 --out $out/membw_20g.json > $out/membw_20g.log 2>&1 || exit 1
timeout -k 10 500 python -u -m k8s_vgpu_scheduler_amd.bench.membw --gib 4 --shared-only 4,8 --out $out/membw_4g.json > $out/membw_4g.log 2>&1 || exit 1
