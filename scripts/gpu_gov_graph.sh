# governor at 50 %: graph replays vs eager launches of the same decode step
set -o pipefail
out=gpurun_out/govgraph; mkdir -p $out
S=$GRAFT_REPO_ROOT/k8s_vgpu_scheduler_amd/lib/libmivgpu.so
for g in "" "--no-graph"; do
  tag=graph; [ -n "$g" ] && tag=eager
  timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 40 $g > $out/full_$tag.log 2>&1 || exit 1
  LD_PRELOAD=$S MIVGPU_SHARED_CACHE=/tmp/gg_$tag.cache HIP_DEVICE_CORE_LIMIT=50 GPU_CORE_UTILIZATION_POLICY=force MIVGPU_LOG_LEVEL=1 \
    timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 40 $g > $out/gov50_$tag.log 2>&1 || exit 1
done
