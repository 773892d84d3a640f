# kernel traces: row-norm fusion on/off, whole GPU
set -o pipefail
out=gpurun_out/normprof; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
  MIVGPU_NORM_FUSED=$f timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/n$f -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 > $GRAFT_REPO_ROOT/$out/n$f.log 2>&1 || exit 1
done
