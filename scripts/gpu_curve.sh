# slice curve 1/2/4/8 (bench.py) + kernel profiles of one decode step
set -o pipefail
out=gpurun_out/curve; mkdir -p $out
for n in 1 2 4 8; do
  timeout -k 10 300 python -u bench.py --slices $n --out $out/s$n.json > $out/s$n.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$out/prof_full -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 > $R/$out/prof_full.log 2>&1 || exit 1
HSA_CU_MASK=0:0-63 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$out/prof_cu64 -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 > $R/$out/prof_cu64.log 2>&1 || exit 1
