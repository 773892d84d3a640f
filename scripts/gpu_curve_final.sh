# final slice curve 1/2/4/8 (all rounds) + kernel trace of one 64-CU slice decode step
set -o pipefail
out=gpurun_out/curve_final; mkdir -p $out
for n in 1 2 4 8; do
  timeout -k 10 400 python -u bench.py --slices $n --out $out/s$n.json > $out/s$n.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
HSA_CU_MASK=0:0-63 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$out/prof_cu64 -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 > $R/$out/prof_cu64.log 2>&1 || exit 1
