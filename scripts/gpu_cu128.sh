# 128-CU slice (2 slices per GPU) and whole GPU: GEMM plans vs hipBLASLt, kernel profiles
set -o pipefail
out=gpurun_out/cu128; mkdir -p $out
R=$GRAFT_REPO_ROOT
HSA_CU_MASK=0:0-127 timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --out $out/gemm_cu128.json > $out/gemm_cu128.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && export PYTHONPATH=$R
HSA_CU_MASK=0:0-127 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$out/prof_cu128 -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 > $R/$out/prof_cu128.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$out/prof_full -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 > $R/$out/prof_full.log 2>&1 || exit 1
