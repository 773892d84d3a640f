# 32-CU slice (the 8-slice partition): decode step, kernel profile, GEMM plans vs hipBLASLt
set -o pipefail
out=gpurun_out/cu32; mkdir -p $out
R=$GRAFT_REPO_ROOT
HSA_CU_MASK=0:0-31 timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 30 > $out/decode_cu32.log 2>&1 || exit 1
HSA_CU_MASK=0:0-31 timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --out $out/gemm_cu32.json > $out/gemm_cu32.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
HSA_CU_MASK=0:0-31 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$out/prof_cu32 -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 > $R/$out/prof_cu32.log 2>&1 || exit 1
