#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r37
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step env MIVGPU_SKINNY_KMAJOR=1 timeout -k 10 600 python -m pytest tests/test_skinny_gemm_gpu.py -q -x > gpurun_out/r37/pytest_km1.log 2>&1
step env MIVGPU_SKINNY_KMAJOR=1 MIVGPU_SKINNY_DB=1 HSA_CU_MASK=0:0-63 timeout -k 10 600 python -m pytest tests/test_skinny_gemm_gpu.py -q -x > gpurun_out/r37/pytest_km1_db1_cu64.log 2>&1
for km in 1; do for db in 0 1; do
step env HSA_CU_MASK=0:0-63 GPU_MAX_HW_QUEUES=2 MIVGPU_SKINNY_DB=$db MIVGPU_SKINNY_KMAJOR=$km timeout -k 10 900 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --sweep --out gpurun_out/r37/gemm_cu64_km${km}_db${db}.json > gpurun_out/r37/gemm_cu64_km${km}_db${db}.log 2>&1
done; done
for km in 0 1; do
step env MIVGPU_SKINNY_KMAJOR=$km timeout -k 10 900 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --sweep --out gpurun_out/r37/gemm_full_km${km}.json > gpurun_out/r37/gemm_full_km${km}.log 2>&1
done
