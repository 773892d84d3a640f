#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r36
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step env MIVGPU_SKINNY_DB=1 timeout -k 10 600 python -m pytest tests/test_skinny_gemm_gpu.py -q -x > gpurun_out/r36/pytest_db1.log 2>&1
step env MIVGPU_SKINNY_DB=1 HSA_CU_MASK=0:0-63 timeout -k 10 600 python -m pytest tests/test_skinny_gemm_gpu.py -q -x > gpurun_out/r36/pytest_db1_cu64.log 2>&1
step env HSA_CU_MASK=0:0-63 GPU_MAX_HW_QUEUES=2 MIVGPU_SKINNY_DB=0 timeout -k 10 900 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --sweep --out gpurun_out/r36/gemm_cu64_db0.json > gpurun_out/r36/gemm_db0.log 2>&1
step env HSA_CU_MASK=0:0-63 GPU_MAX_HW_QUEUES=2 MIVGPU_SKINNY_DB=1 timeout -k 10 900 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --sweep --out gpurun_out/r36/gemm_cu64_db1.json > gpurun_out/r36/gemm_db1.log 2>&1
