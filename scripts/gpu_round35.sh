#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r40
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 900 python -m pytest tests/test_skinny_gemm_gpu.py tests/test_ops_gpu.py -q -x > gpurun_out/r40/pytest.log 2>&1
step env HSA_CU_MASK=0:0-63 timeout -k 10 900 python -m pytest tests/test_skinny_gemm_gpu.py tests/test_ops_gpu.py -q -x -k "skinny or decoder or Decoder or wide" > gpurun_out/r40/pytest_cu64.log 2>&1
step env HSA_CU_MASK=0:0-63 GPU_MAX_HW_QUEUES=2 timeout -k 10 900 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --out gpurun_out/r40/gemm_cu64.json > gpurun_out/r40/gemm_cu64.log 2>&1
step timeout -k 10 900 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 1,8,32,64,128 --out gpurun_out/r40/gemm_full.json > gpurun_out/r40/gemm_full.log 2>&1
step env HSA_CU_MASK=0:0-63 GPU_MAX_HW_QUEUES=2 timeout -k 10 600 python -m k8s_vgpu_scheduler_amd.bench.decode --batch 32 --steps 30 > gpurun_out/r40/decode_cu64.log 2>&1
step timeout -k 10 600 python -m k8s_vgpu_scheduler_amd.bench.decode --batch 32 --steps 30 > gpurun_out/r40/decode_full.log 2>&1
step timeout -k 10 1200 python bench.py > gpurun_out/r40/bench.log 2>&1
