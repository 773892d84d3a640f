#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r39
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 600 python -m pytest tests/test_skinny_gemm_gpu.py -q -x > gpurun_out/r39/pytest.log 2>&1
step env HSA_CU_MASK=0:0-63 timeout -k 10 600 python -m pytest tests/test_skinny_gemm_gpu.py -q -x > gpurun_out/r39/pytest_cu64.log 2>&1
step env HSA_CU_MASK=0:0-63 GPU_MAX_HW_QUEUES=2 timeout -k 10 900 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --sweep --out gpurun_out/r39/gemm_cu64.json > gpurun_out/r39/gemm_cu64.log 2>&1
step timeout -k 10 900 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --sweep --out gpurun_out/r39/gemm_full.json > gpurun_out/r39/gemm_full.log 2>&1
for w in 0 1; do
step env HSA_CU_MASK=0:0-63 GPU_MAX_HW_QUEUES=2 MIVGPU_SKINNY_WIDE=$w timeout -k 10 600 python -m k8s_vgpu_scheduler_amd.bench.decode --batch 32 --steps 30 > gpurun_out/r39/decode_cu64_wide$w.log 2>&1
step env MIVGPU_SKINNY_WIDE=$w timeout -k 10 600 python -m k8s_vgpu_scheduler_amd.bench.decode --batch 32 --steps 30 > gpurun_out/r39/decode_full_wide$w.log 2>&1
done
