#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r38
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step env HSA_CU_MASK=0:0-63 GPU_MAX_HW_QUEUES=2 MIVGPU_OPS_LIB=$GRAFT_REPO_ROOT/build/exp/libmivgpu_ops_nox.so timeout -k 10 600 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --sweep --shapes down,gate_up,lm_head --out gpurun_out/r38/gemm_cu64_nox.json > gpurun_out/r38/gemm_cu64_nox.log 2>&1
step env MIVGPU_OPS_LIB=$GRAFT_REPO_ROOT/build/exp/libmivgpu_ops_nox.so timeout -k 10 600 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --shapes down,gate_up,lm_head --out gpurun_out/r38/gemm_full_nox.json > gpurun_out/r38/gemm_full_nox.log 2>&1
cd /tmp && step timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/r38/counters.txt 2>&1
