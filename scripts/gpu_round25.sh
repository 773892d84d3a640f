#!/bin/bash
# governor PMC evidence: per-kernel SQ_WAVES / SQ_BUSY_CU_CYCLES / GRBM_GUI_ACTIVE and MFMA bf16 ops, native vs 50 %.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r30
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd /tmp
step timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r30/native_a -o run -- python3 -m k8s_vgpu_scheduler_amd.shim.probe --child mfma --iters 30 > $GRAFT_REPO_ROOT/gpurun_out/r30/native_a.log 2>&1
step timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r30/native_b -o run -- python3 -m k8s_vgpu_scheduler_amd.shim.probe --child mfma --iters 30 > $GRAFT_REPO_ROOT/gpurun_out/r30/native_b.log 2>&1
export LD_PRELOAD=$GRAFT_REPO_ROOT/k8s_vgpu_scheduler_amd/lib/libmivgpu.so MIVGPU_SHARED_CACHE=/tmp/gov50.cache HIP_DEVICE_CORE_LIMIT=50 GPU_CORE_UTILIZATION_POLICY=force
step timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r30/gov50_a -o run -- python3 -m k8s_vgpu_scheduler_amd.shim.probe --child mfma --iters 30 > $GRAFT_REPO_ROOT/gpurun_out/r30/gov50_a.log 2>&1
step timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r30/gov50_b -o run -- python3 -m k8s_vgpu_scheduler_amd.shim.probe --child mfma --iters 30 > $GRAFT_REPO_ROOT/gpurun_out/r30/gov50_b.log 2>&1
