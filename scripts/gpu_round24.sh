#!/bin/bash
# governor evidence: counter list, kernel trace of a governed MFMA load (50 %, force), native trace.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r29
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd /tmp
step timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/r29/counters.txt 2>&1
step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r29/native -o run -- python3 -m k8s_vgpu_scheduler_amd.shim.probe --child mfma --iters 60 > $GRAFT_REPO_ROOT/gpurun_out/r29/native.log 2>&1
export LD_PRELOAD=$GRAFT_REPO_ROOT/k8s_vgpu_scheduler_amd/lib/libmivgpu.so MIVGPU_SHARED_CACHE=/tmp/gov50.cache HIP_DEVICE_CORE_LIMIT=50 GPU_CORE_UTILIZATION_POLICY=force
step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r29/gov50 -o run -- python3 -m k8s_vgpu_scheduler_amd.shim.probe --child mfma --iters 60 > $GRAFT_REPO_ROOT/gpurun_out/r29/gov50.log 2>&1
