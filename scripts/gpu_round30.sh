#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r35
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 600 python -m k8s_vgpu_scheduler_amd.bench.membw --out gpurun_out/r35/membw.json > gpurun_out/r35/membw.log 2>&1
export HSA_CU_MASK=0:0-63 GPU_MAX_HW_QUEUES=2
cd /tmp
step timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r35/prof64 -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --batch 32 --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/r35/decode64.log 2>&1
