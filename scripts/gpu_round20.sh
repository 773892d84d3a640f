#!/bin/bash
# profile a 64-CU slice (decode) with the current code.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r24
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
export HSA_CU_MASK=0:0-63
cd /tmp && step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r24/prof_cu64 -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode > $GRAFT_REPO_ROOT/gpurun_out/r24/prof_cu64.log 2>&1
