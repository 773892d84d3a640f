#!/bin/bash
# attention v2 (all loads up front): numerics, decode full GPU and 64-CU slice (profiled), 4-slice bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r21
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q -x > gpurun_out/r21/pytest.log 2>&1
step timeout -k 10 200 python -m k8s_vgpu_scheduler_amd.bench.decode > gpurun_out/r21/decode_full.log 2>&1
export HSA_CU_MASK=0:0-63
step timeout -k 10 200 python -m k8s_vgpu_scheduler_amd.bench.decode > gpurun_out/r21/decode_cu64.log 2>&1
cd /tmp && step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r21/prof_cu64 -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode > $GRAFT_REPO_ROOT/gpurun_out/r21/prof_cu64.log 2>&1
unset HSA_CU_MASK
cd $GRAFT_REPO_ROOT && step timeout -k 10 420 python bench.py --mode shim --out gpurun_out/r21/s4.json > gpurun_out/r21/s4.log 2>&1
