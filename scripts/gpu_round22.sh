#!/bin/bash
# attention split size 128 vs 256 (PF auto/2) at 256/64/32 CUs.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r27
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 600 python -m k8s_vgpu_scheduler_amd.bench.attention --variants 0,2 --out gpurun_out/r27/attn256.json > gpurun_out/r27/attn256.log 2>&1
step env MIVGPU_OPS_LIB=$GRAFT_REPO_ROOT/build/exp/libmivgpu_ops_split128.so timeout -k 10 600 python -m k8s_vgpu_scheduler_amd.bench.attention --variants 0,2 --out gpurun_out/r27/attn128.json > gpurun_out/r27/attn128.log 2>&1
