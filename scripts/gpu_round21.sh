#!/bin/bash
# streaming attention (pf 3): numerics + variants x masks.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r26
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -q -x -k "attention" > gpurun_out/r26/pytest.log 2>&1
step timeout -k 10 600 python -m k8s_vgpu_scheduler_amd.bench.attention --variants 2,3 --out gpurun_out/r26/attn.json > gpurun_out/r26/attn.log 2>&1
