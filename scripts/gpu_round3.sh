#!/bin/bash
# Governor trace + CU-mask -> XCD mapping + decode kernel profile.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/prof
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ge 124 ]; then exit $rc; fi; return 0; }
step timeout -k 10 300 python -m k8s_vgpu_scheduler_amd.shim.probe --quick --hwid --out gpurun_out/probe_quick3.json > gpurun_out/probe_quick3.log 2>&1
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof/decode_b32 -o run --output-format csv -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --batch 32 --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/prof/decode_b32.log 2>&1
