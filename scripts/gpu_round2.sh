#!/bin/bash
# Round-1 step 2: governor re-check + decode profile.  Stops at the first
# GPU step that times out / faults (rc >= 124).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/prof
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ge 124 ]; then exit $rc; fi; return 0; }
step timeout -k 10 300 python -m k8s_vgpu_scheduler_amd.shim.probe --quick --out gpurun_out/probe_quick2.json > gpurun_out/probe_quick2.log 2>&1
for b in 1 32 128; do
  step timeout -k 10 200 python -m k8s_vgpu_scheduler_amd.bench.decode --batch $b --steps 20 >> gpurun_out/decode_single.log 2>&1
done
cd /tmp && step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof/decode_b32 -o run --output-format csv -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --batch 32 --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/prof/decode_b32.log 2>&1
