#!/bin/bash
# Why do 64-CU slices underperform? single-slice decode under CU masks + profile.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/prof
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ge 124 ]; then exit $rc; fi; return 0; }
for m in "" "0:0-127" "0:0-63" "0:0-31"; do
  HSA_CU_MASK="$m" step timeout -k 10 200 python -m k8s_vgpu_scheduler_amd.bench.decode --batch 32 --steps 20 >> gpurun_out/decode_cumask.log 2>&1
  echo "mask=[$m]" >> gpurun_out/decode_cumask.log
done
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && HSA_CU_MASK=0:0-63 step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof/decode_b32_cu64 -o run --output-format csv -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --batch 32 --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/prof/decode_b32_cu64.log 2>&1
