#!/bin/bash
# Default bench (4 slices, 2 HW queues) + native baselines with 2 queues/process.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/exp9
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ge 124 ]; then exit $rc; fi; return 0; }
step timeout -k 10 300 python bench.py --out gpurun_out/exp9/default.json > gpurun_out/exp9/default.log 2>&1
for s in 2 4 8; do
  step timeout -k 10 300 python bench.py --slices $s --mode native --child-env GPU_MAX_HW_QUEUES=2 --out gpurun_out/exp9/native_q2_s$s.json > gpurun_out/exp9/native_q2_s$s.log 2>&1
done
step timeout -k 10 300 python bench.py --slices 4 --mode shim --no-spatial --policy disable --out gpurun_out/exp9/s4_nomask_q2.json > gpurun_out/exp9/s4_nomask_q2.log 2>&1
