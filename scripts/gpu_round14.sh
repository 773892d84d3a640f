#!/bin/bash
# Slice scaling curve 1/2/4/8 with the current code (3 rounds each: native same-queues, native HIP default, shim).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r18
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for s in 1 2 4 8; do
  step timeout -k 10 480 python bench.py --slices $s --out gpurun_out/r18/s$s.json > gpurun_out/r18/s$s.log 2>&1
done
step timeout -k 10 480 python bench.py --slices 8 --mode shim --no-spatial --policy disable --out gpurun_out/r18/s8_nomask.json > gpurun_out/r18/s8_nomask.log 2>&1
