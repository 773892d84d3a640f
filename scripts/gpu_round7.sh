#!/bin/bash
# Slice scaling 1/2/4/8 with 1 HW queue per slice; 2-queue and temporal variants.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/exp7
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ge 124 ]; then exit $rc; fi; return 0; }
for s in 1 2 4 8; do
  step timeout -k 10 400 python bench.py --slices $s --steps 20 --out gpurun_out/exp7/s$s.json > gpurun_out/exp7/s$s.log 2>&1
done
step timeout -k 10 300 python bench.py --slices 4 --steps 20 --hw-queues 2 --mode shim --out gpurun_out/exp7/s4_q2.json > gpurun_out/exp7/s4_q2.log 2>&1
step timeout -k 10 300 python bench.py --slices 4 --steps 20 --no-spatial --mode shim --out gpurun_out/exp7/s4_temporal_default.json > gpurun_out/exp7/s4_temporal_default.log 2>&1
step timeout -k 10 300 python bench.py --slices 4 --steps 10 --batch 128 --out gpurun_out/exp7/s4_b128.json > gpurun_out/exp7/s4_b128.log 2>&1
