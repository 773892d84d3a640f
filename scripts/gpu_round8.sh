#!/bin/bash
# HW-queue sweep per slice count (shim round only; native numbers from exp7).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/exp8
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ge 124 ]; then exit $rc; fi; return 0; }
for cfg in "2 2" "2 4" "4 4" "8 2" "8 4"; do
  set -- $cfg
  step timeout -k 10 300 python bench.py --slices $1 --hw-queues $2 --mode shim --steps 20 --out gpurun_out/exp8/s$1_q$2.json > gpurun_out/exp8/s$1_q$2.log 2>&1
done
step timeout -k 10 300 python bench.py --slices 8 --hw-queues 1 --mode shim --steps 20 --batch 16 --out gpurun_out/exp8/s8_q1_b16.json > gpurun_out/exp8/s8_q1_b16.log 2>&1
