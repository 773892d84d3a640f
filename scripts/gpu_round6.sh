#!/bin/bash
# Multi-slice concurrency experiments.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/exp6
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ge 124 ]; then exit $rc; fi; return 0; }
step timeout -k 10 300 python bench.py --slices 4 --steps 20 --out gpurun_out/exp6/s4.json > gpurun_out/exp6/s4.log 2>&1
step timeout -k 10 300 python bench.py --slices 4 --steps 20 --child-env GPU_MAX_HW_QUEUES=1 --out gpurun_out/exp6/s4_q1.json > gpurun_out/exp6/s4_q1.log 2>&1
step timeout -k 10 300 python bench.py --slices 4 --steps 10 --batch 128 --out gpurun_out/exp6/s4_b128.json > gpurun_out/exp6/s4_b128.log 2>&1
step timeout -k 10 400 python bench.py --slices 8 --steps 10 --out gpurun_out/exp6/s8.json > gpurun_out/exp6/s8.log 2>&1
