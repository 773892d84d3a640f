#!/bin/bash
# 8-slice A/B: skinny GEMM on/off (repeat), to find the source of the 8-slice unfairness.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r19
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 420 python bench.py --slices 8 --mode shim --steps 40 --out gpurun_out/r19/s8_skinny_a.json > gpurun_out/r19/s8_skinny_a.log 2>&1
step timeout -k 10 420 python bench.py --slices 8 --mode shim --steps 40 --child-env MIVGPU_SKINNY_GEMM=0 --out gpurun_out/r19/s8_blas.json > gpurun_out/r19/s8_blas.log 2>&1
step timeout -k 10 420 python bench.py --slices 8 --mode shim --steps 40 --out gpurun_out/r19/s8_skinny_b.json > gpurun_out/r19/s8_skinny_b.log 2>&1
step timeout -k 10 420 python bench.py --slices 4 --mode shim --steps 40 --child-env MIVGPU_SKINNY_GEMM=0 --out gpurun_out/r19/s4_blas.json > gpurun_out/r19/s4_blas.log 2>&1
