#!/bin/bash
# interleaved A/B at 4 and 8 slices, 100 steps: skinny vs hipBLASLt projections.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r20
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in a b; do
  for s in 4 8; do
    step timeout -k 10 420 python bench.py --slices $s --mode shim --out gpurun_out/r20/s${s}_skinny_$rep.json > gpurun_out/r20/s${s}_skinny_$rep.log 2>&1
    step timeout -k 10 420 python bench.py --slices $s --mode shim --child-env MIVGPU_SKINNY_GEMM=0 --out gpurun_out/r20/s${s}_blas_$rep.json > gpurun_out/r20/s${s}_blas_$rep.log 2>&1
  done
done
