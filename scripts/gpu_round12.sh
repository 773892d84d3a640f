#!/bin/bash
# skinny GEMM plan + decoder integration: numerics, decode A/B, profile, headline bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r16
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 400 python -m pytest tests/test_skinny_gemm_gpu.py tests/test_ops_gpu.py -q -x > gpurun_out/r16/pytest.log 2>&1
step timeout -k 10 300 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --out gpurun_out/r16/gemm.json > gpurun_out/r16/gemm.log 2>&1
step timeout -k 10 200 python -m k8s_vgpu_scheduler_amd.bench.decode --gemm hipblaslt > gpurun_out/r16/decode_blas.log 2>&1
step timeout -k 10 200 python -m k8s_vgpu_scheduler_amd.bench.decode --gemm skinny > gpurun_out/r16/decode_skinny.log 2>&1
cd /tmp && step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r16/prof -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --gemm skinny > $GRAFT_REPO_ROOT/gpurun_out/r16/prof.log 2>&1
cd $GRAFT_REPO_ROOT && step timeout -k 10 420 python bench.py --out gpurun_out/r16/bench.json > gpurun_out/r16/bench.log 2>&1
