#!/bin/bash
# skinny MFMA GEMM: numerics, then microbench vs hipBLASLt.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r15
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 300 python -m pytest tests/test_skinny_gemm_gpu.py -q -x > gpurun_out/r15/pytest.log 2>&1
step timeout -k 10 300 python -m k8s_vgpu_scheduler_amd.bench.gemm --sweep --out gpurun_out/r15/gemm.json > gpurun_out/r15/gemm.log 2>&1
