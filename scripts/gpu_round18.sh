#!/bin/bash
# attention variants x CU masks; GEMM at 64 CUs (skinny plan vs hipBLASLt) for the slice-size question.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r22
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q -x > gpurun_out/r22/pytest.log 2>&1
step timeout -k 10 600 python -m k8s_vgpu_scheduler_amd.bench.attention --out gpurun_out/r22/attn.json > gpurun_out/r22/attn.log 2>&1
export HSA_CU_MASK=0:0-63
step timeout -k 10 400 python -m k8s_vgpu_scheduler_amd.bench.gemm --batches 32 --shapes gate_up,down,qkv,o_proj --sweep --out gpurun_out/r22/gemm_cu64.json > gpurun_out/r22/gemm_cu64.log 2>&1
