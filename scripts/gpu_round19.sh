#!/bin/bash
# CU-aware variants: tests, attention auto choice, decode at 256/64 CUs, 4- and 8-slice bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r23
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 600 python -m pytest tests/test_ops_gpu.py tests/test_skinny_gemm_gpu.py -q -x > gpurun_out/r23/pytest.log 2>&1
step timeout -k 10 400 python -m k8s_vgpu_scheduler_amd.bench.attention --variants auto --out gpurun_out/r23/attn_auto.json > gpurun_out/r23/attn.log 2>&1
step timeout -k 10 200 python -m k8s_vgpu_scheduler_amd.bench.decode > gpurun_out/r23/decode_full.log 2>&1
step env HSA_CU_MASK=0:0-63 timeout -k 10 200 python -m k8s_vgpu_scheduler_amd.bench.decode > gpurun_out/r23/decode_cu64.log 2>&1
step timeout -k 10 420 python bench.py --mode shim --out gpurun_out/r23/s4_a.json > gpurun_out/r23/s4_a.log 2>&1
step timeout -k 10 420 python bench.py --mode shim --slices 8 --out gpurun_out/r23/s8_a.json > gpurun_out/r23/s8_a.log 2>&1
step timeout -k 10 420 python bench.py --mode shim --out gpurun_out/r23/s4_b.json > gpurun_out/r23/s4_b.log 2>&1
