#!/bin/bash
# Round 6: 8k prefill kernel profile on the final code (XCD-ordered flash attention, GEMM residual add).
set -o pipefail
O=gpurun_out/r6pp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 8448 --iters 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
grep '^{' $O/prof.log | tail -1
