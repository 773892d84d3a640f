#!/bin/bash
# Round 6: vectorised prefill QK-norm/RoPE kernel -- numerics, 8k prefill A/B, kernel stats.
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -v --timeout 300 --timeout-method thread \
  -k "prefill" > $O/pf_tests.log 2>&1 || { echo "prefill tests failed"; tail -40 $O/pf_tests.log; exit 1; }
grep -E "passed|failed" $O/pf_tests.log | tail -1
timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 8448 --iters 10 > $O/pf8k_vec.json 2>$O/pf8k_vec.err || exit 1
MIVGPU_PREFILL_QK=8 timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 8448 --iters 10 > $O/pf8k_old.json 2>$O/pf8k_old.err || exit 1
cat $O/pf8k_vec.json $O/pf8k_old.json
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 8448 --iters 3 > $O/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $O/prof.log; }
find $O/prof -name "*kernel_stats.csv" | head -3
