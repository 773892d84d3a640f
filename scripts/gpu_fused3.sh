# rmsnorm + fused-mode defaults: numerics, decode step, 4-slice bench, kernel profile
set -o pipefail
out=gpurun_out/fused3; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > $out/ops_tests.log 2>&1 || exit 1
for m in "" "0:0-63"; do
  tag=$(echo "$m" | tr -d ':-'); [ -z "$m" ] && tag=full
  if [ -n "$m" ]; then export HSA_CU_MASK="$m"; else unset HSA_CU_MASK; fi
  timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 30 > $out/decode_$tag.log 2>&1 || exit 1
done
unset HSA_CU_MASK
timeout -k 10 300 python -u bench.py --out $out/s4.json > $out/s4.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_full -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 > $GRAFT_REPO_ROOT/$out/prof_full.log 2>&1 || exit 1
