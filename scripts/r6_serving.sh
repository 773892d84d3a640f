#!/bin/bash
# Serving TTFT / per-token natively and in the gpumem-50 % slice, with 8k prompts (heartbeat every minute).
set -o pipefail
O=${O:-gpurun_out/r6s}
mkdir -p $O
timeout -k 10 900 python -u -m k8s_vgpu_scheduler_amd.bench.serving --configs native,vgpu50 --warmup 30 --runs 200 \
  --long-prompt-tokens 8000 --long-runs 5 --out-dir $O > $O/serving.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 60; echo "$(date +%T) $(tail -c 200 $O/serving.log | tr '\n' ' ')"; done
wait $pid; rc=$?
echo "serving rc=$rc"
cat $O/summary.json 2>/dev/null | head -60
exit $rc
