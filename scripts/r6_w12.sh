#!/bin/bash
# Round 6: decode attention on twelve-wave workgroups, one split per (b, kv-head), no combine launch.
set -o pipefail
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -v --timeout 120 --timeout-method thread \
  -k "fused_modes" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for rep in 1 2; do
  timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 50 --warmup 10 > $O/dec_base_$rep.json 2>$O/dec_base_$rep.err || exit 1
  echo "base $rep $(tail -1 $O/dec_base_$rep.json)"
  MIVGPU_ATTN_SPLITS=1 MIVGPU_ATTN_W12=1 timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 50 --warmup 10 > $O/dec_w12_$rep.json 2>$O/dec_w12_$rep.err || exit 1
  echo "w12 $rep $(tail -1 $O/dec_w12_$rep.json)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MIVGPU_ATTN_SPLITS=1 MIVGPU_ATTN_W12=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r6x/prof/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
for r in rows[:12]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), r["Percentage"])
PY
