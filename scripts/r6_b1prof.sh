#!/bin/bash
# Round 6: batch-1 decode kernel profile (whole GPU).
set -o pipefail
O=gpurun_out/r6b1
mkdir -p $O
timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 1 --steps 50 --warmup 10 > $O/dec_b1.json 2>$O/dec_b1.err || { tail -5 $O/dec_b1.err; exit 1; }
tail -1 $O/dec_b1.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --batch 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo prof done
