#!/bin/bash
# Round 6: 8k prefill with the MLP over row chunks (Infinity-Cache-resident gate_up output) -- A/B + profile.
set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
pf() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 8448 --iters 10 > $O/pf_$tag.json 2>$O/pf_$tag.err || { echo "$tag failed"; tail -5 $O/pf_$tag.err; exit 1; }
  echo "$tag $(tail -1 $O/pf_$tag.json)"
}
for rep in 1 2; do
  pf c0_$rep MIVGPU_PREFILL_MLP_CHUNK=0
  pf c2048_$rep MIVGPU_PREFILL_MLP_CHUNK=2048
  pf c4096_$rep MIVGPU_PREFILL_MLP_CHUNK=4096
done
pf c1024_1 MIVGPU_PREFILL_MLP_CHUNK=1024
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 8448 --iters 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo prof done
