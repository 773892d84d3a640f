#!/bin/bash
# Round 6: decode projection plans at batch 32 on the whole GPU (down / gate_up overrides, K-split down).
set -o pipefail
O=gpurun_out/r6pl
mkdir -p $O
dec() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 40 --warmup 8 > $O/dec_$tag.json 2>$O/dec_$tag.err || { echo "$tag failed"; tail -3 $O/dec_$tag.err; return 0; }
  echo "$tag $(python -c "import json;d=json.loads(open('$O/dec_$tag.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3))")"
}
dec base MIVGPU_X=1
dec wk_down MIVGPU_WIDEK=qkv,o,down
dec wk_all MIVGPU_WIDEK=qkv,o,down,gu
for p in 2,1 2,2 2,4 4,1 4,2 1,2 1,4 8,1; do dec down_$p MIVGPU_DOWN_PLAN=$p; done
for p in 2,1 2,2 4,1 1,1 1,2; do dec gu_$p MIVGPU_GU_PLAN=$p; done
dec base2 MIVGPU_X=1
