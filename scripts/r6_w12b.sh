#!/bin/bash
# Round 6: twelve-wave one-split decode attention as the default -- numerics, whole GPU and 64-CU A/B, headline.
set -o pipefail
O=gpurun_out/r6y
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -v --timeout 120 --timeout-method thread \
  -k "fused_modes or one_split or fused_matches_unfused or decoder_native or skinny_path or norm_fused_matches or combine_in_o_proj or widek_matches" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
dec() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 50 --warmup 10 > $O/dec_$tag.json 2>$O/dec_$tag.err || { echo "$tag failed"; tail -5 $O/dec_$tag.err; exit 1; }
  echo "$tag $(python -c "import json;d=json.loads(open('$O/dec_$tag.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), round(d['tok_s']))")"
}
for rep in 1 2; do
  dec def_$rep MIVGPU_X=1
  dec off_$rep MIVGPU_ATTN_W12=0
  dec c64def_$rep HSA_CU_MASK=0:0-63
  dec c64off_$rep HSA_CU_MASK=0:0-63 MIVGPU_ATTN_W12=0
done
timeout -k 10 400 python -u bench.py --out $O/bench.json > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench',d['value'],d.get('native_value'),d.get('slice_fairness_min_over_max'),d.get('shim_overhead_pct'),d.get('temporal_value'))"
