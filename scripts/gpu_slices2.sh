# slice-partition plan table: plan tests, decode step at 32/64 CUs, 4- and 8-slice benches
set -o pipefail
out=gpurun_out/slices2; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_skinny_gemm_gpu.py tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for m in 0:0-31 0:0-63; do
  tag=$(echo $m | tr -d ':-')
  HSA_CU_MASK=$m timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 50 > $out/decode_$tag.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --slices 8 --mode shim --out $out/s8_shim.json > $out/s8_shim.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --out $out/s4_all.json > $out/s4_all.log 2>&1 || exit 1
