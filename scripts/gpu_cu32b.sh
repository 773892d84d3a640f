# 32-CU slice: qkv on the wide kernel vs hipBLASLt, kernel profile, 8-slice bench
set -o pipefail
out=gpurun_out/cu32b; mkdir -p $out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "decoder" > $out/tests.log 2>&1 || exit 1
for q in 48 0; do
  HSA_CU_MASK=0:0-31 MIVGPU_QKV_WIDE_CUS=$q timeout -k 10 200 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 30 > $out/decode_cu32_q$q.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --slices 8 --mode shim --out $out/s8_shim.json > $out/s8_shim.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && export PYTHONPATH=$R
HSA_CU_MASK=0:0-31 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$out/prof_cu32 -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 > $R/$out/prof_cu32.log 2>&1 || exit 1
