# runtime-VRAM (context) accounting in the shim: shim + e2e GPU tests, 4-slice bench shim round
set -o pipefail
out=gpurun_out/ctx; mkdir -p $out
ls -la /sys/class/kfd/kfd/proc/ > $out/kfd_proc_ls.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests/test_shim_gpu.py tests/test_e2e_gpu.py -x -v -s --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --mode shim --out $out/s4_shim.json > $out/s4_shim.log 2>&1 || exit 1
