# temporal governor with the cross-tenant share board: duty cycle alone, 4 x 25 % and 2 x 50 % tenants
set -o pipefail
out=gpurun_out/board; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_shim_gpu.py -x -q --timeout 200 --timeout-method thread -k "governor" > $out/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --slices 4 --no-spatial --policy force --mode shim --out $out/s4_board.json > $out/s4_board.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --slices 4 --no-spatial --policy force --mode shim --child-env MIVGPU_SHARE_BOARD=0 --out $out/s4_noboard.json > $out/s4_noboard.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --slices 2 --no-spatial --policy force --mode shim --out $out/s2_board.json > $out/s2_board.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --slices 1 --mode shim --child-env HIP_DEVICE_CORE_LIMIT=50 --child-env GPU_CORE_UTILIZATION_POLICY=force --out $out/s1_50.json > $out/s1_50.log 2>&1 || exit 1
