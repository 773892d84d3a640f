# round 2: temporal (governor) 4 x 25 % slices -- tuning sweep of the share EWMA and burst
set -o pipefail
out=gpurun_out/r2_temporal; mkdir -p $out
common="--slices 4 --no-spatial --policy force --mode shim --steps 100 --warmup 10"
timeout -k 10 200 python -u bench.py --slices 4 --mode native --steps 100 --warmup 10 --out $out/native.json > $out/native.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py $common --out $out/default.json > $out/default.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py $common --child-env MIVGPU_SHARE_TAU_MS=100 --out $out/tau100.json > $out/tau100.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py $common --child-env MIVGPU_GATE_BURST_US=100000 --out $out/burst100.json > $out/burst100.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py $common --child-env MIVGPU_SHARE_TAU_MS=100 --child-env MIVGPU_GATE_BURST_US=100000 --out $out/both.json > $out/both.log 2>&1 || exit 1
