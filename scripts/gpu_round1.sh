cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo pytest_rc=$? ; tail -5 gpurun_out/pytest_gpu.log; \
timeout -k 10 300 python -m k8s_vgpu_scheduler_amd.shim.probe --quick --out gpurun_out/probe_quick.json > gpurun_out/probe_quick.log 2>&1; echo probe_rc=$?; \
MIVGPU_BENCH_LOGS=gpurun_out/bench_tiny timeout -k 10 300 python bench.py --model qwen3-tiny --steps 10 --warmup 3 --slices 2 > gpurun_out/bench_tiny.log 2>&1; echo tiny_rc=$?; tail -3 gpurun_out/bench_tiny.log; \
MIVGPU_BENCH_LOGS=gpurun_out/bench_full timeout -k 10 600 python bench.py --steps 20 --warmup 5 --out gpurun_out/bench_full.json > gpurun_out/bench_full.log 2>&1; echo full_rc=$?; tail -3 gpurun_out/bench_full.log
