#!/bin/bash
set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
export MIVGPU_TEST_BENCH_LOGS=$PWD/$O/benchlogs
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_e2e_gpu.py::test_time_sharing_mode_on_the_real_node \
  tests/test_shim_interpose_gpu.py::test_triton_kernel_loop_held_to_its_share \
  "tests/test_shim_gpu.py::test_eight_temporal_tenants_run_like_native" \
  "tests/test_shim_gpu.py::test_eight_pooled_slices_with_the_monitor_switch" > $O/fix_tests.log 2>&1
echo "rc=$?"
grep -E "PASSED|FAILED|passed|failed|ratio|temporal\"|\"shim\"" $O/fix_tests.log | cut -c1-400 | tail -12
