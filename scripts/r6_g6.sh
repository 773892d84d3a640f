#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6r
timeout -k 10 300 python -u -m pytest -v -s --timeout 280 --timeout-method thread \
  tests/test_shim_gpu.py::test_temporal_slices_charged_the_share_they_receive > gpurun_out/r6r/t.log 2>&1
echo "rc=$?"; grep -E "passed|failed|governed" gpurun_out/r6r/t.log | cut -c1-300
O=gpurun_out/r6s bash scripts/r6_serving.sh
