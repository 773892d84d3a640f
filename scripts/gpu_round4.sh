#!/bin/bash
# Governor after the stamper fix; temporal vs spatial slices on the decode bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ge 124 ]; then exit $rc; fi; return 0; }
step timeout -k 10 300 python -m k8s_vgpu_scheduler_amd.shim.probe --quick --out gpurun_out/probe_quick4.json > gpurun_out/probe_quick4.log 2>&1
step timeout -k 10 400 python bench.py --slices 4 --no-spatial --policy force --mode shim --steps 20 --out gpurun_out/bench_temporal4.json > gpurun_out/bench_temporal4.log 2>&1
step timeout -k 10 400 python bench.py --slices 1 --steps 20 --out gpurun_out/bench_s1.json > gpurun_out/bench_s1.log 2>&1
step timeout -k 10 400 python bench.py --slices 2 --steps 20 --out gpurun_out/bench_s2.json > gpurun_out/bench_s2.log 2>&1
