#!/bin/bash
# full regression: smoke + all GPU tests + headline bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r28
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r28/smoke.log 2>&1
step timeout -k 10 1200 python -m pytest tests -m gpu -q -x > gpurun_out/r28/pytest_gpu.log 2>&1
step timeout -k 10 600 python bench.py --out gpurun_out/r28/bench.json > gpurun_out/r28/bench.log 2>&1
