#!/bin/bash
# smoke + full GPU test suite + default headline bench (3 rounds).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r10
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r10/smoke.log 2>&1
step timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/r10/pytest_gpu.log 2>&1
step timeout -k 10 420 python bench.py --out gpurun_out/r10/bench.json > gpurun_out/r10/bench.log 2>&1
