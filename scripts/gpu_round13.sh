#!/bin/bash
# full GPU test suite incl. load generators.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out/r17
step() { "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 900 python -m pytest tests -m gpu -q -x -rs > gpurun_out/r17/pytest_gpu.log 2>&1
