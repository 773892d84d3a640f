#!/bin/bash
# Round 6: PyTorch TunableOp over the prefill GEMMs (hipBLASLt + rocBLAS solutions, timed per shape).
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
P="python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 8448"
timeout -k 10 300 $P --iters 10 > $O/base.json 2>$O/base.err || exit 1
cat $O/base.json
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
  PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tune%d.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=300 \
  timeout -k 10 900 $P --iters 1 --eager > $O/tune.json 2>$O/tune.err || { echo "tune rc=$?"; tail -5 $O/tune.err; exit 1; }
ls -la $O; head -20 $O/tune0.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tune%d.csv \
  timeout -k 10 300 $P --iters 10 > $O/tuned.json 2>$O/tuned.err || exit 1
cat $O/tuned.json
timeout -k 10 300 $P --iters 10 > $O/base2.json 2>$O/base2.err || exit 1
cat $O/base2.json
