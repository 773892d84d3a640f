# 8-slice round-order effect after the bench parent stopped holding GPU queues
set -o pipefail
out=gpurun_out/s8exp; mkdir -p $out
b() { local name=$1; shift; timeout -k 10 600 python -u bench.py "$@" --out $out/$name.json > $out/$name.log 2>&1; }
b order_fixed --slices 8 --rounds masked_noshim,shim,native --round-gap 0 &&
b all8 --slices 8
