# 8-slice temporal governor over a long run (steady state): 600 steps
set -o pipefail
out=gpurun_out/s8exp; mkdir -p $out
b() { local name=$1; shift; timeout -k 10 600 python -u bench.py "$@" --out $out/$name.json > $out/$name.log 2>&1; }
b t8_long --slices 8 --rounds temporal,native --steps 600 --warmup 10
