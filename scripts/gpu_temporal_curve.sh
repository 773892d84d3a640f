# temporal-only isolation (no CU masks, governor forced, 100/N % each) at 2 and 8 slices
set -o pipefail
out=gpurun_out/temporal; mkdir -p $out
for n in 2 8; do
  timeout -k 10 400 python -u bench.py --slices $n --no-spatial --policy force --mode shim --out $out/s$n.json > $out/s$n.log 2>&1 || exit 1
done
