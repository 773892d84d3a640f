# PMC counters of one 64-CU slice decode step (eager launches): HBM bytes per kernel, MFMA ops, LDS conflicts
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/pmc; mkdir -p $out
cd /tmp && export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT HSA_CU_MASK=0:0-63
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/a -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 3 --warmup 1 --no-graph > $out/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d $out/b -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 3 --warmup 1 --no-graph > $out/b.log 2>&1 || exit 1
