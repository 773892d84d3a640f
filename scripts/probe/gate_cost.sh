# cost of one gate kernel: rocprofv3 kernel trace of the launch microbenchmark
# (native, shim governor off, shim governor on -- stops at the first failure)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; out=$R/gpurun_out/gate_cost; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
run() {  # run <name> <env...>
  local name=$1; shift
  echo "[gate_cost] $name"
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/$name -- $R/build/bench/launch_bench 20000 500 > $out/$name.log 2>&1
}
SHIM=$R/k8s_vgpu_scheduler_amd/lib/libmivgpu.so
run native A=1 && \
run shim_off LD_PRELOAD=$SHIM MIVGPU_SHARED_CACHE=/tmp/gc1.cache && \
run shim_on_nograph LD_PRELOAD=$SHIM MIVGPU_SHARED_CACHE=/tmp/gc2.cache HIP_DEVICE_CORE_LIMIT=90 GPU_CORE_UTILIZATION_POLICY=force LAUNCH_BENCH_NO_GRAPH=1
