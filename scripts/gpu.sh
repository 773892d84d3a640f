#!/usr/bin/env bash
# One parameterised runner for the GPU-box measurements (replaces the round-1
# one-off scripts/gpu_*.sh; their commands live on in git history).  Run on a
# MI355X box, e.g. through gpurun:
#     gpurun --timeout 1200 -- 'bash scripts/gpu.sh full'
# Suites (each step has its own time limit; the first failure ends the run):
#   full        GPU test suite + smoke + default bench (all rounds)
#   bench [N..] bench.py --slices N for each N (default 1 2 4 8), all rounds
#   governor    governor GPU tests + bench (spatial, temporal, native rounds)
#   interpose   run-time lookup / governor / tamper GPU tests + governed bench rounds
#   busyshare   rocprofv3 busy share of governed tenants (scripts/probe/governor_busyshare.py)
#   probes      KFD occupancy + topology probes (scripts/probe/*.py)
#   kernels     rocprofv3 --kernel-trace --stats of one 64-CU slice decode step
#   kernels_full  the same on the whole GPU (kernel trace: durations and the gaps between them)
#   pmc [cfg..] PMC passes over a decode step: whole GPU, 64 CUs, 32 CUs (one counter group per pass)
#   membw       partition read ceilings (bench/membw.py)
#   widek       K-split wide GEMM kernel: numerics, GEMM sweep, decode A/B
#   decode      ops + GEMM GPU tests, decode per partition size and batch 1, whole-GPU kernel trace
#   normfused   row-norm fusion on the wide / K-split kernels: tests, decode A/B, profile
#   attnsplit   fused attention, one split per (b, kv-head) vs per 256 keys: tests, decode A/B, profile
#   mall        projection GEMMs cold vs with their weights prefetched into the Infinity Cache
#   serving     TTFT / per-token latency, native vs vGPU slices (bench/serving.py)
#   mixed       governed server + 3 governed decode tenants; 8 x 12 % temporal over 600 steps
#   board       share board: 4 x 25 % / 8 x 12.5 % temporal vs native, unequal limits, time-sharing e2e
#   fair        temporal (fair-share governor) vs native: 4 slices at 20 / 100 steps, 8 slices
#   fair2       fair-share governor: 4 / 8 symmetric tenants, 75/25 and 50/25/25
#   eight       8 slices: disjoint ranges vs one pooled whole-GPU range (cuShareUnit 256), monitor on/off
#   kern        prefill kernels: flash attention at 512 / 2048 / 8192, packed-weight GEMM v2 / v1 vs hipBLASLt,
#               8k-token TTFT (library and native GEMM)
#   prefill     prefill microbench + rocprofv3 kernel summary, whole GPU and 64 CUs
# Results go to gpurun_out/<suite>/ (copy the ones to keep into profiles/).
set -o pipefail
suite=${1:-full}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$suite; mkdir -p "$out"
cd "$R"

step() {  # step <seconds> <log name> <command...>
  local t=$1 name=$2; shift 2
  echo "[gpu.sh] $suite/$name: $*"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "[gpu.sh] $name failed rc=$rc (see $out/$name.log)"; exit $rc; }
}

case $suite in
  full)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1
    rc=$?; [ $rc -le 1 ] || exit $rc
    step 200 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
    step 400 bench python -u bench.py --out "$out/bench.json"
    exit $rc ;;
  bench)
    for n in ${@:-1 2 4 8}; do step 400 "s$n" python -u bench.py --slices "$n" --out "$out/s$n.json"; done ;;
  governor)
    step 900 tests python -u -m pytest tests/test_shim_gpu.py -v -s --timeout 300 --timeout-method thread \
      -k "governor or temporal or masked or heavy or launch or grant"
    step 400 bench python -u bench.py --out "$out/bench.json" ;;
  interpose)
    step 900 tests python -u -m pytest tests/test_shim_interpose_gpu.py tests/test_shim_gpu.py -v -s --timeout 300 \
      --timeout-method thread -k "interpose or governor or temporal or heavy or triton or compile or tamper or queue"
    step 400 bench python -u bench.py --rounds governed_ref,governed,temporal --steps 100 --out "$out/bench.json" ;;
  busyshare)
    step 500 busyshare python -u scripts/probe/governor_busyshare.py ;;
  probes)
    step 120 kfd_matmul python -u scripts/probe/kfd_occupancy.py
    step 500 kfd_decode python -u scripts/probe/kfd_decode_occupancy.py
    step 120 topology python -u scripts/probe/topology_probe.py ;;
  kernels)
    cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
    HSA_CU_MASK=0:0-63 step 240 prof_cu64 rocprofv3 --kernel-trace --stats -d "$out/prof_cu64" -o run -- \
      python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 ;;
  kernels_full)
    cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
    step 240 prof_full rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_full" -o run -- \
      python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20
    MIVGPU_NORM_FUSED=1 step 240 prof_fused rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$out/prof_fused" -o run -- python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 ;;
  pmc)
    # per-kernel counters of one decode step for each partition size: the whole
    # GPU (1 slice), 64 CUs (4 slices) and 32 CUs (8 slices); one counter group
    # per pass.  pmc [full|cu64|cu32 ...]
    cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
    dec="python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 3 --warmup 1 --no-graph"
    for cfg in ${@:-full cu64 cu32}; do
      case $cfg in full) unset HSA_CU_MASK ;; cu64) export HSA_CU_MASK=0:0-63 ;; cu32) export HSA_CU_MASK=0:0-31 ;;
        *) echo "unknown $cfg"; exit 2 ;; esac
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
        -d "$out/$cfg/a" -o run -- $dec > "$out/$cfg.a.log" 2>&1 || exit 1
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 \
        SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d "$out/$cfg/b" -o run -- $dec \
        > "$out/$cfg.b.log" 2>&1 || exit 1
      # per-kernel summary; the raw CSVs are tens of MB per configuration
      python3 "$R/scripts/probe/pmc_summary.py" "$out/$cfg" > "$out/$cfg.json" && rm -rf "$out/$cfg"
    done ;;
  govmodes)
    # A/B of the governor's bucket (host / device) and share estimator on 8 x 12 %
    step 400 host_ratio python -u bench.py --slices 8 --rounds temporal --steps 600 --out "$out/host_ratio.json"
    MIVGPU_GATE_MODE=device step 400 device_ratio python -u bench.py --slices 8 --rounds temporal --steps 600 \
      --out "$out/device_ratio.json"
    MIVGPU_GATE_MODE=device MIVGPU_SHARE_EST=instant MIVGPU_SHARE_TAU_MS=20 step 400 device_inst20 \
      python -u bench.py --slices 8 --rounds temporal --steps 600 --out "$out/device_inst20.json"
    MIVGPU_SHARE_EST=instant MIVGPU_SHARE_TAU_MS=20 step 400 host_inst20 \
      python -u bench.py --slices 8 --rounds temporal --steps 600 --out "$out/host_inst20.json" ;;
  widek)
    # K-split wide kernel: numerics, GEMM sweep, decode A/B (whole GPU and 64 CUs)
    step 600 tests python -u -m pytest tests/test_ops_gpu.py -v --timeout 300 --timeout-method thread -k "widek"
    step 300 gemm python -u -m k8s_vgpu_scheduler_amd.bench.gemm --shapes qkv,o_proj,down --batches 1,32 \
      --out "$out/gemm.json"
    for wk in off qkv,o qkv,o,down; do
      tag=${wk//,/_}
      MIVGPU_WIDEK=$wk step 300 "full_$tag" python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 200
    done
    HSA_CU_MASK=0:0-63 MIVGPU_WIDEK=qkv,o step 300 cu64_qkv_o python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 100
    HSA_CU_MASK=0:0-63 MIVGPU_WIDEK=off step 300 cu64_off python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 100
    step 300 serve_b1 python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 1 --steps 200
    MIVGPU_WIDEK=off step 300 serve_b1_off python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 1 --steps 200 ;;
  attnsplit)
    # fused attention with one split per (b, kv-head) (waves loop over the
    # context, no combine launch) vs one split per 256 keys: numerics, decode A/B
    step 600 tests python -u -m pytest tests/test_ops_gpu.py -v --timeout 300 --timeout-method thread -k "fused"
    for sp in "" 0; do
      tag=split${sp:-auto}
      MIVGPU_ATTN_SPLITS=$sp step 300 "full_$tag" python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 200
      HSA_CU_MASK=0:0-63 MIVGPU_ATTN_SPLITS=$sp step 300 "cu64_$tag" python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 100
      HSA_CU_MASK=0:0-31 MIVGPU_ATTN_SPLITS=$sp step 300 "cu32_$tag" python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 60
      MIVGPU_ATTN_SPLITS=$sp step 300 "b1_$tag" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 1 --steps 200
    done
    cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
    step 240 prof_full rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_full" -o run -- \
      python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 ;;
  normfused)
    # row-norm fusion with qkv / o_proj on the K-split kernel: numerics, decode A/B per partition size
    step 900 tests python -u -m pytest tests/test_ops_gpu.py tests/test_skinny_gemm_gpu.py -v --timeout 300 \
      --timeout-method thread -k "norm or fused or widek or row_scale"
    for nf in 0 1; do
      MIVGPU_NORM_FUSED=$nf step 300 "full_nf$nf" python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 200
      HSA_CU_MASK=0:0-63 MIVGPU_NORM_FUSED=$nf step 300 "cu64_nf$nf" python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 100
      HSA_CU_MASK=0:0-31 MIVGPU_NORM_FUSED=$nf step 300 "cu32_nf$nf" python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 60
      MIVGPU_NORM_FUSED=$nf step 300 "b1_nf$nf" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 1 --steps 200
    done
    cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
    MIVGPU_NORM_FUSED=1 step 240 prof_nf rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_nf" -o run -- \
      python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20 ;;
  decode)
    # the ops / GEMM GPU tests, then decode per partition size and batch 1, then a kernel trace of the whole GPU
    # (extra env for an A/B: e.g. DEC_ENV="MIVGPU_WIDEK=qkv,o,gu")
    [ -n "$DEC_ENV" ] && export $DEC_ENV
    step 900 tests python -u -m pytest tests/test_ops_gpu.py tests/test_skinny_gemm_gpu.py -v --timeout 300 \
      --timeout-method thread
    step 300 full python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 200
    HSA_CU_MASK=0:0-63 step 300 cu64 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 100
    HSA_CU_MASK=0:0-31 step 300 cu32 python -u -m k8s_vgpu_scheduler_amd.bench.decode --steps 60
    step 300 b1 python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 1 --steps 200
    cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
    step 240 prof rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
      python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 20
    step 240 prof_b1 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_b1" -o run -- \
      python3 -m k8s_vgpu_scheduler_amd.bench.decode --batch 1 --steps 20 ;;
  mall)
    step 300 mall python -u scripts/probe/mall_prefetch.py --out "$out/mall.json" ;;
  membw)
    for b in 2 4 8 16; do
      step 300 "membw8_b$b" python -u -m k8s_vgpu_scheduler_amd.bench.membw --gib 20 --shared-only 8 --shared-bpc "$b" \
        --out "$out/membw8_b$b.json"
    done ;;
  serving)
    step 1100 serving python -u -m k8s_vgpu_scheduler_amd.bench.serving --configs "${1:-native,vgpu50,slice25,slice50}" \
      --warmup "${WARMUP:-30}" --runs "${RUNS:-200}" --max-tokens 128 --out-dir "$out" ;;
  mixed)
    # a governed server next to three governed decode tenants
    # (all 25 %, force), then 8 x 12 % temporal over 600 steps vs native
    step 900 serving python -u -m k8s_vgpu_scheduler_amd.bench.serving --configs temporal25,temporal25+3 \
      --warmup 10 --runs 60 --max-tokens 128 --out-dir "$out/serving"
    step 500 t8 python -u bench.py --slices 8 --rounds temporal,native --steps 600 --out "$out/t8.json" ;;
  board)
    # the share board (one occupancy sampler per GPU): 4 x 25 % temporal vs
    # native, unequal limits, 8 x 12.5 % temporal; then the SMI / RCCL tests
    # and the time-sharing e2e test
    step 400 t4 python -u bench.py --rounds temporal,native --steps 100 --out "$out/t4.json"
    step 300 alone python -u bench.py --slices 1 --mode shim --steps 300 --warmup 5 --out "$out/alone.json"
    step 400 u75 python -u bench.py --slices 2 --no-spatial --mode shim --policy force --slice-limits 75,25 \
      --steps 300 --warmup 5 --out "$out/u75_25.json"
    step 400 u50 python -u bench.py --slices 3 --no-spatial --mode shim --policy force --slice-limits 50,25,25 \
      --steps 300 --warmup 5 --out "$out/u50_25_25.json"
    step 400 t8 python -u bench.py --slices 8 --rounds temporal,native --steps 100 --out "$out/t8.json"
    step 200 smi python -u -m pytest tests/test_smi_gpu.py tests/test_rccl_gpu.py -v -s --timeout 120 \
      --timeout-method thread
    step 300 e2e python -u -m pytest tests/test_e2e_gpu.py -v -s --timeout 240 --timeout-method thread \
      -k "time_sharing or shimless" ;;
  fair)
    # the fair-share governor in the driver's own bench config (20 steps) and at 100 steps, 4 and 8 tenants
    step 300 t4_20 python -u bench.py --rounds temporal,native --steps 20 --warmup 5 --out "$out/t4_20.json"
    step 400 t4 python -u bench.py --rounds temporal,native --steps 100 --out "$out/t4.json"
    step 400 t8 python -u bench.py --slices 8 --rounds temporal,native --steps 100 --out "$out/t8.json"
    # 8 slices with the default layout (pooled whole-GPU range), driver-like 20 steps and 100
    step 400 s8_20 python -u bench.py --slices 8 --rounds shim,native --steps 20 --warmup 5 --out "$out/s8_20.json"
    step 400 s8 python -u bench.py --slices 8 --rounds shim,native --steps 100 --out "$out/s8.json" ;;
  fair2)
    # the fair-share governor: 4 / 8 symmetric tenants at 100 steps, unequal limits (75/25, 50/25/25)
    step 400 t4 python -u bench.py --rounds temporal,native --steps 100 --out "$out/t4.json"
    step 400 t8 python -u bench.py --slices 8 --rounds temporal,native --steps 100 --out "$out/t8.json"
    step 400 u75 python -u bench.py --slices 2 --no-spatial --mode shim --policy force --slice-limits 75,25 \
      --steps 300 --warmup 5 --out "$out/u75_25.json"
    step 400 u50 python -u bench.py --slices 3 --no-spatial --mode shim --policy force --slice-limits 50,25,25 \
      --steps 300 --warmup 5 --out "$out/u50_25_25.json" ;;
  eight)
    # 8 slices per GPU: disjoint 32-CU ranges vs the eight
    # pooled into one whole-GPU shared range (cuShareUnit 256) with and without
    # the node monitor's utilisation switch, 100 and 20 steps, vs native
    step 400 disjoint python -u bench.py --slices 8 --rounds shim,native --layout disjoint --steps 100 \
      --out "$out/disjoint.json"
    step 400 h256 python -u bench.py --slices 8 --rounds shim,native --layout hybrid --share-unit 256 --steps 100 \
      --out "$out/h256.json"
    step 400 h256_mon python -u bench.py --slices 8 --rounds shim,native --layout hybrid --share-unit 256 \
      --steps 100 --monitor 0.5 --out "$out/h256_mon.json"
    step 400 h256_20 python -u bench.py --slices 8 --rounds shim,native --layout hybrid --share-unit 256 \
      --steps 20 --warmup 5 --out "$out/h256_20.json" ;;
  kern)
    # prefill kernels: flash attention (eight-wave vs 32-key-tile kernel) and
    # the packed-weight GEMM (LDS-DMA ring v2 vs register-staged v1 vs unpack +
    # hipBLASLt), numerics then timing, then the 8k-token TTFT
    step 300 tests python -u -m pytest tests/test_ops_gpu.py -v --timeout 120 --timeout-method thread \
      -k "prefill_flash or tr_read or prefill_gemm"
    step 200 fa8 python -u -m k8s_vgpu_scheduler_amd.bench.prefill_attention --lens 512,2048,8192 --eager-max 0 \
      --out "$out/fa8.json"
    step 300 pgemm python -u -m k8s_vgpu_scheduler_amd.bench.prefill_gemm --rows 2048,8192 --out "$out/pgemm.json"
    MIVGPU_PREFILL_GEMM_V=1 step 300 pgemm_v1 python -u -m k8s_vgpu_scheduler_amd.bench.prefill_gemm --rows 8192 \
      --out "$out/pgemm_v1.json"
    # 8k-token TTFT (<= 120 ms): library GEMM path (default) and the native GEMM
    step 300 ttft8k python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 9216 --iters 5
    MIVGPU_PREFILL_GEMM=native step 300 ttft8k_native python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 \
      --ctx 9216 --iters 5 ;;
  pg2)
    # prefill GEMM v2 ring depth (4 / 5 slices) x wave priority over the MFMAs: numerics, then 8192 rows
    MIVGPU_PREFILL_GEMM_ST=5 MIVGPU_PREFILL_GEMM_PRIO=1 step 300 tests python -u -m pytest tests/test_ops_gpu.py -v \
      --timeout 120 --timeout-method thread -k "prefill_gemm"
    for st in 4 5; do for pr in 0 1; do
      MIVGPU_PREFILL_GEMM_ST=$st MIVGPU_PREFILL_GEMM_PRIO=$pr step 300 "pg_st${st}_p${pr}" python -u -m \
        k8s_vgpu_scheduler_amd.bench.prefill_gemm --rows 8192 --out "$out/pg_st${st}_p${pr}.json"
    done; done ;;
  pg3)
    # prefill GEMM v3 (ping-pong wave groups) vs v2: numerics, 2048 / 8192 rows, 8k-token TTFT on it
    step 300 tests python -u -m pytest tests/test_ops_gpu.py -v --timeout 120 --timeout-method thread -k "prefill_gemm"
    step 300 pg_v3 python -u -m k8s_vgpu_scheduler_amd.bench.prefill_gemm --rows 2048,8192 --out "$out/pg_v3.json"
    MIVGPU_PREFILL_GEMM_V=2 step 300 pg_v2 python -u -m k8s_vgpu_scheduler_amd.bench.prefill_gemm --rows 8192 \
      --out "$out/pg_v2.json"
    MIVGPU_PREFILL_GEMM=native step 300 ttft8k_native python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 \
      --ctx 9216 --iters 5
    step 300 ttft8k_lib python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 9216 --iters 5 ;;
  pg4)
    # prefill GEMM v4 (four waves, 128x128 each) vs v3: numerics, 8192 rows, TTFT on it
    MIVGPU_PREFILL_GEMM_V=4 step 300 tests python -u -m pytest tests/test_ops_gpu.py -v --timeout 120 \
      --timeout-method thread -k "prefill_gemm"
    MIVGPU_PREFILL_GEMM_V=4 step 300 pg_v4 python -u -m k8s_vgpu_scheduler_amd.bench.prefill_gemm --rows 2048,8192 \
      --out "$out/pg_v4.json"
    step 300 pg_v3 python -u -m k8s_vgpu_scheduler_amd.bench.prefill_gemm --rows 8192 --out "$out/pg_v3.json"
    MIVGPU_PREFILL_GEMM=native MIVGPU_PREFILL_GEMM_V=4 step 300 ttft8k_v4 python -u -m \
      k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 9216 --iters 5 ;;
  pgpmc)
    # counters of the prefill GEMM (v3) next to hipBLASLt's kernels on the same shapes (8192 rows)
    cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
    pg="python3 -m k8s_vgpu_scheduler_amd.bench.prefill_gemm --rows 8192 --reps 3"
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$out/p/a" -o run -- $pg \
      > "$out/a.log" 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 \
      SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d "$out/p/b" -o run -- $pg \
      > "$out/b.log" 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU \
      --kernel-trace --output-format csv -d "$out/p/c" -o run -- $pg > "$out/c.log" 2>&1 || exit 1
    python3 "$R/scripts/probe/pmc_summary.py" "$out/p" > "$out/pgemm_pmc.json" && rm -rf "$out/p" ;;
  prefill)
    step 120 native python3 -m k8s_vgpu_scheduler_amd.bench.prefill
    HSA_CU_MASK=0:0-63 step 120 cu64 python3 -m k8s_vgpu_scheduler_amd.bench.prefill
    cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
    step 200 prof rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
      python3 -m k8s_vgpu_scheduler_amd.bench.prefill --iters 10 ;;
  pf8k)
    # prefill numerics, 8k TTFT with / without the kept plain down weight, and where the
    # 8192-token prefill's time goes: per-kernel totals over 3 graph replays
    step 600 tests python -u -m pytest tests/test_serving_gpu.py tests/test_ops_gpu.py tests/test_prefill_canary_gpu.py \
      -v --timeout 120 --timeout-method thread -k "prefill or decoder or rope"
    step 300 ttft8k python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 9216 --iters 5
    MIVGPU_KEEP_PLAIN_DOWN=0 step 300 ttft8k_nodown python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 \
      --ctx 9216 --iters 5
    cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
    step 300 prof rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
      python3 -m k8s_vgpu_scheduler_amd.bench.prefill --len 8192 --ctx 9216 --iters 3 ;;
  *) echo "unknown suite $suite"; exit 2 ;;
esac
