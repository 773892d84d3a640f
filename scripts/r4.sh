#!/usr/bin/env bash
# Round-4 GPU runs: each step under its own time limit; a crash, timeout or
# abort (rc >= 2 and not a plain pytest failure) ends the run there.
#   bash scripts/r4.sh <outdir> <step>...   steps: flash, attnbench, shim, other, ttft, slices8, governor
set -o pipefail
out=${1:?outdir}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/$out"; cd "$R"
run() {  # run <seconds> <log> <cmd...>; pytest rc 1 (failures) keeps going
  local t=$1 log=$2; shift 2
  echo "[r4] $log: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$out/$log.log" 2>&1
  local rc=$?
  echo "[r4] $log rc=$rc"
  if [ $rc -ge 2 ]; then echo "[r4] stopping after $log (rc=$rc)"; exit $rc; fi
}
T="--timeout 300 --timeout-method thread"
for s in "$@"; do
  case $s in
    flash) run 400 flash_tests python -u -m pytest tests/test_ops_gpu.py -v -k "prefill_flash or long_prefill or tr_read" $T ;;
    shim2) run 700 shim2_tests python -u -m pytest tests/test_shim_gpu.py tests/test_shim_interpose_gpu.py -v -s $T \
             -k "unequal or tenant_without or tenant_rewriting" ;;
    attnbench) run 300 prefill_attn python -u -m k8s_vgpu_scheduler_amd.bench.prefill_attention \
                 --out "gpurun_out/$out/prefill_attn.json"
               MIVGPU_FA_TR=0 run 300 prefill_attn_tr0 python -u -m k8s_vgpu_scheduler_amd.bench.prefill_attention \
                 --out "gpurun_out/$out/prefill_attn_tr0.json" ;;
    shim) run 700 shim_tests python -u -m pytest tests/test_shim_gpu.py tests/test_shim_interpose_gpu.py -v -s $T ;;
    other) run 700 other_tests python -u -m pytest tests -m gpu -v $T --deselect tests/test_shim_gpu.py \
             --deselect tests/test_shim_interpose_gpu.py ;;
    allgpu) run 1000 gpu_tests python -u -m pytest tests -m gpu -v $T ;;
    ttft) for n in 512 2048 8000; do
            run 400 "ttft_$n" python -u -m k8s_vgpu_scheduler_amd.bench.prefill --len $n --ctx 8192 --iters 5
          done ;;
    chain) run 400 chain_tests python -u -m pytest tests/test_ops_gpu.py -v -k chain $T
           for b in 32 1; do
             for c in 0 1; do
               MIVGPU_CHAIN=$c run 200 "chain_b${b}_c$c" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch $b
             done
             MIVGPU_CHAIN=gd run 200 "chain_b${b}_gd" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch $b
             MIVGPU_CHAIN=1 MIVGPU_CHAIN_SC1=1 run 200 "chain_b${b}_sc1" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch $b
           done ;;
    hbm) # HBM read bytes over ALL TCC channels (FETCH_SIZE covered half of them):
         # the counter list, then one decode pass with the EA read-request counters summed over instances
         export TMPDIR=/tmp PYTHONPATH=$R
         timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/$out/counters.txt" 2>&1
         for cfg in full cu64; do
           if [ $cfg = cu64 ]; then export HSA_CU_MASK=0:0-63; else unset HSA_CU_MASK; fi
           run 150 "hbm_$cfg" rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --kernel-trace \
             --output-format csv -d "$R/gpurun_out/$out/hbm_$cfg" -o run -- \
             python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 3 --warmup 1 --no-graph
           python3 "$R/scripts/probe/pmc_summary.py" "$R/gpurun_out/$out/hbm_$cfg" > "$R/gpurun_out/$out/hbm_$cfg.json" \
             && rm -rf "$R/gpurun_out/$out/hbm_$cfg"
         done
         unset HSA_CU_MASK ;;
    chainprof) export TMPDIR=/tmp PYTHONPATH=$R
         for c in 0 1; do
           MIVGPU_CHAIN=$c run 200 "chainprof_c$c" rocprofv3 --kernel-trace --output-format csv \
             -d "$R/gpurun_out/$out/chainprof_c$c" -o run -- \
             python3 -m k8s_vgpu_scheduler_amd.bench.decode --batch 32 --steps 12 --warmup 2
           python3 scripts/probe/trace_step.py "$R/gpurun_out/$out/chainprof_c$c" --steps 8 --json \
             > "$R/gpurun_out/$out/chainprof_c$c.json" && rm -rf "$R/gpurun_out/$out/chainprof_c$c"
         done ;;
    prof) export TMPDIR=/tmp PYTHONPATH=$R
          for b in 32 1; do
            run 200 "prof_b$b" rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/$out/prof_b$b" -o run -- \
              python3 -m k8s_vgpu_scheduler_amd.bench.decode --batch $b --steps 12 --warmup 2
            python3 scripts/probe/trace_step.py "$R/gpurun_out/$out/prof_b$b" --steps 8 --json \
              > "$R/gpurun_out/$out/prof_b$b.json" && rm -rf "$R/gpurun_out/$out/prof_b$b"
          done ;;
    launch) run 400 launch_test python -u -m pytest tests/test_shim_gpu.py -v -s $T -k launch_overhead ;;
    interpose) run 600 interpose_tests python -u -m pytest tests/test_shim_interpose_gpu.py -v -s $T -k "triton or compile" ;;
    tenant) run 300 tenant_test python -u -m pytest tests/test_shim_interpose_gpu.py -v -s $T -k "tenant_" ;;
    govab) # share-estimator contention window A/B (build/variants/libmivgpu_pb<ms>.so)
         for w in ${GOVAB_WINDOWS:-10 50}; do
           MIVGPU_SHIM_PATH="$R/build/variants/libmivgpu_pb$w.so" run 300 "govab_s8_pb$w" \
             python -u bench.py --slices 8 --rounds temporal --out "gpurun_out/$out/govab_s8_pb$w.json"
           MIVGPU_SHIM_PATH="$R/build/variants/libmivgpu_pb$w.so" run 500 "govab_unequal_pb$w" \
             python -u -m pytest tests/test_shim_gpu.py -v -s $T -k "unequal or charged_the_share"
         done ;;
    serve) run 1100 serving python -u -m k8s_vgpu_scheduler_amd.bench.serving --configs native,vgpu50 \
             --warmup 30 --runs 200 --long-prompt-tokens 8000 --out-dir "gpurun_out/$out/serving" ;;
    s8) run 400 s8_auto python -u bench.py --slices 8 --out "gpurun_out/$out/s8_auto.json"
        run 400 s8_disjoint python -u bench.py --slices 8 --layout disjoint --rounds shim \
          --out "gpurun_out/$out/s8_disjoint.json" ;;
    combine) run 300 attn_tests python -u -m pytest tests/test_ops_gpu.py -v -k "attn or attention or decoder" $T
             for m in 1 2; do
               MIVGPU_ATTN_FUSED=$m run 200 "comb_m$m" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 32
             done ;;
    e2e) run 500 e2e_tests python -u -m pytest tests/test_e2e_gpu.py -v $T ;;
    s8plan) run 400 s8p_base python -u bench.py --slices 8 --layout disjoint --rounds shim \
              --out "gpurun_out/$out/s8p_base.json"
            run 400 s8p_chip python -u bench.py --slices 8 --layout disjoint --rounds shim \
              --child-env MIVGPU_SLICE_PLAN_CUS=0 --out "gpurun_out/$out/s8p_chip.json"
            run 400 s8p_q1 python -u bench.py --slices 8 --layout disjoint --rounds shim --hw-queues 1 \
              --out "gpurun_out/$out/s8p_q1.json" ;;
    s8pool) run 400 s8h128 python -u bench.py --slices 8 --layout hybrid --share-unit 128 --rounds shim --monitor 5 \
              --out "gpurun_out/$out/s8h128.json"
            run 400 s8h256 python -u bench.py --slices 8 --layout hybrid --share-unit 256 --rounds shim --monitor 5 \
              --out "gpurun_out/$out/s8h256.json" ;;
    s8gov) run 500 s8g_default python -u bench.py --slices 8 --no-spatial --rounds shim,native --monitor 1 --steps 300 \
             --out "gpurun_out/$out/s8g_default.json"
           run 500 s8g_burst python -u bench.py --slices 8 --rounds temporal --steps 300 \
             --child-env MIVGPU_GATE_BURST_US=200000 --out "gpurun_out/$out/s8g_burst.json" ;;
    plans2) for p in "" "1,1" "4,1"; do
              MIVGPU_GU_PLAN=$p run 200 "gu2_${p/,/_}" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 32
            done ;;
    plans3) for p in "" "1,2" "2,2" "1,8"; do
              MIVGPU_DOWN_PLAN=$p run 200 "d3_${p/,/_}" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 32
            done ;;
    kw8) run 300 kw8_tests python -u -m pytest tests/test_ops_gpu.py tests/test_skinny_gemm_gpu.py -v $T -k "widek or row_norm"
         for k in "" 8 "" 8; do
           MIVGPU_WIDEK_KW=$k run 200 "kw8_b32_$k" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 32
         done
         for k in "" 8; do
           MIVGPU_WIDEK_KW=$k run 200 "kw8_b1_$k" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 1
         done ;;
    s8queues) for q in 3 4; do
                run 500 "s8q$q" python -u bench.py --slices 8 --layout disjoint --rounds shim,native --hw-queues $q \
                  --out "gpurun_out/$out/s8q$q.json"
              done ;;
    l2) export TMPDIR=/tmp PYTHONPATH=$R
        for b in 32 1; do
          run 150 "l2_b$b" rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --kernel-trace \
            --output-format csv -d "$R/gpurun_out/$out/l2_b$b" -o run -- \
            python3 -m k8s_vgpu_scheduler_amd.bench.decode --batch $b --steps 3 --warmup 1 --no-graph
          python3 "$R/scripts/probe/pmc_summary.py" "$R/gpurun_out/$out/l2_b$b" > "$R/gpurun_out/$out/l2_b$b.json" \
            && rm -rf "$R/gpurun_out/$out/l2_b$b"
        done ;;
    dmax) run 300 dmax_tests env MIVGPU_WIDEK_DMAX=1 python -u -m pytest tests/test_ops_gpu.py tests/test_skinny_gemm_gpu.py -v $T -k "widek or row_norm or decoder"
          for d in 0 1 0 1; do
            MIVGPU_WIDEK_DMAX=$d run 200 "dmax_b32_$d" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 32
            grep -h ms_per_step "gpurun_out/$out/dmax_b32_$d.log" >> "gpurun_out/$out/dmax_summary.txt"
          done ;;
    s8temporal) run 400 s8t_exact python -u bench.py --slices 8 --rounds temporal,native \
              --out "gpurun_out/$out/s8t_exact.json" ;;
    unequal) run 500 unequal_tests python -u -m pytest tests/test_shim_gpu.py -v -s $T -k "unequal or charged_the_share" ;;
    lds) export TMPDIR=/tmp PYTHONPATH=$R
         run 150 lds_full rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 \
           --kernel-trace --output-format csv -d "$R/gpurun_out/$out/lds_full" -o run -- \
           python3 -m k8s_vgpu_scheduler_amd.bench.decode --steps 3 --warmup 1 --no-graph
         python3 "$R/scripts/probe/pmc_summary.py" "$R/gpurun_out/$out/lds_full" > "$R/gpurun_out/$out/lds_full.json" \
           && rm -rf "$R/gpurun_out/$out/lds_full" ;;
    plans) for p in "" "2,2" "2,4" "4,4"; do
             MIVGPU_GU_PLAN=$p run 200 "gu_${p/,/_}" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 32
           done
           for p in "2,8" "2,6" "4,4" "4,8" "1,4"; do
             MIVGPU_DOWN_PLAN=$p run 200 "down_${p/,/_}" python -u -m k8s_vgpu_scheduler_amd.bench.decode --batch 32
           done ;;
    bench) run 400 bench python -u bench.py --out "gpurun_out/$out/bench.json" ;;
    curve) for n in 1 2 8; do
             run 400 "bench_s$n" python -u bench.py --slices $n --out "gpurun_out/$out/s$n.json"
           done ;;
    smoke) run 200 smoke python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
