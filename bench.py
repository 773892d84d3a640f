#!/usr/bin/env python3
"""Headline benchmark: vGPU isolation overhead + aggregate throughput.

BASELINE.json metric "vGPU isolation overhead % + aggregate throughput, N pods
sharing 1 MI355X".  On every GPU (one torchrun rank per GPU) the bench runs
``--slices`` vGPU slices = separate processes, each a pod-equivalent with the
device plugin's environment (libmivgpu.so preloaded, HBM hard limit
``--gpumem-mib``, disjoint HSA_CU_MASK CU ranges = ``gpucores`` 100/slices %),
each decoding a Qwen3-8B-shaped model (random init, synthetic KV context) at
``--batch`` sequences.  The same slices are first run natively (no shim, no
limits, no masks, same GPU_MAX_HW_QUEUES): overhead = 1 - shim / native
aggregate tokens/s.  A third round runs natively with HIP's default 4 queues
per process (naive sharing, what N plain pods get without the device plugin).

``value`` = whole-job aggregate decode tokens/s of the shim round over all
GPUs and slices, timed over exactly ``--steps`` hipGraph-replayed decode steps
per slice between a barrier + torch.cuda.synchronize() on both sides (max
over ranks).  The reference publishes no number -> vs_baseline
is null; the native round is the comparison point.

    python bench.py --gpus 1 --steps 100 --warmup 10
    torchrun --nproc-per-node 8 bench.py --gpus 8 ...
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "vGPU isolation overhead % + aggregate throughput, N pods sharing 1 MI355X"


def physical_gpu_for(local_rank: int) -> str:
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            ids = [x for x in v.split(",") if x != ""]
            if local_rank < len(ids):
                return ids[local_rank]
    return str(local_rank)


def native_rccl_check(rank: int, world: int, local_rank: int, barrier) -> dict:
    """Run mivgpu-rccl-check on every rank (untimed, after the slices): the
    communicator id goes through a file named by the rendezvous port; rank 0's
    view is reported (exit code, rows, failures)."""
    import subprocess

    from k8s_vgpu_scheduler_amd.utils import build
    uid = f"/tmp/mivgpu-rccl-{os.environ.get('MASTER_PORT', '0')}.uid"
    if rank == 0 and os.path.exists(uid):
        os.unlink(uid)
    barrier()
    try:
        r = subprocess.run([str(build.RCCL_CHECK), "--rank", str(rank), "--nranks", str(world), "--device",
                            str(local_rank), "--uid", uid, "--sizes", "1048576,16777216,268435456", "--iters", "10",
                            "--warmup", "3"], capture_output=True, text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return {"rc": "timeout"}
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    rows = [x for x in lines if "op" in x]
    comm = next((x["comm"] for x in lines if "comm" in x), None)
    out = {"rc": r.returncode, "all_ok": r.returncode == 0 and bool(rows) and all(x["ok"] for x in rows),
           "comm": comm, "rows": [{k: x[k] for k in ("op", "bytes", "ms", "busbw_gbs", "ok")} for x in rows]}
    if r.returncode:
        out["stderr"] = r.stderr[-600:]
    return out


def gov_row(d: dict) -> dict:
    """One slice's governor row, every field over the TIMED window (VERDICT r5
    item 6: the instantaneous share sample disagreed with the integral):
    GPU-time share received (the share integral), held ms and gates, the
    sampler's fair-share samples and those held on the lead, and the share
    board's passes; plus the lifetime totals (load + warmup + timed)."""
    t = d.get("timed") or {}
    return {"busy_share_pct": d.get("busy_share_pct"), "received_gpu_ms": d.get("received_gpu_ms"),
            "held_ms": t.get("held_ms"), "gates": t.get("gates"), "fair_samples": t.get("fair_samples"),
            "fair_held_samples": t.get("fair_held_samples"), "samples": t.get("samples"),
            "board_passes": t.get("board_passes"), "board_fair_passes": t.get("board_fair_passes"),
            "seconds": d.get("seconds"), "sampler": d.get("sampler"),
            "lifetime": {"charged_ms": d.get("gov_charged_ms"), "held_ms": d.get("gov_held_ms"),
                         "gates": d.get("gov_gates")},
            "sampler_pass_us_mean": d.get("gov_sampler_pass_us_mean"),
            "sampler_pass_us_max": d.get("gov_sampler_pass_us_max"),
            "at_go": d.get("gov_at_go"), "at_end": d.get("gov_at_end"), "hold_trace": d.get("hold_trace"),
            "nonfair": d.get("gov_nonfair")}


def _share_cus(cus: int) -> int:
    from k8s_vgpu_scheduler_amd.device.amd.cu_alloc import CUTopology, share_unit
    from k8s_vgpu_scheduler_amd.device.amd.device import AMDConfig
    return share_unit(CUTopology(256, 8), cus or AMDConfig().cu_share_unit)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # Timed decode steps per slice.  Steps are cheap next to model load (one
    # step = one token per sequence, ~16 ms at 4 slices); 100 keeps a single
    # scheduling hiccup (seen once: ~190 ms on one of 8 slices) from
    # dominating the slowest slice's wall time.
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--slices", type=int, default=4, help="vGPU slices (pods) per GPU")
    ap.add_argument("--batch", type=int, default=32, help="decode sequences per slice")
    ap.add_argument("--ctx", type=int, default=1024, help="KV context length at decode start")
    ap.add_argument("--gpumem-mib", type=int, default=36864, help="HBM hard limit per slice")
    ap.add_argument("--model", default="qwen3-8b", choices=["qwen3-8b", "qwen3-tiny"])
    ap.add_argument("--layers", type=int, default=0,
                    help="decoder layers per slice (0 = the model's own 36); GPU tests use fewer to keep eight-slice "
                         "rounds short -- such a line is labelled and is not the headline config")
    ap.add_argument("--mode", default="all", choices=["all", "both", "shim", "native"],
                    help="all = shim + masked_noshim + temporal + native (same queues) + native (HIP default "
                         "queues) rounds; both = shim + native")
    ap.add_argument("--round-gap", type=float, default=0.0,
                    help="seconds to idle between rounds (the 8-slice second-round slowdown this was tried for "
                         "was the bench process owning GPU queues, profiles/README.md §27)")
    ap.add_argument("--rounds", default="",
                    help="explicit comma list of rounds to run, in this order (experiments): shim, masked_noshim, "
                         "temporal, native, native_hip_default")
    ap.add_argument("--no-spatial", action="store_true", help="no HSA_CU_MASK (temporal governor)")
    ap.add_argument("--layout", default="auto", choices=["auto", "hybrid", "disjoint"],
                    help="CU ranges of slices below a quarter GPU: shared ranges split by the governor "
                         "(hybrid) or disjoint ranges (auto = the allocator's default, cuShareSmall)")
    ap.add_argument("--share-unit", type=int, default=0, metavar="CUS",
                    help="CUs of one shared range in the hybrid layout (0 = the allocator's cuShareUnit: a quarter)")
    ap.add_argument("--active-slices", type=int, default=0,
                    help="run only the first K of the --slices planned slices (same masks/limits; 0 = all)")
    ap.add_argument("--monitor", type=float, default=5.0, metavar="SECONDS",
                    help="run the node monitor's feedback pass (priority + utilization_switch) over the shim "
                         "rounds' regions every SECONDS while they run, as production does (the reference's 5 s "
                         "feedback period, cmd/vGPUmonitor/feedback.go:143; 0 = off)")
    ap.add_argument("--policy", default="default", choices=["default", "force", "disable"])
    ap.add_argument("--board", default="auto", choices=["auto", "node", "shim", "off"],
                    help="owner of the GPU's share board in the shim rounds: the node sampler (mivgpu-boardd, "
                         "as the monitor runs it) or a governed slice's shim; auto = node on one GPU, shim with "
                         "several ranks (one node sampler per rank would read every GPU's processes); off = no "
                         "board at all (A/B of the sampler's cost)")
    ap.add_argument("--presence-window-us", type=int, default=-1,
                    help="share-board fair-share presence window (experiments; -1 = the owner's default)")
    ap.add_argument("--overhead-pairs", type=int, default=4,
                    help="shim / masked-no-shim round pairs for shim_overhead_pct, interleaved ABBA (the first "
                         "pair is the headline round and its bare twin; 1 = no extra rounds)")
    ap.add_argument("--unequal-limits", default="75,25",
                    help="core limits (%%) of the unequal temporal round (governor, policy force, no masks: the "
                         "round that must throttle); empty = skip")
    ap.add_argument("--slice-limits", default="",
                    help="comma list of per-slice core limits (%%) for the shim and temporal rounds, e.g. 75,25 "
                         "(unequal tenants; default 100/N each)")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    ap.add_argument("--hw-queues", type=int, default=2,
                    help="GPU_MAX_HW_QUEUES per slice in the shim round (0 = HIP default)")
    ap.add_argument("--child-env", action="append", default=[], metavar="K=V",
                    help="extra environment for every slice process (experiments)")
    ap.add_argument("--gov-steps", type=int, default=600,
                    help="decode steps of the two governor rounds (one unthrottled slice, then the same slice "
                         "held to --gov-limit %%): >= 2 s of GPU work whatever --steps is, so the 100 ms burst "
                         "is amortised (0 = skip)")
    ap.add_argument("--gov-limit", type=int, default=25, help="core limit (%%) of the governed round")
    ap.add_argument("--eager-steps", type=int, default=60,
                    help="decode steps of the two eager rounds (one batch-1 slice, every kernel launched from the "
                         "host, under libmivgpu.so and without it: the launch hook's cost on a launch-bound "
                         "tenant); 0 = skip")
    ap.add_argument("--no-collectives", action="store_true",
                    help="skip the untimed all-reduce check between the bench ranks (N > 1)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = rehearse the harness without a GPU: gloo barriers, CPU reference decoder in "
                         "the slice processes (results are not MI355X numbers)")
    args = ap.parse_args()

    from k8s_vgpu_scheduler_amd.bench.slices import pct_text, plan_slices, run_round, spawn_round
    from k8s_vgpu_scheduler_amd.utils import build

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if rank == 0 and not build.SHIM_SO.exists():
        build.build_all()
    phys = physical_gpu_for(local_rank)
    work = Path(tempfile.mkdtemp(prefix=f"mivgpu-bench-r{rank}-"))
    log_dir = Path(os.environ.get("MIVGPU_BENCH_LOGS", work))
    log_dir.mkdir(parents=True, exist_ok=True)
    child_args = ["--model", args.model, "--layers", str(args.layers), "--batch", str(args.batch), "--ctx", str(args.ctx),
                  "--steps", str(args.steps), "--warmup", str(args.warmup), "--device", args.device]
    cpu = args.device == "cpu"

    extra_env = dict(kv.split("=", 1) for kv in args.child_env)

    limits = [float(x) for x in args.slice_limits.split(",") if x.strip()]
    if limits and len(limits) != args.slices:
        ap.error(f"--slice-limits has {len(limits)} entries for {args.slices} slices")

    def with_env(specs):
        for sp in specs:
            if args.board == "off" and sp.shim:
                sp.env["MIVGPU_BOARD_DIR"] = "none"
            if args.presence_window_us >= 0 and sp.shim:
                sp.env["MIVGPU_PRESENCE_WINDOW_US"] = str(args.presence_window_us)
            sp.env.update(extra_env)
        return specs[:args.active_slices] if args.active_slices > 0 else specs

    def with_limits(specs):
        if limits and len(specs) == len(limits):
            for sp, lim in zip(specs, limits):
                sp.core_pct = lim
        return specs

    def native_specs(queues):
        specs = plan_slices(args.slices, shim=False, gpumem_mib=None)
        for sp in specs:
            if queues and args.slices > 1:
                sp.env["GPU_MAX_HW_QUEUES"] = str(queues)
        return with_env(specs)

    # Spawn every slice process of every round BEFORE this process touches HIP.
    # "native" uses the same HW-queue count as the shim round, so the overhead
    # isolates the cost of the vGPU layer itself (shim + CU masks + limits);
    # "native_hip_default" is naive sharing with HIP's default queue count.
    # Round order: the headline (shim) first, the naive-sharing round last.  A
    # round that oversubscribes the hardware queues (8 slices x HIP's default 4
    # queues) was seen to leave the next round on the GPU unfair (one 8-slice
    # shim round behind it: fairness 0.51, 6.3k tok/s; alone: 0.99, 8.2k).
    wanted = [r for r in args.rounds.split(",") if r]
    if not wanted:
        wanted = {"all": ["shim", "masked_noshim", "temporal", "native", "native_hip_default"],
                  "both": ["shim", "native"], "shim": ["shim"], "native": ["native"]}[args.mode]
        if args.slices <= 1 or args.no_spatial:
            wanted = [r for r in wanted if r not in ("masked_noshim", "temporal")]
        if args.slices <= 1 or not args.hw_queues:
            wanted = [r for r in wanted if r != "native_hip_default"]
    # The governor must HOLD in the driver-timed bench:
    # four symmetric 25 % tenants get 25 % each without it, so two extra
    # rounds time one slice alone on the whole GPU, unthrottled and then held
    # to --gov-limit % (policy force, no CU mask), over --gov-steps steps.
    if args.gov_steps > 0 and args.mode == "all" and not args.rounds and not cpu:
        wanted += ["governed_ref", "governed"]
    if args.eager_steps > 0 and args.mode == "all" and not args.rounds and not cpu:
        wanted += ["eager_shim", "eager_noshim"]
    # a temporal round that must throttle: unequal limits
    unequal = [float(x) for x in args.unequal_limits.split(",") if x.strip()]
    if unequal and args.mode == "all" and not args.rounds and not cpu and args.slices > 1:
        wanted += ["temporal_unequal"]
    # extra shim / masked-no-shim pairs, interleaved ABBA after everything else
    # (one 0.28 s sample must not swing the shim's cost)
    pairs = []
    if "shim" in wanted and "masked_noshim" in wanted and args.overhead_pairs > 1:
        for k in range(1, args.overhead_pairs):
            pair = [f"masked_noshim#{k}", f"shim#{k}"] if k % 2 else [f"shim#{k}", f"masked_noshim#{k}"]
            pairs.append(pair)
            wanted += pair
    gov_args = list(child_args)
    gov_args[gov_args.index("--steps") + 1] = str(max(args.gov_steps, args.steps))
    rounds = []
    if "governed_ref" in wanted:
        rounds.append(("governed_ref", spawn_round(
            with_env(plan_slices(1, shim=True, gpumem_mib=args.gpumem_mib, spatial=False)),
            phys, work / "gref", log_dir, gov_args, "governed_ref")))
    if "governed" in wanted:
        gspec = plan_slices(1, shim=True, gpumem_mib=args.gpumem_mib, spatial=False, policy="force")
        gspec[0].core_pct = args.gov_limit
        rounds.append(("governed", spawn_round(with_env(gspec), phys, work / "gov", log_dir, gov_args,
                                               "governed")))
    def shim_specs():
        return with_env(with_limits(plan_slices(args.slices, shim=True, gpumem_mib=args.gpumem_mib,
                                                spatial=not args.no_spatial, policy=args.policy,
                                                hw_queues=args.hw_queues or None, layout=args.layout,
                                                share_unit=args.share_unit)))

    def bare_specs():
        # the same CU masks and queues without libmivgpu.so: what the shim
        # itself costs (the overhead vs native also contains the
        # partitioning's own benefit)
        bare = plan_slices(args.slices, shim=True, gpumem_mib=None, hw_queues=args.hw_queues or None,
                           layout=args.layout, share_unit=args.share_unit)
        for sp in bare:
            sp.shim = False
        return with_env(bare)

    for nm in wanted:
        base = nm.split("#")[0]
        sub = nm.replace("#", "_")
        if base == "shim":
            rounds.append((nm, spawn_round(shim_specs(), phys, work if nm == "shim" else work / sub, log_dir,
                                           child_args, sub)))
        elif base == "masked_noshim":
            rounds.append((nm, spawn_round(bare_specs(), phys, work / ("bare" if nm == base else sub), log_dir,
                                           child_args, sub)))
    if "temporal" in wanted:
        # the same slices time-shared by the governor gate instead of CU masks
        # (BASELINE config 3: "4 pods x 25% gpucores, CU-throttle governor kernel")
        rounds.append(("temporal", spawn_round(
            with_env(with_limits(plan_slices(args.slices, shim=True, gpumem_mib=args.gpumem_mib, spatial=False,
                                             policy="force", hw_queues=args.hw_queues or None))),
            phys, work / "temporal", log_dir, child_args, "temporal")))
    if "temporal_unequal" in wanted:
        # unequal tenants time-shared by the governor: must throttle (each held
        # to its limit's share of the GPU, not an equal split)
        uspecs = plan_slices(len(unequal), shim=True, gpumem_mib=args.gpumem_mib, spatial=False, policy="force",
                             hw_queues=args.hw_queues or None)
        for sp, lim in zip(uspecs, unequal):
            sp.core_pct = lim
        # the governor rounds' step count (>= 2 s of GPU work): a 20-step
        # window is mostly the buckets' initial burst
        rounds.append(("temporal_unequal", spawn_round(with_env(uspecs), phys, work / "unequal", log_dir,
                                                       gov_args, "temporal_unequal")))
    if "native" in wanted:
        rounds.append(("native", spawn_round(native_specs(args.hw_queues), phys, work, log_dir, child_args,
                                             "native")))
    if "native_hip_default" in wanted:
        rounds.append(("native_hip_default", spawn_round(native_specs(0), phys, work, log_dir, child_args,
                                                         "native_hip_default")))
    eager_args = list(child_args)
    eager_args[eager_args.index("--steps") + 1] = str(args.eager_steps)
    eager_args[eager_args.index("--batch") + 1] = "1"
    eager_args.append("--eager")
    for nm, with_shim in (("eager_shim", True), ("eager_noshim", False)):
        if nm in wanted:
            sp = plan_slices(1, shim=True, gpumem_mib=args.gpumem_mib, spatial=False)
            sp[0].shim = with_shim
            sp[0].gpumem_mib = args.gpumem_mib if with_shim else None
            rounds.append((nm, spawn_round(with_env(sp), phys, work / nm, log_dir, eager_args, nm)))
    order = {name: i for i, name in enumerate(wanted)}
    rounds.sort(key=lambda r: order[r[0]])

    import torch
    import torch.distributed as dist

    # The bench process itself must hold no hardware queues while the slices
    # run: a GPU tensor or an RCCL barrier gives it two, and at 8 slices the
    # ninth queue-owning process on the GPU pushed the round after the first
    # into hardware-scheduler oversubscription (half the slices at half speed,
    # fairness 0.49; parent_queues probe, profiles/README.md §27).  So the
    # harness talks over gloo with CPU tensors; RCCL is only used after the
    # timed rounds, for the collective check (cuda tensors -> nccl).
    if world > 1:
        if cpu:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local_rank)
            dist.init_process_group("cpu:gloo,cuda:nccl")

        def barrier():
            dist.all_reduce(torch.zeros(1))       # CPU tensor: gloo
    else:
        if not cpu:
            torch.cuda.set_device(0)
        barrier = None

    def sync():
        if not cpu:
            torch.cuda.synchronize()

    gap = args.round_gap
    results = {}
    for i, (name, procs) in enumerate(rounds):
        if i and gap > 0 and not cpu:
            time.sleep(gap)
        mon = None
        if args.monitor > 0 and name.split("#")[0] in ("shim", "temporal", "temporal_unequal"):
            from k8s_vgpu_scheduler_amd.bench.slices import RoundMonitor
            mon = RoundMonitor([p.cache for p in procs], args.monitor).start()
        # the GPU's share board owned by the node sampler, as the monitor runs
        # it in production (--board shim: a governed slice takes the role)
        boardd = None
        bdir = next((p.board_dir for p in procs if getattr(p, "board_dir", None)), None)
        if (args.board == "node" or (args.board == "auto" and world == 1)) and bdir and bdir != "none" and not cpu:
            from k8s_vgpu_scheduler_amd.monitor.board import BoardSampler
            boardd = BoardSampler(bdir, extra_args=(["--presence-window-us", str(args.presence_window_us)]
                                                    if args.presence_window_us >= 0 else [])).start()
        try:
            # with the monitor: one pass once every slice is READY, then a few
            # untimed steps, so the timed window sees the switch as production
            # keeps it (on while several tenants are busy)
            # (ten steps at least: the switch engages every tenant's governor at
            # once, and the first ~100-150 ms -- the node sampler leaving its
            # dormant period, the fair-share mode establishing -- are the
            # buckets' transient; production keeps the switch on between its
            # 5 s passes, so the timed window measures the steady state)
            r = run_round(procs, barrier=barrier, sync=sync, before_go=mon.pass_now if mon else None,
                          rewarm=max(10, args.warmup) if mon else 0)
        finally:
            if boardd is not None:
                boardd.stop()
        r["specs"] = [p.spec for p in procs]
        if mon is not None:
            r["monitor"] = mon.stop()
        r["local_tokens"] = float(r["tokens"])
        wall = torch.tensor([r["wall_s"]], dtype=torch.float64)        # CPU: no queues in this process
        toks = torch.tensor([float(r["tokens"])], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(wall, op=dist.ReduceOp.MAX)
            dist.all_reduce(toks, op=dist.ReduceOp.SUM)
        r["max_wall_s"] = wall.item()
        r["total_tokens"] = toks.item()
        r["tok_s"] = toks.item() / wall.item()
        results[name] = r

    # N > 1: after the timed rounds (slice processes gone), an untimed RCCL
    # all-reduce between the ranks: exact result + busBW over xGMI, the data
    # plane a multi-GPU pod placed by the topology score runs on
    # (parallel/collectives.py).  Reported next to the headline, never in it.
    coll = None
    if world > 1 and not args.no_collectives:
        from k8s_vgpu_scheduler_amd.parallel.collectives import measure
        from k8s_vgpu_scheduler_amd.parallel.dist import DistEnv
        env = DistEnv(rank, world, local_rank, "gloo" if cpu else "nccl",
                      torch.device("cpu" if cpu else f"cuda:{local_rank}"))
        sizes = (64 << 10, 1 << 20) if cpu else (1 << 20, 16 << 20, 256 << 20)
        coll = [measure("all_reduce", nb, env, iters=10, warmup=3) for nb in sizes]
    # ... and the native validator (csrc/bench/rccl_check.cpp): all-reduce,
    # all-gather and reduce-scatter through librccl directly, every element
    # checked, one child process per rank on this rank's GPU
    rccl_native = None
    if world > 1 and not args.no_collectives and not cpu and build.RCCL_CHECK.exists():
        rccl_native = native_rccl_check(rank, world, local_rank, barrier)
    # every rank's own view, so an N-GPU record reads from one line: its GPU,
    # its slices' tokens/s and wall time in the headline round, and what its
    # RCCL validator measured and saw
    per_rank = None
    if world > 1:
        hname = "shim" if "shim" in results else ("native" if "native" in results else next(iter(results)))
        mine = {"rank": rank, "local_rank": local_rank, "gpu": phys, "host": os.uname().nodename,
                "tok_s": round(results[hname]["local_tokens"] / results[hname]["wall_s"], 2),
                "wall_s": round(results[hname]["wall_s"], 4),
                "per_slice_tok_s": [round(d["tok_s"], 1) for d in results[hname]["done"]],
                "rccl": rccl_native}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)

    if rank == 0:
        head = results.get("shim") or results.get("native") or next(iter(results.values()))
        per_slice = [round(d["tok_s"], 1) for d in head["done"]]
        out = {
            "metric": METRIC,
            "value": round(head["tok_s"], 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(head["max_wall_s"] / args.steps * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if not cpu else "fp32-reference (CPU rehearsal)",
            "data": "synthetic (random-init weights, random KV context)",
            "config": {
                "model": ("Qwen3-8B" if args.model == "qwen3-8b" else "Qwen3-tiny")
                + (f" ({args.layers} layers, test config)" if args.layers > 0 else ""),
                "global_batch": world * args.slices * args.batch,
                "seq_len": args.ctx,
                "parallelism": f"dp{world} x {args.slices} vGPU slices/GPU",
                "slices_per_gpu": args.slices,
                "batch_per_slice": args.batch,
                "gpumem_mib_per_slice": args.gpumem_mib,
                "gpucores_per_slice": limits or (100 // args.slices if args.slices > 1 else 100),
                # the grant's HIP_DEVICE_CORE_LIMIT: the CUs charged, as an exact share
                "core_limit_pct_per_slice": [pct_text(sp.core_pct) for sp in head.get("specs", [])],
                "isolation": (f"HSA_CU_MASK ({args.layout} layout"
                              + (f", {_share_cus(args.share_unit)}-CU shared ranges" if args.layout == "hybrid" else "")
                              + ") + libmivgpu" if not args.no_spatial
                              else f"governor ({args.policy})")
                + (f" + {args.hw_queues} HW queue/slice" if args.hw_queues and args.slices > 1 else ""),
            },
            "round": "shim" if "shim" in results else ("native" if "native" in results else next(iter(results))),
            "per_slice_tok_s_rank0": per_slice,
            "slice_fairness_min_over_max": round(min(per_slice) / max(per_slice), 3) if per_slice else None,
            "slice_mem_total_mib": [rd["mem_total_mib"] for rd in head["ready"]],
            "slice_runtime_vram_charged_mib": [rd.get("context_mib") for rd in head["ready"]],
            "tpot_ms_p50_rank0": [round(d.get("tpot_ms_p50", 0), 3) for d in head["done"]],
            "tpot_ms_p99_rank0": [round(d.get("tpot_ms_p99", 0), 3) for d in head["done"]],
        }
        if any("gov_gates" in d or "busy_share_pct" in d for d in head["done"]):
            out["governor_rank0"] = [gov_row(d) for d in head["done"]]
        if "native" in results:
            out["native_value"] = round(results["native"]["tok_s"], 2)
        if "native" in results and "shim" in results:
            nat = results["native"]["tok_s"]
            out["isolation_overhead_pct"] = round((1.0 - head["tok_s"] / nat) * 100.0, 2)
            nd = results["native"]["done"]
            out["native_tpot_ms_p50_rank0"] = [round(d.get("tpot_ms_p50", 0), 3) for d in nd]
        if "masked_noshim" in results and "shim" in results:
            bare = results["masked_noshim"]["tok_s"]
            out["masked_noshim_value"] = round(bare, 2)
            # every interleaved pair (the headline round and its bare twin first)
            prs = [("shim", "masked_noshim")] + [(f"shim#{k}", f"masked_noshim#{k}")
                                                 for k in range(1, args.overhead_pairs)]
            prs = [(a, b) for a, b in prs if a in results and b in results]
            per = [round((1.0 - results[a]["tok_s"] / results[b]["tok_s"]) * 100.0, 2) for a, b in prs]
            ssum = sum(results[a]["tok_s"] for a, _ in prs)
            bsum = sum(results[b]["tok_s"] for _, b in prs)
            out["shim_overhead_pct"] = round((1.0 - ssum / bsum) * 100.0, 2)
            out["shim_overhead"] = {
                "what": "1 - shim / masked-no-shim aggregate tok/s, pooled over interleaved ABBA pairs",
                "pairs": len(prs), "per_pair_pct": per,
                "spread_pct": [min(per), max(per)] if per else None,
                "shim_tok_s": [round(results[a]["tok_s"], 1) for a, _ in prs],
                "masked_noshim_tok_s": [round(results[b]["tok_s"], 1) for _, b in prs],
                "headline_pair_pct": per[0] if per else None,
                "board": args.board, "monitor_period_s": args.monitor}
        if "temporal" in results:
            tr = results["temporal"]
            tps = [round(d["tok_s"], 1) for d in tr["done"]]
            out["temporal_value"] = round(tr["tok_s"], 2)
            out["temporal_per_slice_tok_s_rank0"] = tps
            out["temporal_fairness_min_over_max"] = round(min(tps) / max(tps), 3) if tps else None
            lims = sorted({pct_text(sp.core_pct) for sp in tr.get("specs", [])}) or ["?"]
            out["temporal_isolation"] = f"governor gate (force, {'/'.join(lims)} % each, occupancy-charged)"
            out["temporal_governor_rank0"] = [gov_row(d) for d in tr["done"]]
            if "native" in results:
                out["temporal_overhead_pct"] = round((1.0 - tr["tok_s"] / results["native"]["tok_s"]) * 100.0, 2)
        if "temporal_unequal" in results:
            tu = results["temporal_unequal"]
            tps = [d["tok_s"] for d in tu["done"]]
            lims = [sp.core_pct for sp in tu.get("specs", [])]
            out["temporal_unequal"] = {
                "what": "governor gate, policy force, no CU masks, unequal core limits: must throttle",
                "steps": max(args.gov_steps, args.steps),
                "limits_pct": [pct_text(x) for x in lims],
                "aggregate_tok_s": round(tu["tok_s"], 1),
                "per_slice_tok_s": [round(x, 1) for x in tps],
                "share_of_aggregate_pct": [round(100.0 * x / sum(tps), 1) for x in tps] if tps else None,
                "gpu_share_pct": [d.get("busy_share_pct") for d in tu["done"]],
                "held_ms": [(d.get("timed") or {}).get("held_ms") for d in tu["done"]],
                "governor_rank0": [gov_row(d) for d in tu["done"]]}
        if "eager_shim" in results and "eager_noshim" in results:
            es, en = results["eager_shim"], results["eager_noshim"]
            out["eager_launch_bound"] = {
                "what": "1 slice, batch 1, no hipGraph (every kernel launched from the host)",
                "steps": args.eager_steps, "shim_tok_s": round(es["tok_s"], 2),
                "noshim_tok_s": round(en["tok_s"], 2),
                "shim_overhead_pct": round((1.0 - es["tok_s"] / en["tok_s"]) * 100.0, 2),
                "ms_per_step_shim": round(es["max_wall_s"] / args.eager_steps * 1e3, 3),
                "ms_per_step_noshim": round(en["max_wall_s"] / args.eager_steps * 1e3, 3)}
        for nm in ("shim", "temporal", "temporal_unequal"):
            if nm in results and "monitor" in results[nm]:
                out[f"{nm}_monitor"] = results[nm]["monitor"]
        if "governed" in results and "governed_ref" in results:
            g, ref = results["governed"], results["governed_ref"]
            gd = g["done"][0]
            out["governor_enforcement"] = {
                "limit_pct": args.gov_limit, "policy": "force", "steps": max(args.gov_steps, args.steps),
                "unthrottled_tok_s": round(ref["tok_s"], 1), "governed_tok_s": round(g["tok_s"], 1),
                "fraction_of_unthrottled": round(g["tok_s"] / ref["tok_s"], 4),
                "unthrottled_gpu_s": round(ref["max_wall_s"], 3), "governed_wall_s": round(g["max_wall_s"], 3),
                "held_ms": gd.get("gov_held_ms"), "gates": gd.get("gov_gates"),
                "busy_share_pct": gd.get("busy_share_pct"), "received_gpu_ms": gd.get("received_gpu_ms")}
        if "native_hip_default" in results:
            nd = results["native_hip_default"]["tok_s"]
            out["native_hip_default_queues_value"] = round(nd, 2)
            out["speedup_vs_naive_sharing"] = round(head["tok_s"] / nd, 3)
        if coll:
            out["allreduce_between_gpus"] = [{k: r[k] for k in ("bytes", "us", "busbw_gbps", "correct")}
                                              for r in coll]
            out["allreduce_peak_busbw_gbps"] = max(r["busbw_gbps"] for r in coll)
        if rccl_native is not None:
            out["rccl_native_check"] = rccl_native
        if per_rank is not None:
            out["per_rank"] = per_rank
            out["rccl_ranks_seen"] = sorted({(pr.get("rccl") or {}).get("comm", {}).get("nranks", -1)
                                             for pr in per_rank if pr})
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            Path(args.out).parent.mkdir(parents=True, exist_ok=True)
            Path(args.out).write_text(line + "\n")
    if world > 1:
        barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
