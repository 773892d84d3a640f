"""N vGPU slices sharing one MI355X: the isolation-overhead benchmark engine.

BASELINE.json metric: "vGPU isolation overhead % + aggregate throughput, N
pods sharing 1 MI355X".  Each slice is a separate process (one pod's
container), started with exactly the environment the device plugin's
``Allocate`` would inject (``deviceplugin.allocate.container_env``):
``LD_PRELOAD=libmivgpu.so``, ``HIP_DEVICE_MEMORY_LIMIT_0``, ``HSA_CU_MASK``,
``HIP_DEVICE_CORE_LIMIT`` ... and runs the Qwen3-8B-shaped decode workload.
The native round runs the same processes with no shim, no mask, no limit.

Protocol (stdin/stdout lines, JSON payloads):
    parent -> child  LOAD            child builds model, captures graph, warms up
    child  -> parent READY {...}
    parent -> child  GO              child times `steps` graph replays
    child  -> parent DONE {...}
Children are spawned before the parent initialises HIP (fork/exec after GPU
init is forbidden on the box), and block on LOAD without touching the GPU.
"""

from __future__ import annotations

import argparse
import json
import os
import select
import subprocess
import sys
import time
from dataclasses import dataclass, field
from pathlib import Path

from k8s_vgpu_scheduler_amd.deviceplugin.allocate import core_limit_text
from k8s_vgpu_scheduler_amd.shim import shim_env

MI355X_CUS = 256
MI355X_XCDS = 8


@dataclass
class SliceSpec:
    index: int
    gpumem_mib: int | None      # None = no limit
    cu_ranges: list | None      # [(lo, hi), ...] for HSA_CU_MASK, None = all CUs
    core_pct: float = 100   # the grant's HIP_DEVICE_CORE_LIMIT (exact share of the CUs charged)
    shim: bool = True
    policy: str = "default"
    # HW queues per slice process (GPU_MAX_HW_QUEUES).  HIP's default of 4 per
    # process oversubscribes the hardware scheduler once several tenants share
    # a GPU (measured: 4 slices 4.5k -> 7.6k tok/s with 2 queues each, see
    # profiles/README.md §2); the device plugin injects the same value.
    hw_queues: int | None = None
    env: dict = field(default_factory=dict)


def pct_text(pct: float) -> str:
    """A core limit as the device plugin writes it (up to three decimals)."""
    return f"{pct:.3f}".rstrip("0").rstrip(".")


def cu_mask_string(ranges) -> str:
    return ",".join(f"{a}-{b}" if b > a else f"{a}" for a, b in ranges)


def plan_slices(n: int, shim: bool, gpumem_mib: int | None, spatial: bool = True,
                policy: str = "default", hw_queues: int | None = 2, layout: str = "auto",
                share_unit: int = MI355X_CUS // 4) -> list[SliceSpec]:
    """Equal split of one GPU into n slices (CUs in contiguous, XCD-sized runs).

    ``layout`` = what the scheduler's CU allocator hands out
    (device/amd/cu_alloc.py): ``disjoint`` = a range of its own per slice;
    ``hybrid`` = slices below a quarter of the GPU share ranges of
    ``share_unit`` CUs (as many as fit), split among them by the governor; ``auto`` =
    the allocator's default (``cuShareSmall``, on: shared ranges of
    ``cuShareUnit`` CUs, the whole GPU by default)."""
    specs = []
    per = (MI355X_CUS // n) // MI355X_XCDS * MI355X_XCDS   # whole 8-CU granules: XCD-balanced
    from k8s_vgpu_scheduler_amd.device.amd.cu_alloc import CUTopology
    from k8s_vgpu_scheduler_amd.device.amd.cu_alloc import share_unit as _unit
    from k8s_vgpu_scheduler_amd.device.amd.device import AMDConfig
    # 0: the allocator's shared-range size (cuShareUnit, a quarter by default)
    unit = _unit(CUTopology(MI355X_CUS, MI355X_XCDS), share_unit or AMDConfig().cu_share_unit)
    hybrid = layout == "hybrid" or (layout == "auto" and AMDConfig().cu_share_small)
    if layout == "auto" and not AMDConfig().cu_partition:
        spatial = False   # the allocator's time-sharing mode: no CU ranges at all
    quarter = _unit(CUTopology(MI355X_CUS, MI355X_XCDS))
    share = unit // per if (hybrid and 0 < per < quarter and per < unit) else 1
    for i in range(n):
        if share > 1:
            q = i // share
            ranges = [(q * unit, (q + 1) * unit - 1)] if (shim and spatial and n > 1) else None
        else:
            ranges = [(i * per, (i + 1) * per - 1)] if (shim and spatial and n > 1) else None
        # gpucores 100 // n, charged as whole granules (device/amd/device.py):
        # the grant states that charge exactly (deviceplugin/allocate.py)
        specs.append(SliceSpec(index=i, gpumem_mib=gpumem_mib if shim else None, cu_ranges=ranges,
                               core_pct=float(core_limit_text(per, MI355X_CUS)) if n > 1 else 100, shim=shim,
                               policy=policy, hw_queues=hw_queues if (shim and n > 1) else None))
    return specs


def slice_env(spec: SliceSpec, physical_gpu: str | None, cache_dir: Path) -> dict:
    env = {}
    if physical_gpu is not None:
        env["ROCR_VISIBLE_DEVICES"] = physical_gpu
        env.pop("HIP_VISIBLE_DEVICES", None)
    if spec.shim:
        env.update(shim_env(""))
        env["MIVGPU_SHARED_CACHE"] = str(cache_dir / f"slice{spec.index}.cache")
        # the GPU's share board (one sampler for every slice): writable, so a
        # governed slice holds the owner role as on a node without a monitor
        env["MIVGPU_BOARD_DIR"] = str(cache_dir / "board")
        if spec.gpumem_mib:
            env["HIP_DEVICE_MEMORY_LIMIT_0"] = f"{spec.gpumem_mib}m"
        if spec.core_pct < 100:
            env["HIP_DEVICE_CORE_LIMIT"] = pct_text(spec.core_pct)
        env["GPU_CORE_UTILIZATION_POLICY"] = spec.policy
    # the partition and queue count are properties of the slice, with or
    # without the shim (the "masked, no shim" round isolates the shim's cost)
    if spec.cu_ranges:
        env["HSA_CU_MASK"] = "0:" + cu_mask_string(spec.cu_ranges)
    if spec.hw_queues:
        env["GPU_MAX_HW_QUEUES"] = str(spec.hw_queues)
    env.update(spec.env)
    if spec.shim:
        # as in a pod: the grant also goes to a read-only file the shim takes it
        # from (deviceplugin/allocate.py; MIVGPU_LIMITS_FILE stands in for the
        # /etc/mivgpu/limits.conf mount)
        from k8s_vgpu_scheduler_amd.deviceplugin.allocate import grant_text
        grant = cache_dir / f"slice{spec.index}.grant"
        grant.write_text(grant_text(env))
        env["MIVGPU_LIMITS_FILE"] = str(grant)
    return env


class RoundMonitor:
    """The node monitor's feedback pass (monitor/feedback.py observe: priority
    blocking + utilization_switch) over a round's slice regions, every
    ``period`` s on a thread -- the production loop runs every 5 s over the
    regions of all containers on the node."""

    class _C:
        def __init__(self, region):
            self.region = region

    def __init__(self, caches: list, period: float):
        import threading
        self.caches, self.period = [c for c in caches if c], period
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, name="round-monitor", daemon=True)
        self._mu = threading.Lock()
        self._regions = {}
        self.passes = 0
        self.switch_seen = 0

    def start(self):
        self._th.start()
        return self

    def _run(self):
        while not self._stop.wait(self.period):
            self.pass_now()

    def pass_now(self):
        """One feedback pass now (the harness runs it once every slice is
        READY, so the switch is engaged before the timed window -- in
        production it stays on between the 5 s passes)."""
        from k8s_vgpu_scheduler_amd.monitor.feedback import observe
        from k8s_vgpu_scheduler_amd.monitor.region import SharedRegion
        with self._mu:
            for c in self.caches:
                if c not in self._regions and os.path.exists(c):
                    try:
                        self._regions[c] = SharedRegion(c)
                    except (OSError, ValueError):
                        pass
            cs = [self._C(r) for r in self._regions.values()]
            observe(type("L", (), {"list_containers": lambda _self: cs})())
            self.passes += 1
            self.switch_seen += sum(1 for x in cs if x.region.utilization_switch() == 1)

    def stop(self) -> dict:
        self._stop.set()
        self._th.join(timeout=10)
        with self._mu:
            for r in self._regions.values():
                r.close()
            self._regions = {}
        return {"period_s": self.period, "passes": self.passes, "switch_on_slice_passes": self.switch_seen}


class SliceProc:
    def __init__(self, spec: SliceSpec, env: dict, args: list, log_path: Path):
        full = dict(os.environ)
        for k in ("LD_PRELOAD", "HSA_CU_MASK", "HIP_DEVICE_CORE_LIMIT"):
            full.pop(k, None)
        full.update(env)
        # the child runs `-m k8s_vgpu_scheduler_amd...`: importable from any cwd
        root = str(Path(__file__).resolve().parents[2])
        full["PYTHONPATH"] = root + (os.pathsep + full["PYTHONPATH"] if full.get("PYTHONPATH") else "")
        if env.get("ROCR_VISIBLE_DEVICES") is not None:
            full.pop("HIP_VISIBLE_DEVICES", None)
            full.pop("CUDA_VISIBLE_DEVICES", None)
        self.spec = spec
        self.cache = env.get("MIVGPU_SHARED_CACHE")
        self.board_dir = env.get("MIVGPU_BOARD_DIR")
        self.log = open(log_path, "w")
        self.p = subprocess.Popen(
            [sys.executable, "-m", "k8s_vgpu_scheduler_amd.bench.slices", "--child", *args],
            env=full, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=self.log, text=True,
            bufsize=1)

    def send(self, line: str):
        self.p.stdin.write(line + "\n")
        self.p.stdin.flush()

    def expect(self, tag: str, timeout: float) -> dict:
        deadline = time.time() + timeout
        while True:
            left = deadline - time.time()
            if left <= 0:
                raise TimeoutError(f"slice {self.spec.index}: no {tag} within {timeout}s")
            r, _, _ = select.select([self.p.stdout], [], [], left)
            if not r:
                continue
            line = self.p.stdout.readline()
            if not line:
                try:
                    self.p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    pass
                self.log.flush()
                try:   # the slice's own error output, so a remote run shows it
                    tail = Path(self.log.name).read_text(errors="replace")[-3000:]
                except OSError:
                    tail = ""
                raise RuntimeError(f"slice {self.spec.index} exited (rc={self.p.poll()}) before {tag}; "
                                   f"see {self.log.name}; its log ends:\n{tail}")
            if line.startswith(tag + " "):
                return json.loads(line[len(tag) + 1:])

    def close(self, timeout=60):
        try:
            if self.p.stdin:
                self.p.stdin.close()
        except OSError:
            pass
        try:
            self.p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            self.p.kill()
            self.p.wait()
        self.log.close()


def child_main(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-8b")
    ap.add_argument("--layers", type=int, default=0, help="decoder layers (0 = the model's own; tests only)")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = harness rehearsal (fp32 reference path, no GPU)")
    ap.add_argument("--eager", action="store_true",
                    help="no hipGraph: every kernel of every step launched from the host (launch-bound)")
    ap.add_argument("--loop", action="store_true",
                    help="after GO, decode until STOP arrives on stdin (a noisy neighbour for the serving "
                         "bench); the context position wraps every --steps steps")
    a = ap.parse_args(argv)
    cmd = sys.stdin.readline().strip()
    if cmd != "LOAD":
        return 0
    tq = os.environ.get("MIVGPU_BENCH_TENANT_QUEUES")
    if tq:
        # a tenant raising its own hardware queue count before the runtime
        # starts (tests: the grant's cap must hold against it)
        os.environ["GPU_MAX_HW_QUEUES"] = tq
    import torch

    from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_8B, QWEN3_TINY, Qwen3Decoder

    cfg = {"qwen3-8b": QWEN3_8B, "qwen3-tiny": QWEN3_TINY}[a.model]
    if a.layers > 0:
        import dataclasses
        cfg = dataclasses.replace(cfg, layers=a.layers)
    if a.device == "cpu":
        return _child_cpu(a, cfg, Qwen3Decoder)
    t_load = time.time()
    max_ctx = a.ctx + a.warmup + a.steps + 16
    dec = Qwen3Decoder(cfg, batch=a.batch, max_ctx=max_ctx, device="cuda")
    dec.fill_context(a.ctx)
    if not a.eager:
        dec.capture(warmup=1)
    for _ in range(a.warmup):
        dec.step()
    torch.cuda.synchronize()
    free, total = torch.cuda.mem_get_info()
    ready = {"load_s": round(time.time() - t_load, 2), "mem_total_mib": total >> 20,
             "mem_free_mib": free >> 20, "allocated_mib": torch.cuda.memory_allocated() >> 20,
             "cus": torch.cuda.get_device_properties(0).multi_processor_count,
             "preload": os.environ.get("LD_PRELOAD", ""), "cu_mask": os.environ.get("HSA_CU_MASK", "")}
    cache = os.environ.get("MIVGPU_SHARED_CACHE")
    if cache and os.environ.get("LD_PRELOAD") and os.path.exists(cache):
        # what the shim charged beyond the hooked allocations (runtime VRAM)
        from k8s_vgpu_scheduler_amd.monitor.region import SharedRegion

        reg = SharedRegion(cache, writable=False)
        me = [p for p in reg.active_procs() if p.pid == os.getpid()]
        ready["context_mib"] = (me[0].used[0].context >> 20) if me else None
        ready["kfd_entry_found"] = bool(me and me[0].hostpid)
        reg.close()
    print("READY " + json.dumps(ready), flush=True)
    cmd = sys.stdin.readline().strip()
    while cmd.startswith("WARM"):
        # more untimed steps after the harness ran a monitor pass (the
        # governor's utilisation switch engaged before the timed window)
        for _ in range(int(cmd.split()[1]) if len(cmd.split()) > 1 else a.warmup):
            dec.step()
        torch.cuda.synchronize()
        print("WARMED {}", flush=True)
        cmd = sys.stdin.readline().strip()
    if cmd != "GO":
        return 0
    if a.loop:
        return _loop_until_stop(a, dec, torch.cuda.synchronize)
    # per-step completion events: time per output token (TPOT) of this slice
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    torch.cuda.synchronize()
    rx0 = _received_ns()
    c0 = _timed_counters()
    t_start = time.time()
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(a.steps):
        dec.step()
        evs[i + 1].record()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tpot = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(a.steps))
    done = {"seconds": dt, "tokens": a.batch * a.steps, "tok_s": a.batch * a.steps / dt,
            "t_start": t_start, "t_end": t_start + dt,
            "tpot_ms_p50": tpot[len(tpot) // 2],
            "tpot_ms_p99": tpot[min(len(tpot) - 1, int(0.99 * len(tpot)))]}
    rx1 = _received_ns()
    c1 = _timed_counters()
    if c0.get("tokens_ms") is not None:
        # the governor's state when GO arrived (a bucket already in debt
        # holds the first gates of the window) and at the end
        done["gov_at_go"] = {k: c0.get(k) for k in ("tokens_ms", "lead_ms", "fair_samples")}
        done["gov_at_end"] = {k: c1.get(k) for k in ("tokens_ms", "lead_ms", "fair_samples")}
    if c0 and c1:
        # the governor over the timed steps only (its totals include the load
        # and warmup, when the slices ran at different times)
        done["timed"] = {k: round(c1[k] - c0[k], 1) for k in c1 if k in c0 and k not in ("tokens_ms", "lead_ms")}
        if os.environ.get("MIVGPU_GATE_TRACE") == "1":
            from k8s_vgpu_scheduler_amd.shim.probe import gate_stats
            # the window's holds: [hold ms, bucket ms at the gate] of the last gates
            tr = gate_stats().get("trace") or []
            n = int(done["timed"].get("gates", 0))
            done["hold_trace"] = [[round(e[4] / 1e6, 2), round(e[5] / 1e6, 2)] for e in tr[-n:] if e[4] > 0]
    if rx0 is not None and rx1 is not None:
        # GPU time the slice received over the timed steps (the governor's
        # share integral), as a share of the wall time
        done["received_gpu_ms"] = round((rx1 - rx0) / 1e6, 1)
        done["busy_share_pct"] = round(100.0 * (rx1 - rx0) / 1e9 / dt, 2)
    done.update(_governor_stats())
    print("DONE " + json.dumps(done), flush=True)
    return 0


def _received_ns():
    """The shim's share integral on device 0 (ns of GPU time received), or
    None without a host bucket."""
    import ctypes
    if not os.environ.get("LD_PRELOAD"):
        return None
    try:
        fn = ctypes.CDLL(None).mivgpu_gate_balance
    except (OSError, AttributeError):
        return None
    t, r = ctypes.c_longlong(), ctypes.c_ulonglong()
    if fn(0, ctypes.byref(t), ctypes.byref(r)) != 0:
        return None
    return r.value


def _timed_counters() -> dict:
    """Governor counters to difference over the timed steps (empty without
    the shim): held time and gates, the sampler's samples in fair-share mode
    and held there, and the share board's passes (all / fully subscribed /
    in fair-share mode)."""
    import ctypes
    if not os.environ.get("LD_PRELOAD"):
        return {}
    out = {}
    try:
        b, h, g = ctypes.c_ulonglong(), ctypes.c_ulonglong(), ctypes.c_ulonglong()
        if ctypes.CDLL(None).mivgpu_gate_stats(0, ctypes.byref(b), ctypes.byref(h), ctypes.byref(g)) == 0:
            out.update({"held_ms": h.value / 1e6, "gates": g.value})
    except (OSError, AttributeError):
        return out
    from k8s_vgpu_scheduler_amd.shim.probe import sampler_info
    si = sampler_info() or {}
    bd = si.get("board") or {}
    for k in ("samples", "fair_samples", "fair_held_samples", "tokens_ms", "lead_ms"):
        if k in si:
            out[k] = si[k]

    for k in ("passes", "sub_passes", "fair_passes"):
        if k in bd:
            out["board_" + k] = bd[k]
    return out


def _governor_stats() -> dict:
    """This slice's governor counters (shim ABI) and measured GPU share (region)."""
    import ctypes
    out = {}
    if not os.environ.get("LD_PRELOAD"):
        return out
    try:
        lib = ctypes.CDLL(None)
        b, h, g = ctypes.c_ulonglong(), ctypes.c_ulonglong(), ctypes.c_ulonglong()
        if lib.mivgpu_gate_stats(0, ctypes.byref(b), ctypes.byref(h), ctypes.byref(g)) == 0:
            out.update({"gov_charged_ms": round(b.value / 1e6, 1), "gov_held_ms": round(h.value / 1e6, 1),
                        "gov_gates": g.value})
    except (OSError, AttributeError):
        pass
    from k8s_vgpu_scheduler_amd.shim.probe import gate_stats
    g = gate_stats()
    for k in ("received_ms", "tokens_ms", "sampler_state_ms", "sampler_samples", "sampler_pass_us_mean",
              "sampler_pass_us_max"):
        if k in g:
            out["gov_" + k] = g[k]
    si = g.get("sampler")
    if si and os.environ.get("MIVGPU_GATE_TRACE") == "1":
        # the samples outside the fair-share mode: [t ms, interval ms, share,
        # run ms, bucket ms after, previous sample in the mode]
        out["gov_nonfair"] = si.get("nonfair")
    if si:
        # how the share was charged: from the GPU's one sampler (board) or the
        # local estimate, and whose board it was
        bd = si.get("board") or {}
        out["sampler"] = {"board_charged": si.get("board_charged"), "local_charged": si.get("local_charged"),
                          "board_share": si.get("board_share"), "board_owner": bd.get("owner"),
                          "owner_kind": bd.get("owner_kind"), "board_slots": len(bd.get("slots") or []),
                          # fair-share mode (board.h): samples in it / held there on the lead
                          "fair_samples": si.get("fair_samples"), "fair_held_samples": si.get("fair_held_samples"),
                          "board_passes": bd.get("passes"), "board_sub_passes": bd.get("sub_passes"),
                          "board_fair_passes": bd.get("fair_passes")}
    cache = os.environ.get("MIVGPU_SHARED_CACHE")
    if cache and os.path.exists(cache):
        from k8s_vgpu_scheduler_amd.monitor.region import SharedRegion
        reg = SharedRegion(cache, writable=False)
        me = [p for p in reg.active_procs() if p.pid == os.getpid()]
        if me:
            out.update({"share_pct": round(me[0].util[0].share_ppm / 1e4, 1), "util_pct": me[0].util[0].util_pct})
        reg.close()
    return out


def _child_cpu(a, cfg, Qwen3Decoder):
    """The same LOAD/READY/GO/DONE protocol on the CPU reference decoder, so
    the multi-rank harness (spawn, barriers, MAX wall, token sum, JSON line)
    can be rehearsed without a GPU (tests/test_bench_harness.py)."""
    t_load = time.time()
    dec = Qwen3Decoder(cfg, batch=a.batch, max_ctx=a.ctx + a.warmup + a.steps + 16, device="cpu", native=False)
    dec.fill_context(a.ctx)
    for _ in range(a.warmup):
        dec.step()
    print("READY " + json.dumps({"load_s": round(time.time() - t_load, 2), "mem_total_mib": 0, "mem_free_mib": 0,
                                 "allocated_mib": 0, "cus": 0, "preload": os.environ.get("LD_PRELOAD", ""),
                                 "cu_mask": os.environ.get("HSA_CU_MASK", "")}), flush=True)
    cmd = sys.stdin.readline().strip()
    while cmd.startswith("WARM"):
        for _ in range(int(cmd.split()[1]) if len(cmd.split()) > 1 else a.warmup):
            dec.step()
        print("WARMED {}", flush=True)
        cmd = sys.stdin.readline().strip()
    if cmd != "GO":
        return 0
    if a.loop:
        return _loop_until_stop(a, dec, lambda: None)
    t_start = time.time()
    t0 = time.perf_counter()
    tpot = []
    for _ in range(a.steps):
        s0 = time.perf_counter()
        dec.step()
        tpot.append((time.perf_counter() - s0) * 1e3)
    dt = time.perf_counter() - t0
    tpot.sort()
    print("DONE " + json.dumps({"seconds": dt, "tokens": a.batch * a.steps, "tok_s": a.batch * a.steps / dt,
                                "t_start": t_start, "t_end": t_start + dt, "tpot_ms_p50": tpot[len(tpot) // 2],
                                "tpot_ms_p99": tpot[min(len(tpot) - 1, int(0.99 * len(tpot)))]}), flush=True)
    return 0


def _loop_until_stop(a, dec, sync) -> int:
    """Decode rounds of a.steps steps (position rewound to the context each
    round, so the cache never grows) until STOP arrives; DONE carries the
    tokens/s over the whole loop."""
    import select as _select
    t0, steps = time.perf_counter(), 0
    while True:
        dec.pos.fill_(a.ctx)
        dec.seqlens.fill_(a.ctx + 1)
        for _ in range(a.steps):
            dec.step()
        steps += a.steps
        sync()
        r, _, _ = _select.select([sys.stdin], [], [], 0)
        if r and sys.stdin.readline().strip() in ("STOP", ""):
            break
    dt = time.perf_counter() - t0
    done = {"seconds": dt, "tokens": a.batch * steps, "tok_s": a.batch * steps / dt, "loop": True}
    if a.device != "cpu":
        done.update(_governor_stats())
    print("DONE " + json.dumps(done), flush=True)
    return 0


def spawn_round(specs, physical_gpu, cache_dir: Path, log_dir: Path, child_args, tag: str):
    cache_dir.mkdir(parents=True, exist_ok=True)
    procs = []
    for s in specs:
        env = slice_env(s, physical_gpu, cache_dir)
        procs.append(SliceProc(s, env, child_args, log_dir / f"{tag}_slice{s.index}.log"))
    return procs


def run_round(procs, barrier=None, sync=None, load_timeout=900, run_timeout=900, before_go=None,
              rewarm: int = 0) -> dict:
    """Drive one spawned round through LOAD/READY/GO/DONE; returns timings.
    ``before_go()``: called once every slice is READY (a monitor pass); then
    ``rewarm`` more untimed steps per slice (WARM/WARMED) before GO."""
    for p in procs:
        p.send("LOAD")
    readies = [p.expect("READY", load_timeout) for p in procs]
    if before_go is not None:
        before_go()
    if rewarm > 0:
        for p in procs:
            p.send(f"WARM {rewarm}")
        for p in procs:
            p.expect("WARMED", load_timeout)
    if barrier:
        barrier()
    if sync:
        sync()
    t0 = time.perf_counter()
    for p in procs:
        p.send("GO")
    dones = [p.expect("DONE", run_timeout) for p in procs]
    if sync:
        sync()
    t1 = time.perf_counter()
    if barrier:
        barrier()
    for p in procs:
        p.close()
    return {"wall_s": t1 - t0, "ready": readies, "done": dones,
            "tokens": sum(d["tokens"] for d in dones)}


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        sys.exit(child_main(sys.argv[2:]))
    print("use bench.py", file=sys.stderr)
    sys.exit(2)
