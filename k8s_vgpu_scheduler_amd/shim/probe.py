"""GPU isolation probe: runs workload children natively and under libmivgpu.so.

Each scenario is a separate child process (the shim must be LD_PRELOADed
before the HIP runtime initialises), started BEFORE this process touches the
GPU.  Children print one JSON line.  Used for the first-light GPU validation
and by ``bench.py``/tests marked ``gpu``.

    python -m k8s_vgpu_scheduler_amd.shim.probe --out gpurun_out/probe.json
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import time
from pathlib import Path

from k8s_vgpu_scheduler_amd.shim import shim_env, shim_path


def child_matmul(args) -> dict:
    import torch

    dev = torch.device("cuda:0")
    free, total = torch.cuda.mem_get_info()
    props = torch.cuda.get_device_properties(0)
    n = args.n
    a = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        c = a @ b
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tflops = 2 * n ** 3 * args.iters / dt / 1e12
    out = {"mode": "matmul", "tflops": tflops, "seconds": dt, "mem_free_mib": free >> 20,
           "mem_total_mib": total >> 20, "props_total_mib": props.total_memory >> 20,
           "cus": props.multi_processor_count}
    if args.oom_probe_mib:
        try:
            x = torch.empty(args.oom_probe_mib << 20, dtype=torch.uint8, device=dev)
            out["oom_probe"] = "allocated"
            if args.hold_s:
                time.sleep(args.hold_s)   # keep it resident while a sibling probes
            del x
        except torch.OutOfMemoryError:
            out["oom_probe"] = "oom"
        except RuntimeError as e:  # pragma: no cover
            out["oom_probe"] = f"error: {e}"[:200]
    del c
    out.update(gate_stats())
    return out


def gate_stats() -> dict:
    """Governor counters of the preloaded shim (empty if not preloaded)."""
    import ctypes

    try:
        fn = ctypes.CDLL(None).mivgpu_gate_stats
    except AttributeError:
        return {}
    b, h, g = ctypes.c_ulonglong(), ctypes.c_ulonglong(), ctypes.c_ulonglong()
    if fn(0, ctypes.byref(b), ctypes.byref(h), ctypes.byref(g)) != 0:
        return {"gate": "inactive"}
    out = {"gate_busy_ms": b.value / 1e6, "gate_held_ms": h.value / 1e6, "gates": g.value}
    try:
        bal = ctypes.CDLL(None).mivgpu_gate_balance
        t, r = ctypes.c_longlong(), ctypes.c_ulonglong()
        if bal(0, ctypes.byref(t), ctypes.byref(r)) == 0:
            out["received_ms"] = r.value / 1e6       # the host bucket's share integral
            out["tokens_ms"] = t.value / 1e6
        st = ctypes.CDLL(None).mivgpu_occ_states
        ns5, n = (ctypes.c_double * 5)(), ctypes.c_ulonglong()
        if st(0, ns5, ctypes.byref(n)) == 0:
            out["sampler_state_ms"] = dict(zip(("own", "alone_busy", "held", "others", "idle"),
                                               (round(v / 1e6, 1) for v in ns5)))
            out["sampler_samples"] = n.value
        tm = ctypes.CDLL(None).mivgpu_occ_timing
        passes, tot, mx = ctypes.c_ulonglong(), ctypes.c_ulonglong(), ctypes.c_ulonglong()
        if tm(ctypes.byref(passes), ctypes.byref(tot), ctypes.byref(mx)) == 0 and passes.value:
            out["sampler_pass_us_mean"] = round(tot.value / passes.value / 1e3, 1)
            out["sampler_pass_us_max"] = round(mx.value / 1e3, 1)
    except AttributeError:
        pass
    info = sampler_info()
    if info is not None:
        out["sampler"] = info
    try:
        tr = ctypes.CDLL(None).mivgpu_gate_trace
        buf = (ctypes.c_longlong * (128 * 8))()
        n = tr(0, buf, 128)
        out["trace"] = [[buf[i * 8 + k] for k in range(7)] for i in range(n)]
    except AttributeError:
        pass
    return out


def sampler_info(dev: int = 0) -> dict | None:
    """The preloaded shim's own account of how it charges the governor
    (mivgpu_sampler_info): the share board (owner role, owner, age, every
    process's integrals), samples charged from the board or the local
    estimate, the local estimate's peers and the sampler's state split."""
    import ctypes
    import json

    try:
        fn = ctypes.CDLL(None).mivgpu_sampler_info
    except AttributeError:
        return None
    buf = ctypes.create_string_buffer(32768)
    n = fn(dev, buf, len(buf))
    if n <= 0:
        return None
    try:
        return json.loads(buf.value.decode(errors="replace"))
    except ValueError:
        return {"raw": buf.value.decode(errors="replace")[:2000]}


def child_stream(args) -> dict:
    import torch

    dev = torch.device("cuda:0")
    n = args.n * 1024 * 1024 * 16  # float elements
    x = torch.empty(n, device=dev, dtype=torch.float32).fill_(1.0)
    y = torch.empty_like(x)
    for _ in range(3):
        y.copy_(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        y.copy_(x)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"mode": "stream", "gbps": 2 * x.numel() * 4 * args.iters / dt / 1e9, "seconds": dt}


def _timed(fn, iters: int) -> float:
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def child_mfma(args) -> dict:
    """Hand-written matrix-core load (csrc/ops/loadgen.hip): exact FLOP count."""
    from k8s_vgpu_scheduler_amd import ops

    blocks, inner = 256 * 4, 2048
    out = ops.mfma_burn(blocks, inner)
    dt = _timed(lambda: ops.mfma_burn(blocks, inner, out=out), args.iters)
    res = {"mode": "mfma", "tflops": ops.mfma_burn_flops(blocks, inner) * args.iters / dt / 1e12, "seconds": dt,
           "finite": bool(out.isfinite().all().item())}
    res.update(gate_stats())
    return res


def child_hipstream(args) -> dict:
    """Hand-written HBM stream copy (csrc/ops/loadgen.hip)."""
    import torch

    from k8s_vgpu_scheduler_amd import ops

    nbytes = args.n << 20
    src = torch.empty(nbytes // 4, dtype=torch.int32, device="cuda").random_()
    dst = torch.empty_like(src)
    dt = _timed(lambda: ops.stream_copy(src, dst), args.iters)
    res = {"mode": "hipstream", "gbps": 2 * nbytes * args.iters / dt / 1e9, "seconds": dt,
           "exact": bool(torch.equal(src, dst))}
    res.update(gate_stats())
    return res


def child_hwid(args) -> dict:
    """Which XCD / SE / CU ids does a grid touch under the current HSA_CU_MASK?"""
    from k8s_vgpu_scheduler_amd import ops

    t = ops.hwid_probe(4096)
    hw = [v & 0xFFFFFFFF for v in t[:, 0].tolist()]
    xcc = [v & 0xFFFFFFFF for v in t[:, 1].tolist()]
    places = sorted({((x & 0xF), (h >> 13) & 0x7, (h >> 12) & 0x1, (h >> 8) & 0xF) for h, x in zip(hw, xcc)})
    return {"mode": "hwid", "cu_mask": os.environ.get("HSA_CU_MASK", ""), "distinct": len(places),
            "xccs": sorted({p[0] for p in places}), "places": places[:512]}


def child_light(args) -> dict:
    """A light tenant: one tiny kernel every 50 ms for --hold-s seconds (an
    inference server idling between requests)."""
    import torch

    x = torch.zeros(1024, device="cuda")
    n = 0
    t_end = time.time() + args.hold_s
    while time.time() < t_end:
        x.add_(1)
        torch.cuda.synchronize()
        n += 1
        time.sleep(0.05)
    return {"mode": "light", "kernels": n}


def child_region(args) -> dict:
    """Allocate through PyTorch under the shim and read the accounting back
    through the monitor's shared-region reader (what vGPUmonitor sees)."""
    import torch

    from k8s_vgpu_scheduler_amd.monitor.region import SharedRegion

    x = torch.empty(args.oom_probe_mib << 20, dtype=torch.uint8, device="cuda")
    x.fill_(1)
    torch.cuda.synchronize()
    time.sleep(0.05)                   # past the shim's 20 ms runtime-VRAM refresh interval
    torch.cuda.mem_get_info()          # the meminfo hook refreshes the context charge
    reg = SharedRegion(os.environ["MIVGPU_SHARED_CACHE"], writable=False)
    me = [p for p in reg.active_procs() if p.pid == os.getpid()]
    # KFD names the entry by the host pid, which the shim published in the slot
    kfd = Path("/sys/class/kfd/kfd/proc") / str(me[0].hostpid if me and me[0].hostpid else os.getpid())
    kfd_vram = sum(int(f.read_text()) for f in kfd.glob("vram_*")) if kfd.is_dir() else -1
    out = {"mode": "region", "dev_used_mib": reg.dev_used(0) >> 20, "limit_mib": reg.memory_limit(0) >> 20,
           "procs": len(list(reg.active_procs())), "self_found": bool(me),
           "self_buffer_mib": (me[0].used[0].buffer >> 20) if me else -1,
           "self_vmm": me[0].used[0].vmm if me else -1,
           "self_context": me[0].used[0].context if me else -1,
           "self_total": me[0].used[0].total if me else -1,
           "self_buffer": me[0].used[0].buffer if me else -1,
           "kfd_vram": kfd_vram, "hostpid": me[0].hostpid if me else -1,
           "launches": reg.launches(0), "uuid": reg.uuid(0)}
    reg.close()
    del x
    return out


def _launch_count() -> int:
    """Launches the preloaded shim has seen in this process (-1 without it)."""
    import ctypes

    try:
        fn = ctypes.CDLL(None).mivgpu_launch_count
    except AttributeError:
        return -1
    fn.restype = ctypes.c_ulonglong
    return int(fn())


def child_triton(args) -> dict:
    """A @triton.jit matmul loop: Triton resolves every HIP entry point at run
    time (dlopen + dlsym("hipGetProcAddress") + hipGetProcAddress), the path
    that bypassed PLT interposition before round 3."""
    import torch
    import triton
    import triton.language as tl

    @triton.jit
    def mm_kernel(a, b, c, M, N, K, BM: tl.constexpr, BN: tl.constexpr, BK: tl.constexpr):
        pid_m = tl.program_id(0)
        pid_n = tl.program_id(1)
        rm = pid_m * BM + tl.arange(0, BM)
        rn = pid_n * BN + tl.arange(0, BN)
        rk = tl.arange(0, BK)
        acc = tl.zeros((BM, BN), dtype=tl.float32)
        for k0 in range(0, K, BK):
            x = tl.load(a + rm[:, None] * K + (k0 + rk)[None, :])
            y = tl.load(b + (k0 + rk)[:, None] * N + rn[None, :])
            acc += tl.dot(x, y)
        tl.store(c + rm[:, None] * N + rn[None, :], acc.to(tl.bfloat16))

    n = args.n
    a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    grid = (n // 128, n // 128)

    def step():
        mm_kernel[grid](a, b, c, n, n, n, BM=128, BN=128, BK=64, num_warps=4)

    step()
    torch.cuda.synchronize()
    ref = (a[:64].float() @ b.float())[:, :64]
    err = ((c[:64, :64].float() - ref).abs().max() / ref.abs().max()).item()
    l0 = _launch_count()
    dt = _timed(step, args.iters)
    launches = _launch_count() - l0 if l0 >= 0 else -1
    res = {"mode": "triton", "tflops": 2 * n ** 3 * args.iters / dt / 1e12, "seconds": dt, "rel_err": err,
           "shim_launches": launches, "iters": args.iters}
    res.update(gate_stats())
    return res


def child_compile(args) -> dict:
    """A torch.compile'd MLP whose GEMMs and epilogues are Inductor-generated
    Triton kernels (max-autotune, Triton GEMM backend only), launched through
    Triton's run-time-resolved HIP entry points."""
    import torch
    import torch._inductor.config as ic

    ic.max_autotune = True
    ic.max_autotune_gemm_backends = "TRITON"
    ic.max_autotune_gemm_search_space = "DEFAULT"
    ic.coordinate_descent_tuning = False
    d, h, m = 4096, 8192, args.n
    w1 = torch.randn(d, h, device="cuda", dtype=torch.bfloat16) * d ** -0.5
    w2 = torch.randn(h, d, device="cuda", dtype=torch.bfloat16) * h ** -0.5
    x = torch.randn(m, d, device="cuda", dtype=torch.bfloat16)

    def mlp(x):
        return torch.nn.functional.gelu(x @ w1) @ w2 + x

    f = torch.compile(mlp)
    y = f(x)
    torch.cuda.synchronize()
    ref = mlp(x)
    err = ((y.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
    l0 = _launch_count()
    dt = _timed(lambda: f(x), args.iters)
    launches = _launch_count() - l0 if l0 >= 0 else -1
    res = {"mode": "compile", "tflops": 2 * m * d * h * 2 * args.iters / dt / 1e12, "seconds": dt,
           "rel_err": err, "shim_launches": launches, "iters": args.iters}
    res.update(gate_stats())
    return res


def _hip_runtime_path() -> str:
    """Path of the libamdhip64 the process has mapped (PyTorch's copy)."""
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64.so" in line:
                return line.split()[-1]
    raise RuntimeError("libamdhip64 not mapped")


def child_lookup(args) -> dict:
    """HIP allocators reached by run-time lookup from Python -- ctypes dlsym
    on the runtime's handle, hipGetProcAddress, and the array / 3D allocators
    -- past the container's grant."""
    import ctypes

    import torch

    torch.zeros(1, device="cuda")                 # runtime up, context created
    lib = ctypes.CDLL(_hip_runtime_path(), mode=os.RTLD_NOLOAD | os.RTLD_LAZY)
    big = args.oom_probe_mib << 20
    out = {"mode": "lookup"}
    p = ctypes.c_void_p()
    malloc = lib.hipMalloc                         # dlsym(handle, "hipMalloc")
    malloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    out["dlsym_big_rc"] = malloc(ctypes.byref(p), big)
    out["dlsym_small_rc"] = malloc(ctypes.byref(p), 256 << 20)
    if out["dlsym_small_rc"] == 0:
        lib.hipFree(p)
    gpa = lib.hipGetProcAddress
    gpa.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]
    fp = ctypes.c_void_p()
    out["gpa_rc"] = gpa(b"hipMalloc", ctypes.byref(fp), 700, 0, None)
    fmalloc = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t)(fp.value)
    out["gpa_big_rc"] = fmalloc(ctypes.byref(p), big)
    out["gpa_is_hook"] = fp.value == ctypes.cast(ctypes.CDLL(None).hipMalloc, ctypes.c_void_p).value

    class Extent(ctypes.Structure):
        _fields_ = [("width", ctypes.c_size_t), ("height", ctypes.c_size_t), ("depth", ctypes.c_size_t)]

    class PitchedPtr(ctypes.Structure):
        _fields_ = [("ptr", ctypes.c_void_p), ("pitch", ctypes.c_size_t), ("xsize", ctypes.c_size_t),
                    ("ysize", ctypes.c_size_t)]

    class ChannelDesc(ctypes.Structure):
        _fields_ = [("x", ctypes.c_int), ("y", ctypes.c_int), ("z", ctypes.c_int), ("w", ctypes.c_int),
                    ("f", ctypes.c_int)]

    pp = PitchedPtr()
    m3 = lib.hipMalloc3D
    m3.argtypes = [ctypes.POINTER(PitchedPtr), Extent]
    rows = big // (64 << 10)
    out["malloc3d_big_rc"] = m3(ctypes.byref(pp), Extent(64 << 10, rows, 1))
    out["malloc3d_small_rc"] = m3(ctypes.byref(pp), Extent(64 << 10, 4096, 1))       # 256 MiB
    if out["malloc3d_small_rc"] == 0:
        lib.hipFree(ctypes.c_void_p(pp.ptr))
    # a 2D float4 array of 8192 x 8192 x 16 B = 1 GiB while only 0.5 GiB of the slice is free
    free, total = torch.cuda.mem_get_info()
    hold = torch.empty(max(free - (512 << 20), 1), dtype=torch.uint8, device="cuda")
    arr = ctypes.c_void_p()
    ma = lib.hipMallocArray
    ma.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ChannelDesc), ctypes.c_size_t, ctypes.c_size_t,
                   ctypes.c_uint]
    desc = ChannelDesc(32, 32, 32, 32, 2)          # float4
    out["array_rc"] = ma(ctypes.byref(arr), ctypes.byref(desc), 8192, 8192, 0)
    if out["array_rc"] == 0:
        lib.hipFreeArray(arr)
    del hold
    free, total = torch.cuda.mem_get_info()
    out["mem_total_mib"] = total >> 20
    return out


def child_module(args) -> dict:
    """hipModuleLoadData of a gfx950 code object (the governor kernel's offload
    bundle): its load span is charged as `module` bytes, and context + module
    + buffer + vmm is still KFD's per-process VRAM."""
    import ctypes

    import torch

    from k8s_vgpu_scheduler_amd.monitor.region import SharedRegion
    from k8s_vgpu_scheduler_amd.utils import build as b

    x = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    lib = ctypes.CDLL(_hip_runtime_path(), mode=os.RTLD_NOLOAD | os.RTLD_LAZY)
    img = ctypes.create_string_buffer(b.GOV_HSACO.read_bytes())
    mods = []
    for _ in range(max(1, args.iters)):
        m = ctypes.c_void_p()
        rc = lib.hipModuleLoadData(ctypes.byref(m), img)
        if rc != 0:
            return {"mode": "module", "load_rc": rc}
        mods.append(m)
    torch.cuda.synchronize()
    time.sleep(0.05)
    torch.cuda.mem_get_info()                     # refresh the context charge
    reg = SharedRegion(_region_path(), writable=False)
    me = [p for p in reg.active_procs() if p.pid == os.getpid()][0]
    kfd = Path("/sys/class/kfd/kfd/proc") / str(me.hostpid or os.getpid())
    kfd_vram = sum(int(f.read_text()) for f in kfd.glob("vram_*")) if kfd.is_dir() else -1
    u = me.used[0]
    out = {"mode": "module", "load_rc": 0, "modules": len(mods), "module": u.module, "context": u.context,
           "buffer": u.buffer, "vmm": u.vmm, "total": u.total, "kfd_vram": kfd_vram}
    reg.close()
    for m in mods:
        lib.hipModuleUnload(m)
    reg = SharedRegion(os.environ["MIVGPU_SHARED_CACHE"], writable=False)
    out["module_after_unload"] = [p for p in reg.active_procs() if p.pid == os.getpid()][0].used[0].module
    reg.close()
    del x
    return out


def _region_path() -> str | None:
    """This process's shared region: the environment, else the grant file."""
    path = os.environ.get("MIVGPU_SHARED_CACHE")
    if path:
        return path
    grant = os.environ.get("MIVGPU_LIMITS_FILE")
    if grant and os.path.exists(grant):
        from k8s_vgpu_scheduler_amd.deviceplugin.allocate import parse_grant
        return parse_grant(Path(grant).read_text()).get("MIVGPU_SHARED_CACHE")
    return None


def _kfd_pid(pid: int | None = None) -> int:
    """KFD's name for a process (the host pid; the box may run us in a pid
    namespace): the hostpid the shim found for itself and published in its
    region slot, else the pid itself."""
    pid = os.getpid() if pid is None else pid
    path = _region_path()
    if not path or not os.path.exists(path):
        return pid
    from k8s_vgpu_scheduler_amd.monitor.region import SharedRegion
    reg = SharedRegion(path, writable=False)
    try:
        me = [p for p in reg.active_procs() if p.pid == pid]
        return me[0].hostpid if me and me[0].hostpid else pid
    finally:
        reg.close()


def child_queues(args) -> dict:
    """A tenant that raises GPU_MAX_HW_QUEUES before HIP starts, then spreads
    work over 8 streams: how many KFD hardware queues does it own?"""
    if not args.keep_env:
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
    import torch

    streams = [torch.cuda.Stream() for _ in range(8)]
    x = torch.ones(1 << 20, device="cuda")
    for s in streams:
        with torch.cuda.stream(s):
            for _ in range(4):
                x.add_(1)
    torch.cuda.synchronize()
    pid = _kfd_pid()
    qdir = Path("/sys/class/kfd/kfd/proc") / str(pid) / "queues"
    out = {"mode": "queues", "kfd_queues": len(os.listdir(qdir)) if qdir.is_dir() else -1,
           "env_seen_by_python": os.environ.get("GPU_MAX_HW_QUEUES"), "pid": pid}
    if out["kfd_queues"] < 0:
        procs = Path("/sys/class/kfd/kfd/proc")
        out["kfd_procs"] = sorted(os.listdir(procs)) if procs.is_dir() else None
        out["own_entry"] = sorted(os.listdir(procs / str(pid))) if (procs / str(pid)).is_dir() else None
    return out


def child_tamper(args) -> dict:
    """A hostile tenant under a 4 GiB grant.  It maps its
    own shared region, optionally deletes the region file (``--unlink``: the
    monitor then sees no region at all), zeroes the usage counters and tries
    to allocate past its grant (the shim charges the VRAM KFD shows for the
    process beyond its hooked allocations, so the zeroed counter buys no
    headroom: ``first`` is "oom").  After the parent's monitor pass(es) it keeps
    rewriting the region (clearing the block flag, zeroing the counters) from
    a thread while it allocates again and launches a kernel: the verdicts in
    the read-only control file must hold anyway."""
    import threading

    import torch

    from k8s_vgpu_scheduler_amd.monitor.region import SharedRegion

    x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    x.fill_(1)
    torch.cuda.synchronize()
    kfd_pid = _kfd_pid()
    reg = SharedRegion(args.out)
    if args.unlink:
        os.unlink(args.out)
    reg.r.dev_used[0] = 0
    reg.r.mem_limit[0] = 1 << 40
    for p in reg.active_procs():
        p.used[0].total = 0
        p.used[0].buffer = 0
    y = None
    try:
        y = torch.empty(args.oom_probe_mib << 20, dtype=torch.uint8, device="cuda")
        y.fill_(1)
        torch.cuda.synchronize()
        first = "allocated"
    except torch.OutOfMemoryError:
        first = "oom"
    # the launch below must not allocate (an over-grant container gets no
    # memory at all): its operand exists before the verdict
    w = torch.zeros(1 << 16, device="cuda")
    torch.cuda.synchronize()
    print("TAMPERED " + json.dumps({"first": first, "kfd_pid": kfd_pid}), flush=True)
    sys.stdin.readline()                      # the parent's monitor pass(es)
    stop = threading.Event()

    def rewrite():                            # "I am not blocked, I use nothing"
        while not stop.is_set():
            reg.r.recent_kernel = 0
            reg.r.dev_used[0] = 0
            time.sleep(0.002)
    th = threading.Thread(target=rewrite, daemon=True)
    th.start()
    time.sleep(0.05)
    try:
        z = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
        second = "allocated"
        del z
    except torch.OutOfMemoryError:
        second = "oom"
    t0 = time.time()
    w.add_(1)                                 # parked while the control block holds
    torch.cuda.synchronize()
    total = float(w[0].item())
    parked_s = time.time() - t0
    stop.set()
    th.join()
    out = {"mode": "tamper", "first": first, "second": second, "parked_s": round(parked_s, 3),
           "sum": total, "unlinked": bool(args.unlink)}
    reg.close()
    del x, y
    return out


def child_hog(args) -> dict:
    """A process of the container WITHOUT the shim (its LD_PRELOAD stripped or
    ignored): allocates --oom-probe-mib MiB, prints ``HOG {kfd_pid}`` and
    holds the memory until a line arrives on stdin.  KFD names it by the
    host pid: the one /sys/class/kfd/kfd/proc entry that appeared with its
    first allocation (the box may run us in a pid namespace)."""
    kfd = "/sys/class/kfd/kfd/proc"
    before = set(os.listdir(kfd)) if os.path.isdir(kfd) else set()
    import torch

    x = torch.empty(args.oom_probe_mib << 20, dtype=torch.uint8, device="cuda")
    x.fill_(1)
    torch.cuda.synchronize()
    new = sorted((set(os.listdir(kfd)) if os.path.isdir(kfd) else set()) - before)

    # KFD lists every process of the HOST, other jobs on other GPUs too: only
    # this GPU's vram_<gpu_id> counts when the topology names one GPU
    from k8s_vgpu_scheduler_amd.monitor.hosttruth import single_gpu_ids

    try:
        gid = single_gpu_ids("x").get("x")
    except OSError:
        gid = None
    pattern = f"vram_{gid}" if gid else "vram_*"

    def vram(pid):   # this process's VRAM as KFD counts it
        tot = 0
        for f in glob.glob(os.path.join(kfd, pid, pattern)):
            try:
                tot += int(open(f).read().strip() or 0)
            except (OSError, ValueError):
                pass
        return tot
    # the new entry holding at least what this process allocated (several
    # may appear at once when other processes start meanwhile)
    mine = [p for p in new if vram(p) >= args.oom_probe_mib << 20]
    kfd_pid = int(mine[0]) if len(mine) == 1 else (int(new[0]) if len(new) == 1 else os.getpid())
    print("HOG " + json.dumps({"kfd_pid": kfd_pid, "mib": args.oom_probe_mib, "new_entries": len(new)}), flush=True)
    sys.stdin.readline()
    del x
    return {"mode": "hog", "kfd_pid": kfd_pid}


def run_child(mode: str, env_extra: dict, shim: bool, extra_args=(), timeout=300) -> dict:
    env = dict(os.environ)
    if shim:
        env.update(shim_env())
    env.update({k: str(v) for k, v in env_extra.items()})
    cmd = [sys.executable, "-m", "k8s_vgpu_scheduler_amd.shim.probe", "--child", mode, *extra_args]
    t0 = time.time()
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=timeout)
    res = {"rc": r.returncode, "wall_s": round(time.time() - t0, 2)}
    for line in r.stdout.splitlines():
        if line.startswith("{"):
            res.update(json.loads(line))
    if r.returncode != 0:
        res["stderr"] = r.stderr[-2000:]
    return res


def run_parallel(mode: str, envs: list, shim: bool, extra_args=(), timeout=300) -> list:
    procs = []
    for e in envs:
        env = dict(os.environ)
        if shim:
            env.update(shim_env())
        env.update({k: str(v) for k, v in e.items()})
        cmd = [sys.executable, "-m", "k8s_vgpu_scheduler_amd.shim.probe", "--child", mode, *extra_args]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = []
    for p in procs:
        try:
            so, se = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            so, se = p.communicate()
        res = {"rc": p.returncode}
        for line in so.splitlines():
            if line.startswith("{"):
                res.update(json.loads(line))
        if p.returncode != 0:
            res["stderr"] = se[-1500:]
        outs.append(res)
    return outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", default=None)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--oom-probe-mib", type=int, default=0)
    ap.add_argument("--hold-s", type=float, default=0.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--hwid", action="store_true")
    ap.add_argument("--unlink", action="store_true", help="child tamper: delete the region file first")
    ap.add_argument("--keep-env", action="store_true", help="child queues: do not raise GPU_MAX_HW_QUEUES")
    ap.add_argument("--hostile", action="store_true",
                    help="child: rewrite the grant in the environment before the runtime starts "
                         "(all CUs, 200 GiB, control disabled) -- the grant file must still win")
    args = ap.parse_args()
    if args.child and args.hostile:
        os.environ.pop("HIP_DEVICE_MEMORY_LIMIT_0", None)
        os.environ["HIP_DEVICE_MEMORY_LIMIT"] = "200g"
        os.environ["HSA_CU_MASK"] = "0:0-255"
        os.environ["MIVGPU_DISABLE_CONTROL"] = "1"
    if args.child:
        fn = {"matmul": child_matmul, "stream": child_stream, "hwid": child_hwid,
              "region": child_region, "mfma": child_mfma, "hipstream": child_hipstream,
              "light": child_light, "triton": child_triton, "compile": child_compile, "lookup": child_lookup,
              "module": child_module, "queues": child_queues, "tamper": child_tamper,
              "hog": child_hog}[args.child]
        print(json.dumps(fn(args)), flush=True)
        return
    tmp = Path(os.environ.get("TMPDIR", "/tmp")) / f"mivgpu-probe-{os.getpid()}"
    tmp.mkdir(parents=True, exist_ok=True)
    mm = ["--n", "8192", "--iters", "60"]
    results = {}
    if args.hwid:
        for m in ("", "0:0-31", "0:32-63", "0:0-7", "0:0,8,16,24", "0:0-3,128-131"):
            results[f"hwid[{m}]"] = run_child("hwid", {"HSA_CU_MASK": m} if m else {}, False, [])
    if args.quick:
        for pct in (25, 50, 75):
            results[f"gate_force_{pct}"] = run_child(
                "matmul", {"MIVGPU_SHARED_CACHE": tmp / f"q{pct}.cache", "HIP_DEVICE_CORE_LIMIT": pct,
                           "GPU_CORE_UTILIZATION_POLICY": "force"}, True, ["--n", "8192", "--iters", "200"])
        results["native_200"] = run_child("matmul", {}, False, ["--n", "8192", "--iters", "200"])
        txt = json.dumps(results, indent=1)
        print(txt)
        if args.out:
            Path(args.out).parent.mkdir(parents=True, exist_ok=True)
            Path(args.out).write_text(txt)
        return
    results["native"] = run_child("matmul", {}, False, mm)
    results["shim_nolimit"] = run_child("matmul", {"MIVGPU_SHARED_CACHE": tmp / "a.cache"}, True, mm)
    results["shim_36g"] = run_child(
        "matmul", {"MIVGPU_SHARED_CACHE": tmp / "b.cache", "HIP_DEVICE_MEMORY_LIMIT_0": "36864m"},
        True, [*mm, "--oom-probe-mib", "40000"])
    for cus in (64, 128):
        results[f"cumask_{cus}"] = run_child("matmul", {"HSA_CU_MASK": f"0:0-{cus - 1}"}, False, mm)
    results["gate_force_25"] = run_child(
        "matmul", {"MIVGPU_SHARED_CACHE": tmp / "c.cache", "HIP_DEVICE_CORE_LIMIT": "25",
                   "GPU_CORE_UTILIZATION_POLICY": "force", "MIVGPU_LOG_LEVEL": "3"}, True, mm)
    results["stream_native"] = run_child("stream", {}, False, ["--n", "64", "--iters", "50"])
    results["stream_cumask_64"] = run_child("stream", {"HSA_CU_MASK": "0:0-63"}, False,
                                            ["--n", "64", "--iters", "50"])
    if not args.quick:
        envs = [{"HSA_CU_MASK": f"0:{i * 64}-{i * 64 + 63}"} for i in range(4)]
        results["4x_cumask_parallel"] = run_parallel("matmul", envs, False, mm)
        envs = [{"MIVGPU_SHARED_CACHE": tmp / f"g{i}.cache", "HIP_DEVICE_CORE_LIMIT": "25",
                 "GPU_CORE_UTILIZATION_POLICY": "force"} for i in range(4)]
        results["4x_gate_parallel"] = run_parallel("matmul", envs, True, mm)
        results["4x_native_parallel"] = run_parallel("matmul", [{} for _ in range(4)], False, mm)
    txt = json.dumps(results, indent=1)
    print(txt)
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(txt)


if __name__ == "__main__":
    main()
