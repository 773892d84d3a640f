"""Run-time-resolved HIP entry points under libmivgpu.so on an MI355X
(VERDICT r2 "do this" #1, #4c, #6).

Triton (and torch.compile/Inductor, which generates Triton kernels) resolves
every HIP function through dlopen + dlsym("hipGetProcAddress") +
hipGetProcAddress; ctypes resolves through dlsym.  Before round 3 those paths
bypassed every hook: no governor gate, no launch count, no HBM verdict.  The
bounds are those of test_heavy_tenant_held_to_its_share_next_to_light_neighbours
(tests/test_shim_gpu.py).
"""

import json
import time
import os
import tempfile

import pytest

from k8s_vgpu_scheduler_amd.shim.probe import run_child

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tmp():
    from k8s_vgpu_scheduler_amd.utils import build
    if not build.SHIM_SO.exists():
        build.build_all()
    return tempfile.mkdtemp(prefix="mivgpu-interpose-")


GOVERNED_25 = {"HIP_DEVICE_CORE_LIMIT": "25", "GPU_CORE_UTILIZATION_POLICY": "force"}


def test_triton_kernel_loop_held_to_its_share(tmp):
    """(a) a @triton.jit matmul loop at 25 %, policy force: 0.18-0.30 of its
    unthrottled rate, and every Triton launch counted by the shim."""
    args = ["--n", "8192", "--iters", "600"]
    free = run_child("triton", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "tf.cache")}, True, args, timeout=600)
    gov = run_child("triton", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "tg.cache"), **GOVERNED_25}, True, args,
                    timeout=600)
    assert free["rc"] == 0 and gov["rc"] == 0, (free.get("stderr"), gov.get("stderr"))
    ratio = gov["tflops"] / free["tflops"]
    print(json.dumps({"unthrottled_tflops": round(free["tflops"], 1), "governed_tflops": round(gov["tflops"], 1),
                      "ratio": round(ratio, 3), "launches": gov["shim_launches"], "gates": gov.get("gates"),
                      "held_ms": gov.get("gate_held_ms"), "rel_err": gov["rel_err"]}))
    assert free["rel_err"] < 2e-2
    assert free["shim_launches"] >= 601 and gov["shim_launches"] >= 601     # warm-up + timed loop
    assert gov["gates"] > 0 and gov["gate_held_ms"] > 0
    assert 0.18 <= ratio <= 0.30, ratio


def test_torch_compile_mlp_held_to_its_share(tmp):
    """(b) a torch.compile'd MLP (Inductor Triton GEMMs + epilogues) obeys the
    same bound.  1000 iterations (~4 s governed): the tokens the bucket earns
    while Inductor compiles on the CPU (up to its 100 ms burst) are spent at
    the start of the timed loop, which over 400 iterations read 0.31."""
    args = ["--n", "8192", "--iters", "1000"]
    free = run_child("compile", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "cf.cache")}, True, args, timeout=900)
    gov = run_child("compile", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "cg.cache"), **GOVERNED_25}, True, args,
                    timeout=900)
    assert free["rc"] == 0 and gov["rc"] == 0, (free.get("stderr"), gov.get("stderr"))
    ratio = gov["tflops"] / free["tflops"]
    print(json.dumps({"unthrottled_tflops": round(free["tflops"], 1), "governed_tflops": round(gov["tflops"], 1),
                      "ratio": round(ratio, 3), "launches": gov["shim_launches"], "gates": gov.get("gates"),
                      "held_ms": gov.get("gate_held_ms"), "received_ms": gov.get("received_ms"),
                      "sampler_state_ms": gov.get("sampler_state_ms"), "rel_err": gov["rel_err"]}))
    assert free["rel_err"] < 5e-2
    assert gov["shim_launches"] >= 400
    assert 0.18 <= ratio <= 0.30, ratio


def test_run_time_resolved_allocators_held_to_the_grant(tmp):
    """(c)+(d) a 5000 MiB hipMalloc through ctypes dlsym and through
    hipGetProcAddress, and a hipMalloc3D of the same size, all past a 4 GiB
    grant: hipErrorOutOfMemory (2); smaller ones succeed; a 1 GiB
    hipMallocArray with 0.5 GiB of the slice left: OOM."""
    r = run_child("lookup", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "lk.cache"),
                             "HIP_DEVICE_MEMORY_LIMIT_0": "4096m"}, True, ["--oom-probe-mib", "5000"])
    assert r["rc"] == 0, r.get("stderr")
    print(json.dumps(r))
    assert r["mem_total_mib"] == 4096
    assert r["dlsym_big_rc"] == 2 and r["dlsym_small_rc"] == 0
    assert r["gpa_rc"] == 0 and r["gpa_is_hook"] and r["gpa_big_rc"] == 2
    assert r["malloc3d_big_rc"] == 2 and r["malloc3d_small_rc"] == 0
    assert r["array_rc"] == 2


def test_module_bytes_reported_and_kfd_split_exact(tmp):
    """Code objects loaded with hipModuleLoadData are charged as module bytes
    (hami_vgpu_memory_module_bytes > 0); context + module + buffer + vmm is
    still KFD's per-process VRAM."""
    cache = os.path.join(tmp, "mod.cache")
    r = run_child("module", {"MIVGPU_SHARED_CACHE": cache, "HIP_DEVICE_MEMORY_LIMIT_0": "8192m"}, True,
                  ["--iters", "4"])
    assert r["rc"] == 0 and r["load_rc"] == 0, r
    print(json.dumps(r))
    assert r["module"] > 0 and r["module_after_unload"] == 0
    assert r["total"] == r["context"] + r["module"] + r["buffer"] + r["vmm"]
    assert abs(r["total"] - r["kfd_vram"]) <= 64 << 20


def test_granted_queue_cap_holds_against_the_tenant(tmp):
    """(4c) a tenant that exports GPU_MAX_HW_QUEUES=8 before importing torch
    and spreads work over 8 streams still owns at most the 2 hardware queues
    of its grant; without a grant file the same tenant gets more."""
    grant = os.path.join(tmp, "q.conf")
    with open(grant, "w") as f:
        f.write(f"GPU_MAX_HW_QUEUES=2\nMIVGPU_SHARED_CACHE={os.path.join(tmp, 'q.cache')}\n")
    capped = run_child("queues", {"MIVGPU_LIMITS_FILE": grant, "GPU_MAX_HW_QUEUES": "2"}, True, [])
    free = run_child("queues", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "qf.cache"), "GPU_MAX_HW_QUEUES": "2"},
                     True, [])
    # the same process obeying its cap: the queue count a 2-queue tenant has
    honest = run_child("queues", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "qh.cache"), "GPU_MAX_HW_QUEUES": "2"},
                       True, ["--keep-env"])
    assert capped["rc"] == 0 and free["rc"] == 0 and honest["rc"] == 0, (capped.get("stderr"), free.get("stderr"))
    print(json.dumps({"granted": capped, "ungranted": free, "honest": honest}))
    assert capped["env_seen_by_python"] == "8"
    assert 1 <= capped["kfd_queues"] <= honest["kfd_queues"], (capped, honest)      # 2 compute + 1 utility
    assert free["kfd_queues"] > honest["kfd_queues"], (free, honest)


def test_queue_cap_protects_masked_neighbours(tmp):
    """(4c) four 64-CU slices decoding; slice 0's tenant raises
    GPU_MAX_HW_QUEUES to 8 before the runtime starts.  With the queue count in
    the grant, the three other slices run within 3 % of the all-2-queue
    round."""
    from pathlib import Path

    from k8s_vgpu_scheduler_amd.bench.slices import SliceProc, plan_slices, run_round, slice_env

    def round_(tag, hostile):
        specs = plan_slices(4, shim=True, gpumem_mib=36864)
        if hostile:
            specs[0].env["MIVGPU_BENCH_TENANT_QUEUES"] = "8"
        d = Path(tmp) / tag
        d.mkdir(exist_ok=True)
        procs = [SliceProc(s, slice_env(s, None, d), ["--steps", "150", "--warmup", "5"], d / f"slice{s.index}.log")
                 for s in specs]
        return [x["tok_s"] for x in run_round(procs, load_timeout=600, run_timeout=600)["done"]]

    honest = round_("honest", False)
    hostile = round_("hostile", True)
    print(json.dumps({"all_2_queues": [round(v, 1) for v in honest], "slice0_asks_8": [round(v, 1) for v in hostile]}))
    # against the honest round's neighbour mean: one neighbour alone spreads
    # ~3 % from round to round (2444-2515 in one honest round, round 6)
    ref = sum(honest[1:]) / len(honest[1:])
    for b in hostile[1:]:
        assert b >= 0.97 * ref, (honest, hostile)


def _container(tmp, name):
    """A container's host-side state: grant file (4 GiB), control file, the
    directory its region would live in; returns (hook, grant, cache, ctl)."""
    from k8s_vgpu_scheduler_amd.monitor.control import control_host_path, create

    hook = os.path.join(tmp, f"hook-{name}")
    cdir = os.path.join(hook, "vgpu", "containers", "uid-t_main")
    ldir = os.path.join(hook, "vgpu", "limits")
    os.makedirs(cdir)
    os.makedirs(ldir)
    cache = os.path.join(cdir, "r.cache")
    ctl = control_host_path(hook, "uid-t", "main")
    create(ctl)
    grant = os.path.join(ldir, "uid-t_main.conf")
    with open(grant, "w") as f:
        f.write(f"HIP_DEVICE_MEMORY_LIMIT_0=4096m\nMIVGPU_SHARED_CACHE={cache}\nMIVGPU_DEVICE_UUIDS=GPU-tamper\n"
                f"MIVGPU_CONTROL_FILE={ctl}\n")
    return hook, grant, cache, ctl


def _kfd_vram() -> dict:
    """KFD's per-process VRAM on this box's GPU by host pid.  KFD lists every
    host process that opened /dev/kfd, other jobs on the host's other GPUs
    too (one round found a 19 GB stranger next to the hog): only ``vram_<our
    gpu_id>`` counts."""
    import glob

    from k8s_vgpu_scheduler_amd.monitor.hosttruth import single_gpu_ids

    gid = single_gpu_ids("x").get("x")
    out = {}
    for d in glob.glob("/sys/class/kfd/kfd/proc/*"):
        try:
            out[int(os.path.basename(d))] = int(open(os.path.join(d, f"vram_{gid}")).read().strip() or 0)
        except (OSError, ValueError):
            pass
    return out


def _spawn_hog(mib):
    """A container process without the shim holding ``mib`` MiB; its KFD
    (host) pid: the one new KFD process entry holding that much (found from
    here, the box may run us in a pid namespace)."""
    before = set(_kfd_vram())
    p, info = _spawn(["--child", "hog", "--oom-probe-mib", str(mib)], dict(os.environ), "HOG")
    new = {pid: v for pid, v in _kfd_vram().items() if pid not in before and v >= mib << 20}
    assert len(new) == 1, (new, info)
    info["kfd_pid"] = next(iter(new))
    return p, info


def _spawn(args, env, tag):
    import subprocess
    import sys

    p = subprocess.Popen([sys.executable, "-m", "k8s_vgpu_scheduler_amd.shim.probe"] + args, env=env,
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    assert line.startswith(tag + " "), (line, p.stderr.read()[-2000:] if p.poll() is not None else "")
    return p, json.loads(line[len(tag) + 1:])


def _monitor(hook, api, pids, passes):
    from k8s_vgpu_scheduler_amd.k8s.rest import RestClient
    from k8s_vgpu_scheduler_amd.monitor import feedback
    from k8s_vgpu_scheduler_amd.monitor.escalate import OverGrantPolicy
    from k8s_vgpu_scheduler_amd.monitor.hosttruth import HostTruth, single_gpu_ids
    from k8s_vgpu_scheduler_amd.monitor.lister import ContainerLister

    lister = ContainerLister(hook, lambda: api.cluster.list("pods"), resync_interval=3600)
    # the pod's processes as a hostPID monitor's cgroup scan finds them: KFD's
    # (host) pids of the children stand in (the box may run us in a pid namespace)
    truth = HostTruth(lambda: single_gpu_ids("GPU-tamper"), pod_pids=lambda uid: pids)
    pol = OverGrantPolicy("evict", passes=passes, client=RestClient(api.url))
    outs = [feedback.feedback_pass(lister, truth, pol) for _ in range(passes)]
    gid = single_gpu_ids("GPU-tamper")["GPU-tamper"]
    print(json.dumps({"pids": pids, "kfd_vram_mib": {p: truth.vram(p, gid) >> 20 for p in pids}}))
    return outs


def _api():
    from k8s_vgpu_scheduler_amd.e2e.apiserver import FakeApiServer
    from k8s_vgpu_scheduler_amd.k8s.fake import make_pod

    api = FakeApiServer().start()
    pod = make_pod("t", "default")
    pod["metadata"]["uid"] = "uid-t"
    api.cluster.create("pods", pod)
    return api


def test_tenant_without_the_shim_reported_within_one_pass(tmp):
    """a container process the shim is not loaded into
    (no region file ever exists: an image whose loader ignored the preload)
    allocates past its 4 GiB grant.  ONE monitor pass, driven by the grant
    file and KFD, reports it over its grant and shim-less, and the evict
    escalation reaches the API server's Eviction endpoint."""
    hook, grant, cache, ctl = _container(tmp, "noshim")
    from k8s_vgpu_scheduler_amd.monitor.control import ControlFile

    api = _api()
    hog = None
    try:
        hog, info = _spawn_hog(4608)
        outs = _monitor(hook, api, [info["kfd_pid"]], passes=1)
        snap = ControlFile(ctl).snapshot()
        evictions = list(api.cluster.evictions)
    finally:
        if hog is not None:
            hog.communicate("go\n", timeout=60)
        api.stop()
    print(json.dumps({"over": sorted(outs[0]["over"]), "no_shim": sorted(outs[0]["no_shim"]),
                      "control": {k: snap[k] for k in ("block", "over_grant")},
                      "excess_mib": snap["host_excess"][0] >> 20, "evictions": evictions}))
    assert not os.path.exists(cache)
    assert ("uid-t", "main") in outs[0]["over"] and ("uid-t", "main") in outs[0]["no_shim"]
    assert evictions == [("default", "t")]
    assert snap["block"] == 1 and snap["over_grant"] == 1 and snap["host_excess"][0] > 4 << 30


def test_tenant_rewriting_its_region_cannot_unblock_itself(tmp):
    """A shim-loaded tenant zeroes its region's usage counters and tries to
    allocate past its grant: refused (the shim charges the VRAM KFD shows
    for it).  A sibling process without the shim then takes the container
    over its grant; two monitor passes block the container through the
    read-only control file and evict it.  The tenant keeps clearing its
    region's block flag and counters from a thread: its allocations are
    still refused and its launches stay parked until the verdict is lifted."""
    hook, grant, cache, ctl = _container(tmp, "rewrite")
    from k8s_vgpu_scheduler_amd.monitor.control import ControlFile
    from k8s_vgpu_scheduler_amd.shim import shim_env

    env = dict(os.environ)
    env.update(shim_env())
    env["MIVGPU_LIMITS_FILE"] = grant
    api = _api()
    tam = hog = None
    se = ""
    try:
        tam, first = _spawn(["--child", "tamper", "--out", cache, "--oom-probe-mib", "3500"], env, "TAMPERED")
        hog, info = _spawn_hog(4096)
        outs = _monitor(hook, api, [first["kfd_pid"], info["kfd_pid"]], passes=2)
        snap = ControlFile(ctl).snapshot()
        tam.stdin.write("go\n")
        tam.stdin.flush()
        time.sleep(3.0)                       # the tenant rewrites its region meanwhile
        ControlFile(ctl).publish(block=False, switch=False, over=False)   # the verdict lifted
        so, se = tam.communicate(timeout=120)
        evictions = list(api.cluster.evictions)
    finally:
        for p in (tam, hog):
            if p is not None and p.poll() is None:
                try:
                    p.communicate("go\n", timeout=60)
                except Exception:
                    p.kill()
        api.stop()
    assert tam.returncode == 0, se[-3000:]
    res = json.loads([x for x in so.splitlines() if x.startswith("{")][-1])
    print(json.dumps({"over": sorted(outs[-1]["over"]), "control": {k: snap[k] for k in ("block", "over_grant")},
                      "excess_mib": snap["host_excess"][0] >> 20, "evictions": evictions, "child": res}))
    assert first["first"] == "oom"            # the counter rewrite bought no headroom
    assert ("uid-t", "main") in outs[-1]["over"] and not outs[-1]["no_shim"]
    assert snap["block"] == 1 and snap["over_grant"] == 1
    assert evictions == [("default", "t")]
    assert res["second"] == "oom" and res["parked_s"] >= 2.5
