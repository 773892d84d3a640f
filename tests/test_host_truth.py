"""Host-truth HBM accounting (monitor/hosttruth.py; VERDICT r2 weak #3a).

The shared region is tenant-writable: a tenant that zeroes ``dev_used`` and
its slot totals, or raises ``mem_limit``, would allocate past its grant.  Each
monitor pass recomputes usage from KFD's per-process VRAM (simulated here
under a fake KFD root) and blocks a container over its grant.
"""

from __future__ import annotations

import os

from prometheus_client import CollectorRegistry, generate_latest

from k8s_vgpu_scheduler_amd.monitor import feedback
from k8s_vgpu_scheduler_amd.monitor.hosttruth import OVER_GRANT_REASON, HostTruth
from k8s_vgpu_scheduler_amd.monitor.lister import ContainerLister
from k8s_vgpu_scheduler_amd.monitor.metrics import MonitorCollector
from k8s_vgpu_scheduler_amd.scheduler.events import EventRecorder

from test_monitor import make_container, pod

GIB = 1 << 30


def _kfd(root, pid, gid, vram):
    d = root / "proc" / str(pid)
    d.mkdir(parents=True, exist_ok=True)
    (d / f"vram_{gid}").write_text(f"{vram}\n")


def _grant(base, uid, ctr, limit_mib):
    d = base / "vgpu" / "limits"
    d.mkdir(parents=True, exist_ok=True)
    (d / f"{uid}_{ctr}.conf").write_text(f"HIP_DEVICE_MEMORY_LIMIT_0={limit_mib}m\n")


def _setup(tmp_path, vram, limit=4 * GIB, tamper=True):
    kfd = tmp_path / "kfd"
    _kfd(kfd, 4711, 42, vram)
    _kfd(kfd, 4712, 42, 7 * GIB)        # a process of ANOTHER pod on the same GPU
    _grant(tmp_path, "u1", "main", limit >> 20)
    r = make_container(tmp_path, "u1", "main", uuid="GPU-aa", used=GIB, limit=limit)
    if tamper:
        r.r.dev_used[0] = 0
        r.r.mem_limit[0] = 1 << 40
        r.r.procs[0].used[0].total = 0
        r.r.procs[0].used[0].buffer = 0
    r.r.procs[0].hostpid = 4711
    r.close()
    lister = ContainerLister(str(tmp_path), lambda: [pod("u1", "p1")], resync_interval=3600)
    events = EventRecorder(None)
    truth = HostTruth(lambda: {"GPU-aa": 42}, kfd_root=kfd, pod_pids=lambda uid: [4711] if uid == "u1" else [],
                      events=events)
    return kfd, lister, truth, events


def test_tampered_counters_restored_and_over_grant_blocked(tmp_path):
    kfd, lister, truth, events = _setup(tmp_path, vram=6 * GIB)
    out = feedback.feedback_pass(lister, truth)
    c = lister.list_containers()[0]
    r = c.region.r
    assert r.mem_limit[0] == 4 * GIB                     # limits back from the grant file
    assert r.dev_used[0] == 6 * GIB                      # usage back from KFD
    assert r.procs[0].used[0].total == 6 * GIB           # slot total too (excess charged as context)
    assert r.procs[0].used[0].context == 6 * GIB
    assert out["over"] == {("u1", "main")}
    assert r.recent_kernel == -1                         # launches parked
    assert [e[0] for e in events.recorded] == [OVER_GRANT_REASON]
    # the next pass keeps it blocked (the priority feedback must not unblock it) and does not repeat the event
    feedback.feedback_pass(lister, truth)
    assert r.recent_kernel == -1 and len(events.recorded) == 1
    # back under its grant: unblocked
    _kfd(kfd, 4711, 42, 3 * GIB)
    out = feedback.feedback_pass(lister, truth)
    assert out["over"] == set() and r.recent_kernel == 0


def test_within_grant_nothing_blocked_and_usage_never_lowered(tmp_path):
    kfd, lister, truth, events = _setup(tmp_path, vram=2 * GIB, tamper=False)
    c_ = None
    feedback.feedback_pass(lister, truth)
    c_ = lister.list_containers()[0]
    assert c_.region.r.dev_used[0] == 2 * GIB and c_.region.r.recent_kernel >= 0
    # KFD lags a reservation the shim already made: the region keeps the higher count
    c_.region.r.dev_used[0] = 3 * GIB
    feedback.feedback_pass(lister, truth)
    assert c_.region.r.dev_used[0] == 3 * GIB
    assert events.recorded == []


def test_other_pods_processes_are_not_charged(tmp_path):
    kfd, lister, truth, _ = _setup(tmp_path, vram=GIB)
    feedback.feedback_pass(lister, truth)
    assert truth.snapshot()[0] == {("u1", "main", 0): GIB}     # pid 4712's 7 GiB belongs to another pod


def test_hidden_process_in_a_multi_container_pod(tmp_path):
    """Two containers of one pod on one GPU; a pod process that sits in no
    slot (it unloaded or zeroed the shim) holds VRAM: over the pod's total
    grant, both containers are blocked."""
    kfd = tmp_path / "kfd"
    for pid, v in ((5001, GIB), (5002, GIB), (5003, 5 * GIB)):
        _kfd(kfd, pid, 42, v)
    for ctr, pid in (("a", 5001), ("b", 5002)):
        _grant(tmp_path, "u9", ctr, 2048)
        r = make_container(tmp_path, "u9", ctr, uuid="GPU-aa", used=GIB, limit=2 * GIB)
        r.r.procs[0].hostpid = pid
        r.close()
    lister = ContainerLister(str(tmp_path), lambda: [pod("u9", "p9")], resync_interval=3600)
    truth = HostTruth(lambda: {"GPU-aa": 42}, kfd_root=kfd, pod_pids=lambda uid: [5001, 5002, 5003])
    out = feedback.feedback_pass(lister, truth)
    assert out["over"] == {("u9", "a"), ("u9", "b")}
    assert truth.snapshot()[0][("u9", "a", 0)] == GIB        # each container: its own processes
    # without the hidden process both are within their grants
    os.unlink(kfd / "proc" / "5003" / "vram_42")
    assert feedback.feedback_pass(lister, truth)["over"] == set()


def test_metrics_export_host_truth_and_over_grant(tmp_path):
    kfd, lister, truth, _ = _setup(tmp_path, vram=6 * GIB)
    feedback.feedback_pass(lister, truth)
    reg = CollectorRegistry()
    reg.register(MonitorCollector(lister, None, "n1", truth=truth))
    text = generate_latest(reg).decode()
    assert 'mivgpu_container_memory_host_bytes{container="main"' in text
    line = [l for l in text.splitlines() if l.startswith("mivgpu_container_memory_over_grant{")][0]
    assert line.endswith(" 1.0")
