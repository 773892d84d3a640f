"""vGPU monitor: lister, GC, feedback loop and metrics (cudevshr_test.go, feedback_test.go, metrics_test.go)."""

import os
import time

from prometheus_client import CollectorRegistry, generate_latest

from k8s_vgpu_scheduler_amd.monitor import feedback
from k8s_vgpu_scheduler_amd.monitor.lister import ContainerLister
from k8s_vgpu_scheduler_amd.monitor.metrics import MonitorCollector
from k8s_vgpu_scheduler_amd.monitor.region import REGION_SIZE, SharedRegion
from k8s_vgpu_scheduler_amd.smi import FakeBackend


def make_container(base, uid, ctr, uuid="GPU-0000", priority=1, used=0, limit=1 << 30, recent=0):
    d = base / "vgpu" / "containers" / f"{uid}_{ctr}"
    d.mkdir(parents=True, exist_ok=True)
    r = SharedRegion.create(str(d / "x.cache"), num_devices=1, mem_limit=limit)
    r.r.uuids[0].value = uuid.encode()
    r.r.priority = priority
    r.r.procnum = 1
    p = r.r.procs[0]
    p.pid, p.status = os.getpid(), 1
    p.used[0].total = used
    p.used[0].buffer = used
    r.r.recent_kernel = recent
    r.r.last_kernel_time = int(time.time()) - 7
    return r


def pod(uid, name, ns="default"):
    return {"metadata": {"uid": uid, "name": name, "namespace": ns}}


def test_region_size_is_stable():
    # 16-device header + 1024 x 2112-byte process slots; also pinned against the
    # C layout by test_shim_cpu.py::test_abi_offsets_match_c_layout
    assert REGION_SIZE == 2173200


def test_lister_maps_and_gcs(tmp_path):
    make_container(tmp_path, "u1", "main").close()
    make_container(tmp_path, "u2", "main").close()
    pods = [pod("u1", "p1")]
    lister = ContainerLister(str(tmp_path), lambda: pods, resync_interval=0)
    lister.update()
    names = {c.pod_name for c in lister.list_containers()}
    assert names == {"p1"}
    assert not (tmp_path / "vgpu" / "containers" / "u2_main").exists()   # stale dir removed
    assert (tmp_path / "vgpu" / "containers" / "u1_main").exists()


def test_lister_keeps_recent_stale_dirs(tmp_path):
    make_container(tmp_path, "u2", "main").close()
    lister = ContainerLister(str(tmp_path), lambda: [], resync_interval=3600)
    lister.update()
    assert (tmp_path / "vgpu" / "containers" / "u2_main").exists()


def test_lister_skips_corrupt_cache(tmp_path):
    d = tmp_path / "vgpu" / "containers" / "u3_c"
    d.mkdir(parents=True)
    (d / "bad.cache").write_bytes(b"\0" * 100)
    lister = ContainerLister(str(tmp_path), None)
    lister.update()
    assert lister.list_containers() == []


def test_feedback_blocks_lower_priority(tmp_path):
    hi = make_container(tmp_path, "h", "c", priority=0, recent=2)
    lo = make_container(tmp_path, "l", "c", priority=1, recent=2)
    lister = ContainerLister(str(tmp_path), lambda: [pod("h", "hi"), pod("l", "lo")])
    lister.update()
    feedback.observe(lister)
    by = {c.pod_name: c.region for c in lister.list_containers()}
    assert by["lo"].recent_kernel() == -1          # blocked by the active priority-0 task
    assert by["lo"].utilization_switch() == 1
    assert by["hi"].recent_kernel() >= 0
    assert by["hi"].utilization_switch() == 0
    # high-priority task goes idle -> unblocked after decay
    by["hi"].set_recent_kernel(0)
    feedback.observe(lister)
    assert by["lo"].recent_kernel() == 0
    hi.close()
    lo.close()


def test_feedback_same_priority_switches_core_limit_on(tmp_path):
    make_container(tmp_path, "a", "c", priority=1, recent=2).close()
    make_container(tmp_path, "b", "c", priority=1, recent=2).close()
    lister = ContainerLister(str(tmp_path), lambda: [pod("a", "a"), pod("b", "b")])
    lister.update()
    feedback.observe(lister)
    for c in lister.list_containers():
        assert c.region.utilization_switch() == 1
        assert c.region.recent_kernel() == 1   # decayed, not blocked


def test_metrics_series_and_labels(tmp_path):
    make_container(tmp_path, "u1", "main", uuid="GPU-0001", used=300 << 20, limit=2 << 30).close()
    lister = ContainerLister(str(tmp_path), lambda: [pod("u1", "p1", "ns1")])
    lister.update()
    be = FakeBackend(n=2)
    be.used["GPU-0000"] = 1024
    reg = CollectorRegistry()
    reg.register(MonitorCollector(lister, be, "node1"))
    text = generate_latest(reg).decode()
    assert 'hami_vgpu_memory_used_bytes{container="main",device_uuid="GPU-0001",namespace="ns1",pod="p1",vdevice_index="0"} 3.145728e+08' in text
    assert 'hami_vgpu_memory_limit_bytes{' in text and "2.147483648e+09" in text
    assert 'hami_host_gpu_memory_used_bytes{device_index="0",device_type="AMD Instinct MI355X",device_uuid="GPU-0000",node="node1"} 1.073741824e+09' in text
    assert "hami_container_last_kernel_elapsed_seconds" in text
    assert "mivgpu_container_throttled_seconds_total" in text


def test_context_bytes_split_out_of_the_usage(tmp_path):
    """Runtime VRAM the shim charges as context shows in hami_vgpu_memory_context_bytes,
    inside the used total, and not in the buffer series."""
    r = make_container(tmp_path, "u2", "main", uuid="GPU-0002", used=0, limit=4 << 30)
    p = r.r.procs[0]
    p.used[0].buffer, p.used[0].context = 1 << 30, 490 << 20
    p.used[0].total = (1 << 30) + (490 << 20)
    r.close()
    lister = ContainerLister(str(tmp_path), lambda: [pod("u2", "p2", "ns2")])
    lister.update()
    reg = CollectorRegistry()
    reg.register(MonitorCollector(lister, FakeBackend(n=1), "node1"))
    text = generate_latest(reg).decode()
    lab = '{container="main",device_uuid="GPU-0002",namespace="ns2",pod="p2",vdevice_index="0"}'
    assert f"hami_vgpu_memory_context_bytes{lab} 5.1380224e+08" in text
    assert f"hami_vgpu_memory_buffer_bytes{lab} 1.073741824e+09" in text
    assert f"hami_vgpu_memory_used_bytes{lab} 1.587544064e+09" in text


def test_active_tenants_from_the_share_board(tmp_path, monkeypatch):
    """mivgpu_host_gpu_active_tenants counts board slots stamped in the last second."""
    import struct

    from k8s_vgpu_scheduler_amd.monitor import board as B

    monkeypatch.setenv("MIVGPU_LOCK_DIR", str(tmp_path / "lock"))
    (tmp_path / "lock").mkdir()
    be = FakeBackend(n=2)
    g0 = be.gpus()[0]
    path = B.board_path(g0.bdf)
    assert path.name == "mivgpu-board-0000-11-00-0"
    now = B.now_ns()
    slots = [(7, now - 10 ** 8), (8, now - 5 * 10 ** 8), (9, now - 5 * 10 ** 9), (0, now)] + [(0, 0)] * 60
    path.write_bytes(b"".join(struct.pack("<QQ", t, l) for t, l in slots))
    assert B.active_tenants(path, at_ns=now) == 2
    lister = ContainerLister(str(tmp_path), lambda: [])
    reg = CollectorRegistry()
    reg.register(MonitorCollector(lister, be, "node1"))
    text = generate_latest(reg).decode()
    assert 'mivgpu_host_gpu_active_tenants{device_index="0",device_uuid="GPU-0000",node="node1"} 2.0' in text
    assert 'device_index="1"' not in text.split("mivgpu_host_gpu_active_tenants")[-1]   # no board, no series


def test_feedback_loop_fills_host_pids(tmp_path, monkeypatch):
    """watch_and_feedback maps every new slot to its host pid on each pass."""
    import threading

    from k8s_vgpu_scheduler_amd.monitor import hostpid

    uid = "11111111-2222-3333-4444-555555555555"
    r = make_container(tmp_path, uid, "main")
    r.r.procs[0].pid = 42
    r.close()
    monkeypatch.setattr(hostpid, "scan", lambda proc_root="/proc": [(90042, 42, f"0::/kubepods/pod{uid}/c\n")])
    lister = ContainerLister(str(tmp_path), lambda: [pod(uid, "p")])
    stop = threading.Event()
    t = threading.Thread(target=feedback.watch_and_feedback, args=(lister, stop, 0.05), daemon=True)
    t.start()
    deadline = time.time() + 10
    while time.time() < deadline:
        cs = lister.list_containers()
        if cs and cs[0].region.r.procs[0].hostpid == 90042:
            break
        time.sleep(0.05)
    stop.set()
    t.join(timeout=5)
    assert lister.list_containers()[0].region.r.procs[0].hostpid == 90042
