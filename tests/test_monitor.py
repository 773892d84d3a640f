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


def test_lister_refuses_planted_symlinks_and_fifos(tmp_path):
    """The cache directory is writable by the container: a region "file" that
    is a symlink to a host file or a FIFO must never be mapped (let alone
    written) by the privileged monitor."""
    victim = tmp_path / "host_file"
    victim.write_bytes(b"\1" * (REGION_SIZE + 10))
    d = tmp_path / "vgpu" / "containers" / "u9_c"
    d.mkdir(parents=True)
    os.symlink(victim, d / "x.cache")
    f = tmp_path / "vgpu" / "containers" / "u8_c"
    f.mkdir(parents=True)
    os.mkfifo(f / "y.cache")
    lister = ContainerLister(str(tmp_path), None)
    lister.update()
    assert lister.list_containers() == []
    assert victim.read_bytes() == b"\1" * (REGION_SIZE + 10)


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


def fake_kfd(root, occ: dict, bdf_loc=(0x11 << 8), gpu_id=4242):
    """A KFD sysfs tree: one GPU node at PCI 0000:11:00.0 (FakeBackend GPU 0) and
    ``occ`` = {host pid: cu_occupancy} on it."""
    n = root / "topology" / "nodes" / "2"
    n.mkdir(parents=True)
    (n / "gpu_id").write_text(f"{gpu_id}\n")
    (n / "properties").write_text(f"simd_count 1024\nsimd_per_cu 4\nlocation_id {bdf_loc}\ndomain 0\n")
    cpu = root / "topology" / "nodes" / "0"
    cpu.mkdir(parents=True)
    (cpu / "gpu_id").write_text("0\n")
    for pid, v in occ.items():
        d = root / "proc" / str(pid) / f"stats_{gpu_id}"
        d.mkdir(parents=True)
        (d / "cu_occupancy").write_text(f"{v}\n")
    return gpu_id


def test_active_tenants_from_kfd_wave_occupancy(tmp_path):
    """mivgpu_host_gpu_active_tenants counts the processes with waves resident on
    the GPU (KFD cu_occupancy) in the sampling window."""
    from k8s_vgpu_scheduler_amd.monitor.occupancy import OccupancySampler, gpu_ids_by_bdf

    kfd = tmp_path / "kfd"
    gid = fake_kfd(kfd, {100: 12, 101: 0, 102: 4})
    assert gpu_ids_by_bdf(kfd) == {"0000:11:00.0": gid}
    occ = OccupancySampler(root=kfd)
    occ.sample_once()
    assert occ.active_tenants(gid) == 2
    assert occ.share_pct(gid, [100]) == 75.0
    lister = ContainerLister(str(tmp_path), lambda: [])
    reg = CollectorRegistry()
    reg.register(MonitorCollector(lister, FakeBackend(n=2), "node1", occupancy=occ))
    text = generate_latest(reg).decode()
    assert 'mivgpu_host_gpu_active_tenants{device_index="0",device_uuid="GPU-0000",node="node1"} 2.0' in text
    assert 'device_index="1"' not in text.split("mivgpu_host_gpu_active_tenants")[-1]   # no KFD node, no series


def test_container_utilization_from_shim_or_kfd(tmp_path):
    """hami_container_device_utilization_ratio: the shim's own occupancy share
    (util_pct) when it reports one, else the monitor's KFD sample of the
    container's host pids (metrics.go:468-497 exports DeviceSmUtil)."""
    from k8s_vgpu_scheduler_amd.monitor.occupancy import OccupancySampler

    kfd = tmp_path / "kfd"
    fake_kfd(kfd, {100: 12, 102: 4})
    occ = OccupancySampler(root=kfd)
    occ.sample_once()
    busy = make_container(tmp_path, "u1", "main", uuid="GPU-0000")
    busy.r.procs[0].hostpid = 100                    # no shim util: monitor's KFD share 12 / 16
    busy.close()
    rep = make_container(tmp_path, "u2", "main", uuid="GPU-0000")
    rep.r.procs[0].util[0].share_ns, rep.r.procs[0].util[0].util_pct = 5 * 10 ** 9, 40
    rep.r.procs[0].util[0].share_ppm, rep.r.procs[0].util[0].occupancy = 250_000, 64
    rep.close()
    idle = make_container(tmp_path, "u3", "main", uuid="GPU-0000")
    idle.r.procs[0].hostpid = 999                    # holds the GPU, no waves
    idle.close()
    lister = ContainerLister(str(tmp_path), lambda: [pod("u1", "busy"), pod("u2", "rep"), pod("u3", "idle")])
    lister.update()
    reg = CollectorRegistry()
    reg.register(MonitorCollector(lister, FakeBackend(n=1), "node1", occupancy=occ))
    text = generate_latest(reg).decode()

    def util(p):
        pre = f'hami_container_device_utilization_ratio{{container="main",device_uuid="GPU-0000",namespace="default",pod="{p}",vdevice_index="0"}} '
        return float(text.split(pre)[1].split()[0])
    assert util("busy") == 75.0
    assert util("rep") == 40.0
    assert util("idle") == 0.0
    # the governor's measured share and last wave sample, as the shim published them
    lab = 'container="main",device_uuid="GPU-0000",namespace="default",pod="rep",vdevice_index="0"'
    assert f"mivgpu_container_gpu_share_ratio{{{lab}}} 25.0" in text
    assert f"mivgpu_container_wave_occupancy{{{lab}}} 64.0" in text
    assert 'mivgpu_container_gpu_share_ratio{container="main",device_uuid="GPU-0000",namespace="default",pod="idle"' not in text


def test_partition_info_and_legacy_series(tmp_path):
    """Per-container partition identity (the hami_mig_device_info analogue) and
    the --legacy-metrics names (cmd/vGPUmonitor/metrics.go:133-212)."""
    make_container(tmp_path, "u1", "main", uuid="GPU-0001-cpx3", used=300 << 20, limit=2 << 30).close()
    lister = ContainerLister(str(tmp_path), lambda: [pod("u1", "p1", "ns1")])
    lister.update()
    be = FakeBackend(n=2)
    be.modes[1] = "CPX"
    reg = CollectorRegistry()
    reg.register(MonitorCollector(lister, be, "node1", legacy=True))
    text = generate_latest(reg).decode()
    assert ('mivgpu_container_partition_info{compute_partition="CPX",container="main",cus="32",'
            'device_uuid="GPU-0001-cpx3",memory_partition="NPS1",namespace="ns1",partition_index="3",'
            'physical_index="1",pod="p1",vdevice_index="0"} 1.0') in text
    # the reference's series for the same identity (hami_mig_device_info)
    assert ('hami_mig_device_info{compute_instance_id="0",container="main",device_uuid="GPU-0001-cpx3",'
            'gpu_instance_id="3",mig_uuid="GPU-0001-cpx3",namespace="ns1",pod="p1",profile="cpx.32cu",'
            'vdevice_index="0"} 1.0') in text
    assert 'vGPU_device_memory_usage_in_bytes{ctrname="main",deviceuuid="GPU-0001-cpx3",podname="p1",podnamespace="ns1",vdeviceid="0"} 3.145728e+08' in text
    assert 'vGPU_device_memory_limit_in_bytes{' in text
    assert 'Device_memory_desc_of_container{context="0",ctrname="main",data="314572800"' in text
    assert 'HostGPUMemoryUsage{deviceidx="0"' in text and "HostCoreUtilization{" in text
    reg2 = CollectorRegistry()
    reg2.register(MonitorCollector(lister, be, "node1"))
    assert "HostGPUMemoryUsage" not in generate_latest(reg2).decode()


def test_region_limits_reconciled_against_the_grant(tmp_path):
    """A tenant that rewrites its region's limits (the region file is in a
    read-write mount) is put back to the grant the device plugin wrote."""
    from k8s_vgpu_scheduler_amd.deviceplugin.allocate import grant_text

    make_container(tmp_path, "u1", "main", limit=1 << 30).close()
    limits = tmp_path / "vgpu" / "limits"
    limits.mkdir(parents=True)
    (limits / "u1_main.conf").write_text(grant_text({
        "HIP_DEVICE_MEMORY_LIMIT_0": "1024m", "HSA_CU_MASK": "0:0-63", "HIP_DEVICE_CORE_LIMIT": "25",
        "MIVGPU_SHARED_CACHE": "/usr/local/vgpu/x.cache", "NOT_A_GRANT_KEY": "1"}))
    assert "NOT_A_GRANT_KEY" not in (limits / "u1_main.conf").read_text()
    lister = ContainerLister(str(tmp_path), lambda: [pod("u1", "p1")])
    lister.update()
    r = lister.list_containers()[0].region
    r.r.cu_limit[0], r.r.cu_mask_count[0] = 25, 64
    assert feedback.reconcile_limits(lister) == 0          # consistent: nothing to do
    r.r.mem_limit[0], r.r.cu_limit[0], r.r.cu_mask_count[0], r.r.core_policy = 64 << 30, 100, 0, 2
    assert feedback.reconcile_limits(lister) == 4
    assert (r.r.mem_limit[0], r.r.cu_limit[0], r.r.cu_mask_count[0], r.r.core_policy) == (1 << 30, 25, 64, 0)


def test_feedback_pauses_while_a_partition_apply_holds_the_lock(tmp_path):
    """cmd/vGPUmonitor/main.go:79-109: no feedback pass while the device plugin
    reconfigures compute partitions."""
    import threading

    from k8s_vgpu_scheduler_amd.cmd.monitor import watch_partition_lock

    lock = tmp_path / "lockdir" / "partition-apply.lock"
    lock.parent.mkdir()
    pause, stop = threading.Event(), threading.Event()
    t = threading.Thread(target=watch_partition_lock, args=(pause, stop, str(lock), 0.02), daemon=True)
    t.start()
    lock.write_text("applying")
    deadline = time.time() + 5
    while not pause.is_set() and time.time() < deadline:
        time.sleep(0.02)
    assert pause.is_set()
    # a paused loop does not touch the regions
    make_container(tmp_path, "a", "c", priority=1, recent=2).close()
    make_container(tmp_path, "b", "c", priority=1, recent=2).close()
    lister = ContainerLister(str(tmp_path), lambda: [pod("a", "a"), pod("b", "b")])
    lister.update()
    fb_stop = threading.Event()
    fb = threading.Thread(target=feedback.watch_and_feedback, args=(lister, fb_stop, 0.02, pause), daemon=True)
    fb.start()
    time.sleep(0.3)
    assert all(c.region.utilization_switch() == 0 for c in lister.list_containers())
    lock.unlink()
    deadline = time.time() + 5
    while time.time() < deadline and not all(c.region.utilization_switch() == 1 for c in lister.list_containers()):
        time.sleep(0.02)
    assert not pause.is_set()
    assert all(c.region.utilization_switch() == 1 for c in lister.list_containers())
    stop.set()
    fb_stop.set()


def test_node_scoped_pod_informer():
    """The monitor watches only its node's pods (field selector spec.nodeName,
    pkg/monitor/nvidia/cudevshr.go:308); a pod bound to the node later enters
    the cache, one deleted leaves it."""
    from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
    from k8s_vgpu_scheduler_amd.k8s.informer import Informer

    kc = FakeCluster()
    mk = lambda n, node: {"metadata": {"name": n, "namespace": "d", "uid": n}, "spec": {"nodeName": node}}  # noqa: E731
    kc.create("pods", mk("here", "n1"))
    kc.create("pods", mk("there", "n2"))
    kc.create("pods", mk("pending", ""))
    inf = Informer(kc, "pods", field_selector={"spec.nodeName": "n1"})
    inf.start()
    assert [p["metadata"]["name"] for p in inf.list()] == ["here"]
    kc.patch("pods", "pending", {"spec": {"nodeName": "n1"}}, "d")
    assert sorted(p["metadata"]["name"] for p in inf.list()) == ["here", "pending"]
    kc.patch("pods", "there", {"metadata": {"labels": {"x": "1"}}}, "d")   # other node: never seen
    assert "there" not in [p["metadata"]["name"] for p in inf.list()]
    kc.delete("pods", "here", "d")
    assert [p["metadata"]["name"] for p in inf.list()] == ["pending"]


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
