"""Compute partitions (SPX/DPX/QPX/CPX): enumeration, registration, scheduling
with amd.com/vgpu-mode, Allocate inside a partition, and the partition manager
(the MIG-manager analog: apply when idle, busy/locked status, apply lock)."""

import tempfile

import pytest

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device.amd.device import IN_REQUEST_ANNOS, REGISTER_ANNOS, SUPPORT_ANNOS
from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.deviceplugin import partition as P
from k8s_vgpu_scheduler_amd.deviceplugin import server as S
from k8s_vgpu_scheduler_amd.deviceplugin.allocate import PluginConfig
from k8s_vgpu_scheduler_amd.deviceplugin.register import Registrar
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster, make_node
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.smi import FakeBackend, PartitionError
from k8s_vgpu_scheduler_amd.testing import amd_container, amd_pod


@pytest.fixture
def env(monkeypatch, tmp_path):
    monkeypatch.setenv("MIVGPU_DP_DRY_RUN", "1")
    lock = str(tmp_path / "apply.lock")
    monkeypatch.setattr(P, "APPLY_LOCK", lock)
    monkeypatch.setattr(P.is_applying, "__defaults__", (lock,))
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    c.create("nodes", make_node("node1", capacity={"amd.com/gpu": "256"}))
    backend = FakeBackend(n=4)
    backend.set_compute_partition(0, "CPX")
    cfg = PluginConfig(hook_path=tempfile.mkdtemp(), device_split_count=8)
    reg = Registrar(backend, cfg, "node1")
    reg.register_once()
    sched = Scheduler(c, SchedulerConfig())
    sched.start()
    sched.register()
    return c, sched, backend, cfg, reg, lock


def _schedule(c, sched, pod):
    c.create("pods", pod)
    name = pod["metadata"]["name"]
    res = sched.filter({"Pod": c.get_pod("default", name), "NodeNames": ["node1"]})
    if not res["NodeNames"]:
        return None
    p = c.get_pod("default", name)
    assert sched.bind({"PodName": name, "PodNamespace": "default", "PodUID": p["metadata"]["uid"],
                       "Node": "node1"})["Error"] == ""
    return c.get_pod("default", name)


def test_fake_partition_enumeration():
    b = FakeBackend(n=2)
    for mode, parts in (("DPX", 2), ("QPX", 4), ("CPX", 8), ("SPX", 1)):
        b.set_compute_partition(1, mode)
        gs = [g for g in b.gpus() if g.physical == 1]
        assert len(gs) == parts and all(g.cus == 256 // parts and g.memory_mib == 294912 // parts for g in gs)
        assert len({g.render_minor for g in b.gpus()}) == len(b.gpus())
    with pytest.raises(PartitionError):
        b.set_compute_partition(1, "XPX")


def test_registration_publishes_partitions(env):
    c, sched, backend, cfg, reg, _ = env
    devs = codec.unmarshal_node_devices(c.get_node("node1")["metadata"]["annotations"][REGISTER_ANNOS])
    cpx = [d for d in devs if d.mode == "cpx"]
    assert len(devs) == 8 + 3 and len(cpx) == 8
    assert all(d.devcore == 32 and d.devmem == 36864 for d in cpx)
    assert {d.mode for d in devs} == {"cpx", "hami-core"}


def test_vgpu_mode_annotation_selects_partitions(env, monkeypatch):
    c, sched, backend, cfg, reg, _ = env
    pod = _schedule(c, sched, amd_pod("p", annotations={"amd.com/vgpu-mode": "cpx"}, mem=8192, cores=25))
    dev = codec.decode_container_devices(pod["metadata"]["annotations"][SUPPORT_ANNOS].split(";")[0])[0]
    assert "-cpx" in dev.uuid and dev.usedcores == 8            # 25 % of a 32-CU partition
    ranges = codec.decode_cu_ranges(pod["metadata"]["annotations"]["hami.io/amd-cu-ranges"])[0][dev.uuid]
    assert codec.ranges_count(ranges) == 8 and ranges[0][0] == 0  # one XCD: plain CU indices
    # the device plugin turns it into a mask inside the partition
    plugin = S.AMDDevicePlugin(backend, cfg, "node1", socket_dir=tempfile.mkdtemp())
    res = plugin.allocate([["x"]])
    assert res[0]["envs"]["HSA_CU_MASK"] == "0:0-7"
    assert res[0]["envs"]["ROCR_VISIBLE_DEVICES"] == dev.uuid
    # a shared-mode pod never lands on a partition, a whole-card one takes an SPX GPU
    whole = _schedule(c, sched, amd_pod("w", annotations={"amd.com/vgpu-mode": "hami-core"}, cores=100))
    wdev = codec.decode_container_devices(whole["metadata"]["annotations"][SUPPORT_ANNOS].split(";")[0])[0]
    assert "-cpx" not in wdev.uuid and wdev.usedcores == 256
    # a cpx pod that cannot fit anywhere reports ModeNotFit for the SPX GPUs
    big = amd_pod("big", annotations={"amd.com/vgpu-mode": "cpx"}, mem=40000)
    c.create("pods", big)
    r = sched.filter({"Pod": c.get_pod("default", "big"), "NodeNames": ["node1"]})
    assert not r["NodeNames"] and "ModeNotFit" in r["FailedNodes"]["node1"]


def test_manager_applies_when_idle_and_reports(env):
    c, sched, backend, cfg, reg, lock = env
    pm = P.PartitionManager(backend, "node1", lock_path=lock)
    from k8s_vgpu_scheduler_amd.utils import util
    util.patch_node_annotations("node1", {P.REQUEST_ANNOS: "1=QPX,0=CPX"})
    assert pm.reconcile()
    assert backend.partition_calls[-1] == (1, "QPX")
    assert c.get_node("node1")["metadata"]["annotations"][P.STATUS_ANNOS] == "0=CPX,1=QPX,2=SPX,3=SPX"
    assert not pm.reconcile()      # converged
    reg.register_once()
    devs = codec.unmarshal_node_devices(c.get_node("node1")["metadata"]["annotations"][REGISTER_ANNOS])
    assert sum(d.mode == "qpx" for d in devs) == 4


def test_manager_skips_busy_gpus(env):
    c, sched, backend, cfg, reg, lock = env
    pm = P.PartitionManager(backend, "node1", lock_path=lock)
    pod = _schedule(c, sched, amd_pod("p", annotations={"amd.com/use-gpu-uuid": "GPU-0002"}, mem=1000))
    assert pod is not None
    backend.procs["GPU-0003"] = [{"pid": 42}]
    from k8s_vgpu_scheduler_amd.utils import util
    util.patch_node_annotations("node1", {P.REQUEST_ANNOS: "2=DPX,3=DPX"})
    assert not pm.reconcile()
    st = c.get_node("node1")["metadata"]["annotations"][P.STATUS_ANNOS]
    assert "2=SPX>DPX:busy" in st and "3=SPX>DPX:busy" in st
    assert backend.partition_calls == [(0, "CPX")]
    # the pod finishes, the process exits -> applied
    c.patch_pod("default", "p", {"status": {"phase": "Succeeded"}})
    backend.procs.clear()
    assert pm.reconcile() and backend.modes[2] == "DPX" and backend.modes[3] == "DPX"


def test_apply_lock_pauses_registration(env):
    c, sched, backend, cfg, reg, lock = env
    with P.apply_lock(lock):
        assert P.is_applying(lock)
        assert reg.register_once() is False
        with pytest.raises(FileExistsError):
            with P.apply_lock(lock):
                pass
        from k8s_vgpu_scheduler_amd.utils import util
        util.patch_node_annotations("node1", {P.REQUEST_ANNOS: "1=CPX"})
        pm = P.PartitionManager(backend, "node1", lock_path=lock)
        assert not pm.reconcile()
        assert "1=SPX>CPX:locked" in c.get_node("node1")["metadata"]["annotations"][P.STATUS_ANNOS]
    assert not P.is_applying(lock)
    assert P.wait_until_applied(lock, timeout=0.1)


def test_parse_request():
    assert P.parse_request("0=cpx, 3=DPX;4=spx") == {0: "CPX", 3: "DPX", 4: "SPX"}
    assert P.parse_request("") == {}
    with pytest.raises(ValueError):
        P.parse_request("0=NPS2")


def test_partition_metric_and_topology_env(env, monkeypatch):
    from k8s_vgpu_scheduler_amd.scheduler.metrics import SchedulerCollector
    c, sched, backend, cfg, reg, _ = env
    fams = {f.name: f for f in SchedulerCollector(sched).collect()}
    samples = fams["hami_node_gpu_partition_info"].samples
    assert len(samples) == 8 and all(s.labels["mode"] == "cpx" and s.value == 32 for s in samples)
    from k8s_vgpu_scheduler_amd.device.amd.device import PAIR_SCORE_ANNOS
    monkeypatch.setenv("ENABLE_TOPOLOGY_SCORE", "false")
    assert PAIR_SCORE_ANNOS not in reg.annotations(backend.gpus())
    monkeypatch.delenv("ENABLE_TOPOLOGY_SCORE")
    assert PAIR_SCORE_ANNOS in reg.annotations(backend.gpus())
