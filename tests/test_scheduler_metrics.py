"""Scheduler Prometheus collector (cmd/scheduler/metrics_test.go counterpart):
series names and labels, AMD CU -> percent normalisation, quota and
per-container series, legacy names, partition info, build info."""

import pytest
from prometheus_client import CollectorRegistry, generate_latest
from prometheus_client.parser import text_string_to_metric_families

from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.metrics import SchedulerCollector, normalize_amd_core
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.testing import MI355X_MEM_MIB, amd_node, amd_pod


@pytest.fixture
def sched():
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    c.create("nodes", amd_node("n1", n=2))
    s = Scheduler(c, SchedulerConfig())
    s.start()
    s.register()
    return s, c


def scrape(s, legacy=False):
    reg = CollectorRegistry()
    reg.register(SchedulerCollector(s, legacy=legacy))
    out = {}
    for fam in text_string_to_metric_families(generate_latest(reg).decode()):
        for smp in fam.samples:
            out.setdefault(smp.name, []).append((smp.labels, smp.value))
    return out


def one(samples, name, **labels):
    hits = [v for lab, v in samples.get(name, []) if all(lab.get(k) == str(w) for k, w in labels.items())]
    assert len(hits) == 1, (name, labels, samples.get(name))
    return hits[0]


@pytest.mark.parametrize("typ,total,alloc,expect", [
    ("AMD Instinct MI355X", 256, 64, (100.0, 25.0)),
    ("AMD Instinct MI355X", 256, 1, (100.0, 1.0)),      # ceil
    ("AMD Instinct MI355X", 0, 5, (0.0, 5.0)),          # unknown total: raw
    ("NVIDIA A100", 100, 30, (100.0, 30.0)),
])
def test_normalize_amd_core(typ, total, alloc, expect):
    assert normalize_amd_core(typ, total, alloc) == expect


def test_device_series_after_scheduling(sched):
    s, c = sched
    pod = amd_pod("p", mem=36864, cores=25)
    c.create("pods", pod)
    assert s.filter({"Pod": c.get_pod("default", "p"), "NodeNames": ["n1"]})["NodeNames"] == ["n1"]
    s.register()   # the overview the collector reads is refreshed by the register pass (scheduler.go:552)
    m = scrape(s)
    # spread picks the last device of the sorted list: find the used one
    used = [lab["device_uuid"] for lab, v in m["hami_gpu_shared_count"] if v == 1.0]
    assert len(used) == 1
    uuid = used[0]
    assert one(m, "hami_gpu_core_limit_ratio", device_uuid=uuid) == 100.0
    assert one(m, "hami_gpu_core_allocated_ratio", device_uuid=uuid) == 25.0
    assert one(m, "hami_gpu_memory_limit_bytes", device_uuid=uuid) == MI355X_MEM_MIB * 1024 * 1024
    assert one(m, "hami_gpu_memory_allocated_bytes", device_uuid=uuid, device_cores=256) == 36864 * 1024 * 1024
    assert one(m, "hami_node_gpu_memory_allocated_ratio", device_uuid=uuid) == pytest.approx(36864 / MI355X_MEM_MIB)
    assert one(m, "hami_vgpu_memory_allocated_bytes", pod="p", device_uuid=uuid, container_index=0) == \
        36864 * 1024 * 1024
    assert one(m, "hami_vgpu_core_allocated_ratio", pod="p", device_uuid=uuid) == 25.0
    assert all(lab["zone"] == "vGPU" for fam in m.values() for lab, _ in fam)
    assert len(m["hami_gpu_memory_limit_bytes"]) == 2


def test_quota_series(sched):
    s, c = sched
    c.create("resourcequotas", {"metadata": {"name": "q", "namespace": "team"},
                                "spec": {"hard": {"limits.amd.com/gpumem": "100000"}}})
    pod = amd_pod("p", namespace="team", mem=4096)
    c.create("pods", pod)
    s.filter({"Pod": c.get_pod("team", "p"), "NodeNames": ["n1"]})
    m = scrape(s)
    assert one(m, "hami_resource_quota_limit", namespace="team", quota_name="amd.com/gpumem") == 100000
    assert one(m, "hami_resource_quota_used", namespace="team", quota_name="amd.com/gpumem", limit=100000) == 4096


def test_legacy_series_only_when_enabled(sched):
    s, _ = sched
    assert "GPUDeviceMemoryLimit" not in scrape(s)
    m = scrape(s, legacy=True)
    assert {"GPUDeviceMemoryLimit", "GPUDeviceCoreLimit", "GPUDeviceSharedNum"} <= set(m)
    assert len(m["GPUDeviceCoreLimit"]) == 2


def test_partition_info_series():
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    from k8s_vgpu_scheduler_amd.device import codec
    from k8s_vgpu_scheduler_amd.device.amd.device import REGISTER_ANNOS
    from k8s_vgpu_scheduler_amd.testing import mi355x_devices
    from k8s_vgpu_scheduler_amd.k8s.fake import make_node
    devs = mi355x_devices("n1", n=4, cus=64)
    for d in devs:
        d.mode = "qpx"
    cap = {"amd.com/gpu": "32"}
    c.create("nodes", make_node("n1", annotations={REGISTER_ANNOS: codec.marshal_node_devices(devs)},
                                capacity=cap, allocatable=cap))
    s = Scheduler(c, SchedulerConfig())
    s.start()
    s.register()
    m = scrape(s)
    assert len(m["hami_node_gpu_partition_info"]) == 4
    assert {lab["mode"] for lab, _ in m["hami_node_gpu_partition_info"]} == {"qpx"}
    assert {v for _, v in m["hami_node_gpu_partition_info"]} == {64.0}
    # the reference's series name for the same rows (HAMi dashboards)
    mig = m["hami_node_gpu_mig_instance_info"]
    assert len(mig) == 4 and {lab["profile"] for lab, _ in mig} == {"qpx"}
    assert {lab["placement_size"] for lab, _ in mig} == {"64"}
    assert {lab["mig_uuid"] for lab, _ in mig} == {lab["device_uuid"] for lab, _ in mig}


def test_build_info(sched):
    s, _ = sched
    (labels, value), = scrape(s)["hami_build_info"]
    assert value == 1.0 and labels["version"] and labels["python_version"]
