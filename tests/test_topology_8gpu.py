"""Multi-GPU placement without a multi-GPU box: an 8 x MI355X node's KFD
topology (shaped like the one measured on the hardware,
tests/fixtures/mi355x_8gpu_kfd_links.json) driven through discovery ->
registration -> scheduler Filter with the topology-aware policy.

Reference: pkg/device/nvidia/calculate_score.go:177-286 (pair scores),
links.go:411-481, device.go:887-978 (best combination)."""

import json
from pathlib import Path

import pytest

from k8s_vgpu_scheduler_amd import smi
from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device.amd import topology
from k8s_vgpu_scheduler_amd.device.amd.device import PAIR_SCORE_ANNOS, REGISTER_ANNOS
from k8s_vgpu_scheduler_amd.deviceplugin.allocate import PluginConfig
from k8s_vgpu_scheduler_amd.deviceplugin.register import Registrar
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster, make_node
from k8s_vgpu_scheduler_amd.testing import amd_pod, write_mi355x_sysfs
from k8s_vgpu_scheduler_amd.utils import types as T

FIX = Path(__file__).parent / "fixtures" / "mi355x_8gpu_kfd_links.json"


def make_sched(cluster):
    from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig
    from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
    s = Scheduler(cluster, SchedulerConfig())
    s.start()
    s.register()
    assert s.synced
    return s


def filt(s, cluster, pod, nodes):
    cluster.create("pods", pod)
    return s.filter({"Pod": cluster.get_pod("default", pod["metadata"]["name"]), "NodeNames": nodes})


def test_fixture_matches_the_measured_node():
    """The synthetic tree reproduces the link table the hardware reported."""
    meas = json.loads(FIX.read_text())["nodes"]
    xgmi = [l for n in meas.values() for l in n["io_links"].values() if l["type"] == smi.KFD_IOLINK_XGMI]
    assert xgmi and {(l["weight"], l["min_bandwidth"], l["max_bandwidth"]) for l in xgmi} == {(15, 76000, 76000)}
    pcie = [l for n in meas.values() for l in n["io_links"].values()
            if l["type"] == smi.KFD_IOLINK_PCIE and l["max_bandwidth"]]
    assert {(l["weight"], l["max_bandwidth"]) for l in pcie} == {(20, 64000)}
    gpu = next(n for n in meas.values() if n.get("properties", {}).get("simd_count"))
    ids = json.loads(FIX.read_text())["amdsmi_visible_gpu"]
    # one identity across backends: GPU-<KFD unique_id> = amd-smi hip_uuid = asic serial
    assert smi.rocr_uuid(gpu["properties"]["unique_id"]) == ids["amdsmi_get_gpu_enumeration_info"]["hip_uuid"]
    assert smi.rocr_uuid(ids["asic_info"]["asic_serial"]) == ids["amdsmi_get_gpu_enumeration_info"]["hip_uuid"]
    assert smi.canonical_name(ids["amdsmi_get_gpu_board_info"]["product_name"]) == "AMD Instinct MI355 OAM"
    assert smi.canonical_name("AMD Radeon Graphics", device_id=0x75A3) == "AMD Instinct MI355X"


def test_sysfs_backend_reads_the_8gpu_xgmi_mesh(tmp_path):
    kfd, drm = write_mi355x_sysfs(tmp_path)
    b = smi.SysfsBackend(kfd, drm)
    gs = b.gpus()
    assert len(gs) == 8 and len({g.uuid for g in gs}) == 8
    assert all(g.uuid.startswith("GPU-ae8c1614e27cc4") and g.rocr_id == g.uuid for g in gs)
    assert {g.name for g in gs} == {"AMD Instinct MI355 OAM"}
    li = b.link(gs[0], gs[5])
    assert (li.type, li.weight, li.max_bw_gbps) == ("XGMI", 15, 76.0)
    scores = smi.pair_scores(b, gs)
    assert {v for row in scores.values() for v in row.values()} == {100}   # healthy full mesh
    assert topology.is_asymmetric(scores) == []


def test_degraded_and_pcie_pairs_score_lower(tmp_path):
    kfd, drm = write_mi355x_sysfs(tmp_path, degraded={(0, 1): 38000}, pcie_pairs=[(2, 3)])
    b = smi.SysfsBackend(kfd, drm)
    gs = b.gpus()
    scores = smi.pair_scores(b, gs)
    u = [g.uuid for g in gs]
    assert scores[u[0]][u[1]] == scores[u[1]][u[0]] == 50            # half the nominal 76 GB/s
    assert scores[u[2]][u[3]] == 20                                   # PCIe peers, same NUMA node
    assert scores[u[4]][u[5]] == 100


@pytest.fixture
def cluster():
    from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
    from k8s_vgpu_scheduler_amd.scheduler.config import init_devices_with_config
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    return c


def _register(cluster, tmp_path, name, **kw):
    kfd, drm = write_mi355x_sysfs(tmp_path / name, **kw)
    b = smi.SysfsBackend(kfd, drm)
    cluster.create("nodes", make_node(name, capacity={"amd.com/gpu": "64"}, allocatable={"amd.com/gpu": "64"}))
    reg = Registrar(b, PluginConfig(device_split_count=8), name)
    assert reg.register_once()
    return b


def _placed(cluster, pod):
    from k8s_vgpu_scheduler_amd.device.amd.device import SUPPORT_ANNOS
    ann = cluster.get_pod("default", pod)["metadata"]["annotations"][SUPPORT_ANNOS]
    return sorted(d.uuid for d in codec.decode_container_devices(ann.split(";")[0]))


def test_register_filter_places_multi_gpu_pods_on_the_best_links(cluster, tmp_path):
    """register -> node annotations -> Filter: a 2-GPU topology-aware pod avoids
    the degraded and PCIe pairs; a 4-GPU pod lands on 4 fully healthy GPUs."""

    b = _register(cluster, tmp_path, "n1", degraded={(0, 1): 20000, (0, 2): 20000, (1, 2): 20000},
                  pcie_pairs=[(3, 4)])
    node = cluster.get("nodes", "n1")
    annos = node["metadata"]["annotations"]
    assert REGISTER_ANNOS in annos and PAIR_SCORE_ANNOS in annos
    devs = codec.unmarshal_node_devices(annos[REGISTER_ANNOS])
    assert len(devs) == 8 and {d.type for d in devs} == {"AMD Instinct MI355 OAM"}
    s = make_sched(cluster)
    scores = smi.pair_scores(b, b.gpus())
    pol = {T.GPU_POLICY_ANNOTATION: "topology-aware"}
    filt(s, cluster, amd_pod("tp2", gpu=2, mem=1000, annotations=pol), ["n1"])
    a, c = _placed(cluster, "tp2")
    assert scores[a][c] == 100
    filt(s, cluster, amd_pod("tp4", gpu=4, mem=1000, annotations=pol), ["n1"])
    four = _placed(cluster, "tp4")
    assert topology.mean_pair_score(four, scores) == 100


def test_use_gputype_matches_the_registered_board_name(cluster, tmp_path):
    """amd.com/use-gputype: MI355 schedules on a node registered by discovery
    (the board name, not "AMD Radeon Graphics"); a non-matching type does not."""

    _register(cluster, tmp_path, "n1")
    s = make_sched(cluster)
    res = filt(s, cluster, amd_pod("want", mem=1000, annotations={"amd.com/use-gputype": "MI355"}), ["n1"])
    assert res["NodeNames"] == ["n1"]
    res = filt(s, cluster, amd_pod("other", mem=1000, annotations={"amd.com/use-gputype": "MI300X"}), ["n1"])
    assert not res.get("NodeNames")
