"""Table-driven scheduler matrix: Filter outcomes over node states x pod shapes
x policies on the fake API server.

Modelled on the reference's scoring tables (pkg/scheduler/score_test.go:76-4300
Test_calcScore / Test_fitInDevices: single/multi device, sharing, init
containers and slot alignment, spread vs binpack, exhausted and exclusive
cards, type/uuid selectors, mode and NUMA, topology), re-cast for MI355X:
294912 MiB of HBM and 256 CUs per GPU, gpucores -> XCD-balanced CU ranges.
Every case schedules its ``pre`` pods first (each pinned to one node), then
filters the pod under test and checks the chosen node, the failure reason or
the devices written into the pod's allocation annotation.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import pytest

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device.amd.device import CU_RANGES_ANNOS, SUPPORT_ANNOS
from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster, make_node
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.testing import (MI355X_MEM_MIB, amd_container, amd_node, amd_pod, full_mesh_scores,
                                            mi355x_devices)
from k8s_vgpu_scheduler_amd.utils import nodelock
from k8s_vgpu_scheduler_amd.utils import types as T

GPU_POL = T.GPU_POLICY_ANNOTATION
NODE_POL = T.NODE_POLICY_ANNOTATION
MEM = MI355X_MEM_MIB


@dataclass
class Case:
    name: str
    nodes: dict                                  # node name -> amd_node kwargs
    pod: dict                                    # amd_pod kwargs of the pod under test
    node: str | None = None                      # expected node (None: must fail)
    reason: str | None = None                    # expected substring of the failure reason(s)
    pre: list = field(default_factory=list)      # [(node, amd_pod kwargs)] scheduled first
    check: object = None                         # fn(per-container device lists, bound pre devices)
    candidates: list | None = None


def ctr(**kw):
    return amd_container(**kw)


def devs_of(cluster, name):
    """Per-container devices of the allocation annotation (``c0;c1;...;`` wire
    form, one entry per container), with each device's CU ranges attached."""
    annos = cluster.get_pod("default", name)["metadata"].get("annotations") or {}
    ann = annos.get(SUPPORT_ANNOS, "")
    parts = ann.split(";")
    if ann.endswith(";"):
        parts = parts[:-1]
    per = [codec.decode_container_devices(part) if part else [] for part in parts]
    codec.attach_cu_ranges(per, annos.get(CU_RANGES_ANNOS))
    return per


def cus(d):
    from k8s_vgpu_scheduler_amd.device.amd import cu_alloc
    return cu_alloc.bitmap_from_ranges(d.custominfo["cu_ranges"])


def uuids(ctr_devs):
    return sorted(d.uuid for d in ctr_devs)


def _degraded_node(name, n, degraded):
    devs = mi355x_devices(name, n)
    return {"n": n, "scores": full_mesh_scores(devs, 100, degraded=degraded)}


CASES = [
    # ---------------------------------------------------------- single device
    Case("one node one GPU, one container, one slice", {"n1": dict(n=1)}, dict(mem=1000), "n1",
         check=lambda d, p: len(d[0]) == 1 and d[0][0].usedmem == 1000),
    Case("GPU already partly used still takes a fitting slice", {"n1": dict(n=1)}, dict(mem=100000), "n1",
         pre=[("n1", dict(mem=150000))]),
    Case("GPU already used cannot take more HBM than is left", {"n1": dict(n=1)}, dict(mem=200000), None,
         "CardInsufficientMemory", pre=[("n1", dict(mem=150000))]),
    Case("two GPUs, one nearly full: the slice lands on the other", {"n1": dict(n=2)}, dict(mem=100000), "n1",
         pre=[("n1", dict(mem=250000))], check=lambda d, p: d[0][0].uuid != p[0][0][0].uuid),
    Case("binpack GPU policy shares the used GPU", {"n1": dict(n=2)},
         dict(mem=1000, annotations={GPU_POL: "binpack"}), "n1", pre=[("n1", dict(mem=1000))],
         check=lambda d, p: d[0][0].uuid == p[0][0][0].uuid),
    Case("spread GPU policy prefers the idle GPU", {"n1": dict(n=2)},
         dict(mem=1000, annotations={GPU_POL: "spread"}), "n1", pre=[("n1", dict(mem=1000))],
         check=lambda d, p: d[0][0].uuid != p[0][0][0].uuid),
    Case("memory percentage request: half of the HBM", {"n1": dict(n=1)}, dict(mem_pct=50), "n1",
         check=lambda d, p: d[0][0].usedmem == MEM // 2),
    Case("no gpumem: the whole HBM of the GPU", {"n1": dict(n=1)}, dict(gpu=1), "n1",
         check=lambda d, p: d[0][0].usedmem == MEM),
    # ------------------------------------------------------------- CU ranges
    Case("25 % cores = 64 CUs, 8 per XCD", {"n1": dict(n=1)}, dict(mem=1000, cores=25), "n1",
         check=lambda d, p: d[0][0].usedcores == 64 and
         codec.ranges_count(d[0][0].custominfo["cu_ranges"]) == 64),
    Case("10 % cores round up to whole XCD granules (32 CUs)", {"n1": dict(n=1)}, dict(mem=1000, cores=10),
         "n1", check=lambda d, p: d[0][0].usedcores == 32),
    Case("CU ranges of two slices on one GPU are disjoint", {"n1": dict(n=1)}, dict(mem=1000, cores=50), "n1",
         pre=[("n1", dict(mem=1000, cores=50))],
         check=lambda d, p: cus(d[0][0]) & cus(p[0][0][0]) == 0),
    Case("cores beyond what is left on the only GPU", {"n1": dict(n=1)}, dict(mem=1000, cores=50), None,
         "CardInsufficientCore", pre=[("n1", dict(mem=1000, cores=75))]),
    Case("core request above 100 is clamped to an exclusive card", {"n1": dict(n=2)},
         dict(mem=1000, cores=150), "n1", pre=[("n1", dict(mem=1000, cores=10))],
         check=lambda d, p: d[0][0].uuid != p[0][0][0].uuid and d[0][0].usedcores == 256),
    Case("exclusive card (cores 100) cannot share a used GPU", {"n1": dict(n=1)}, dict(mem=1000, cores=100),
         None, "ExclusiveDeviceAllocateConflict", pre=[("n1", dict(mem=1000, cores=0))]),
    Case("whole-card CUs cannot be granted next to a partition", {"n1": dict(n=1)}, dict(mem=1000, cores=100),
         None, "CardInsufficientCore", pre=[("n1", dict(mem=1000, cores=10))]),
    Case("a cores-0 job cannot land on a GPU whose CUs are all taken", {"n1": dict(n=1)},
         dict(mem=1000, cores=0), None, "CardComputeUnitsExhausted", pre=[("n1", dict(mem=1000, cores=100))]),
    # ---------------------------------------------------------- multi device
    Case("two GPUs requested: two distinct GPUs", {"n1": dict(n=2)}, dict(gpu=2, mem=1000), "n1",
         check=lambda d, p: len(set(uuids(d[0]))) == 2),
    Case("two GPUs requested, both already shared", {"n1": dict(n=2)}, dict(gpu=2, mem=1000), "n1",
         pre=[("n1", dict(mem=1000)), ("n1", dict(mem=1000, annotations={GPU_POL: "spread"}))],
         check=lambda d, p: len(set(uuids(d[0]))) == 2),
    Case("more GPUs requested than the node has", {"n1": dict(n=2)}, dict(gpu=3, mem=1000), None,
         "NodeInsufficientDevice"),
    Case("two GPUs requested, only one fits the HBM", {"n1": dict(n=2)}, dict(gpu=2, mem=200000), None,
         "AllocatedCardsInsufficientRequest", pre=[("n1", dict(mem=200000))]),
    # ------------------------------------------------- containers and slots
    Case("two containers, spread: different GPUs", {"n1": dict(n=2)},
         dict(containers=[ctr(name="a", mem=1000), ctr(name="b", mem=1000)], annotations={GPU_POL: "spread"}),
         "n1", check=lambda d, p: len(d) == 2 and d[0][0].uuid != d[1][0].uuid),
    Case("two containers, binpack: the same GPU", {"n1": dict(n=2)},
         dict(containers=[ctr(name="a", mem=1000), ctr(name="b", mem=1000)], annotations={GPU_POL: "binpack"}),
         "n1", check=lambda d, p: len(d) == 2 and d[0][0].uuid == d[1][0].uuid),
    Case("second container uses the device: slot 0 stays empty", {"n1": dict(n=1)},
         dict(containers=[ctr(name="a", gpu=None), ctr(name="b", mem=1000)]), "n1",
         check=lambda d, p: len(d) == 2 and d[0] == [] and len(d[1]) == 1),
    Case("three containers, only the middle one uses a device", {"n1": dict(n=1)},
         dict(containers=[ctr(name="a", gpu=None), ctr(name="b", mem=1000), ctr(name="c", gpu=None)]), "n1",
         check=lambda d, p: len(d) == 3 and d[0] == [] and len(d[1]) == 1 and d[2] == []),
    Case("containers together exceed one GPU's HBM: split over two GPUs", {"n1": dict(n=2)},
         dict(containers=[ctr(name="a", mem=200000), ctr(name="b", mem=200000)]), "n1",
         check=lambda d, p: d[0][0].uuid != d[1][0].uuid),
    Case("containers together exceed the node", {"n1": dict(n=1)},
         dict(containers=[ctr(name="a", mem=200000), ctr(name="b", mem=200000)]), None, "CardInsufficientMemory"),
    # --------------------------------------------------------- init containers
    Case("init container runs first: init + app each 200 GB fit one GPU", {"n1": dict(n=1)},
         dict(init=[ctr(name="init", mem=200000)], containers=[ctr(name="app", mem=200000)]), "n1"),
    Case("init container wants more HBM than any GPU has", {"n1": dict(n=2)},
         dict(init=[ctr(name="init", mem=MEM + 1)], containers=[ctr(name="app", mem=1000)]), None,
         "CardInsufficientMemory"),
    Case("init container wants more cores than are left", {"n1": dict(n=1)},
         dict(init=[ctr(name="init", mem=1000, cores=100)], containers=[ctr(name="app", mem=1000)]), None,
         "CardInsufficientCore", pre=[("n1", dict(mem=1000, cores=10))]),
    Case("init container without a device, app with one: slots align", {"n1": dict(n=1)},
         dict(init=[ctr(name="init", gpu=None)], containers=[ctr(name="app", mem=1000)]), "n1"),
    # ---------------------------------------------------------- selectors
    Case("use-gputype matches the board name", {"n1": dict(n=1)},
         dict(mem=1000, annotations={"amd.com/use-gputype": "MI355X"}), "n1"),
    Case("use-gputype of another card type", {"n1": dict(n=1)},
         dict(mem=1000, annotations={"amd.com/use-gputype": "MI300X"}), None, "CardTypeMismatch"),
    Case("nouse-gputype excludes the card", {"n1": dict(n=1)},
         dict(mem=1000, annotations={"amd.com/nouse-gputype": "MI355"}), None, "CardTypeMismatch"),
    Case("use-gpu-uuid picks that GPU", {"n1": dict(n=4)},
         dict(mem=1000, annotations={"amd.com/use-gpu-uuid": "n1-gpu2"}), "n1",
         check=lambda d, p: d[0][0].uuid == "n1-gpu2"),
    Case("use-gpu-uuid of a GPU elsewhere", {"n1": dict(n=2)},
         dict(mem=1000, annotations={"amd.com/use-gpu-uuid": "other-gpu0"}), None, "CardUuidMismatch"),
    Case("nouse-gpu-uuid skips that GPU", {"n1": dict(n=2)},
         dict(mem=1000, annotations={"amd.com/nouse-gpu-uuid": "n1-gpu1,n1-gpu0"}), None, "CardUuidMismatch"),
    # ------------------------------------------------------- slots and health
    Case("all time-slicing slots of the GPU taken", {"n1": dict(n=1, split=2)}, dict(mem=1000), None,
         "CardTimeSlicingExhausted", pre=[("n1", dict(mem=1000)), ("n1", dict(mem=1000))]),
    Case("an unhealthy GPU is skipped", {"n1": dict(n=1, health=False)}, dict(mem=1000), None, "CardNotHealth"),
    Case("compute-partition mode not offered by the node", {"n1": dict(n=1)},
         dict(mem=1000, annotations={"amd.com/vgpu-mode": "cpx"}), None, "ModeNotFit"),
    Case("numa-bind: two GPUs must share a NUMA node", {"n1": dict(n=2, numa_per=1)},
         dict(gpu=2, mem=1000, annotations={"amd.com/numa-bind": "true"}), None, "NumaNotFit"),
    Case("numa-bind satisfied inside one NUMA node", {"n1": dict(n=4, numa_per=2)},
         dict(gpu=2, mem=1000, annotations={"amd.com/numa-bind": "true"}), "n1"),
    # ---------------------------------------------------------------- mutex
    Case("mutex policy takes an idle GPU", {"n1": dict(n=2)}, dict(mem=1000, annotations={GPU_POL: "mutex"}),
         "n1", pre=[("n1", dict(mem=1000))], check=lambda d, p: d[0][0].uuid != p[0][0][0].uuid),
    Case("mutex policy with no idle GPU left", {"n1": dict(n=1)}, dict(mem=1000, annotations={GPU_POL: "mutex"}),
         None, "ExclusiveDeviceAllocateConflict", pre=[("n1", dict(mem=1000))]),
    # ---------------------------------------------------------- node policy
    Case("binpack node policy picks the used node", {"n1": dict(n=1), "n2": dict(n=1)},
         dict(mem=1000, annotations={NODE_POL: "binpack"}), "n1", pre=[("n1", dict(mem=100000))]),
    Case("spread node policy picks the idle node", {"n1": dict(n=1), "n2": dict(n=1)},
         dict(mem=1000, annotations={NODE_POL: "spread"}), "n2", pre=[("n1", dict(mem=100000))]),
    Case("only one of two nodes fits", {"n1": dict(n=1), "n2": dict(n=1)}, dict(mem=200000), "n2",
         pre=[("n1", dict(mem=200000))]),
    Case("neither node fits: both reported", {"n1": dict(n=1), "n2": dict(n=1)}, dict(mem=MEM + 1), None,
         "CardInsufficientMemory"),
    # ------------------------------------------------------------- topology
    Case("topology-aware 2-GPU pod avoids degraded xGMI links",
         {"n1": _degraded_node("n1", 4, {("n1-gpu0", "n1-gpu1"): 10, ("n1-gpu0", "n1-gpu2"): 10,
                                          ("n1-gpu0", "n1-gpu3"): 10, ("n1-gpu1", "n1-gpu2"): 40})},
         dict(gpu=2, mem=1000, annotations={GPU_POL: "topology-aware"}), "n1",
         check=lambda d, p: uuids(d[0]) in (["n1-gpu1", "n1-gpu3"], ["n1-gpu2", "n1-gpu3"])),
    Case("topology-aware 1-GPU pod keeps the best-connected GPUs free",
         {"n1": _degraded_node("n1", 4, {("n1-gpu0", "n1-gpu1"): 10, ("n1-gpu0", "n1-gpu2"): 10,
                                          ("n1-gpu0", "n1-gpu3"): 10})},
         dict(gpu=1, mem=1000, annotations={GPU_POL: "topology-aware"}), "n1",
         check=lambda d, p: uuids(d[0]) == ["n1-gpu0"]),
    Case("healthy xGMI node preferred for a multi-GPU pod",
         {"good": _degraded_node("good", 2, {}), "bad": _degraded_node("bad", 2, {("bad-gpu0", "bad-gpu1"): 20})},
         dict(gpu=2, mem=1000), "good"),
]


@pytest.fixture
def cluster():
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    return c


def _node(name, spec):
    spec = dict(spec)
    scores = spec.pop("scores", None)
    return amd_node(name, scores=scores, **spec)


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_filter_matrix(cluster, case):
    for name, spec in case.nodes.items():
        cluster.create("nodes", _node(name, spec))
    s = Scheduler(cluster, SchedulerConfig())
    s.start()
    s.register()
    pre_devs = []
    for i, (node, kw) in enumerate(case.pre):
        pod = amd_pod(f"pre{i}", **kw)
        cluster.create("pods", pod)
        res = s.filter({"Pod": cluster.get_pod("default", f"pre{i}"), "NodeNames": [node]})
        assert res["NodeNames"] == [node], (case.name, "pre", i, res)
        p = cluster.get_pod("default", f"pre{i}")
        assert s.bind({"PodName": f"pre{i}", "PodNamespace": "default", "PodUID": p["metadata"]["uid"],
                       "Node": node})["Error"] == ""
        # the device plugin's Allocate releases the node lock once the pod is placed
        nodelock.release_node_lock(node, T.NODE_LOCK_KEY, cluster.get_pod("default", f"pre{i}"))
        pre_devs.append(devs_of(cluster, f"pre{i}"))
    pod = amd_pod("t", **case.pod)
    cluster.create("pods", pod)
    cands = case.candidates or list(case.nodes)
    res = s.filter({"Pod": cluster.get_pod("default", "t"), "NodeNames": cands})
    if case.node is None:
        assert not res.get("NodeNames"), (case.name, res)
        failed = res.get("FailedNodes") or {}
        assert set(failed) == set(cands), (case.name, res)
        if case.reason:
            assert all(case.reason in r for r in failed.values()), (case.name, failed)
        return
    assert res.get("NodeNames") == [case.node], (case.name, res)
    if case.check is not None:
        assert case.check(devs_of(cluster, "t"), pre_devs), (case.name, devs_of(cluster, "t"), pre_devs)
