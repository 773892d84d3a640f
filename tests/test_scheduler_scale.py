"""Scheduler at cluster scale: the per-node usage cache and the Fit memo must
not change a single placement, and must keep Filter fast at 100 nodes.

The reference scores every node in a goroutine on every Filter and rebuilds
usage from all pods (pkg/scheduler/score.go:360-419, scheduler.go:744-863);
here a memoised run and a from-scratch run of the same pod stream (several
namespaces, one with a ResourceQuota, GPU/node policy and selector
annotations, init containers, deletions in between) must agree pod by pod.
"""

import random
import time

import pytest

from k8s_vgpu_scheduler_amd.device.amd.device import CU_RANGES_ANNOS, SUPPORT_ANNOS
from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler, fit_signature
from k8s_vgpu_scheduler_amd.testing import amd_container, amd_node, amd_pod, full_mesh_scores, mi355x_devices
from k8s_vgpu_scheduler_amd.utils import types as T

SHAPES = [
    dict(containers=[amd_container(gpu=1, mem=36864, cores=25)]),
    dict(containers=[amd_container(gpu=1, mem=16384, cores=12)]),
    dict(containers=[amd_container(gpu=2, mem=65536, cores=50)]),
    dict(containers=[amd_container(gpu=1, mem=None, cores=100)]),
    dict(containers=[amd_container(gpu=1, mem=8192)], annotations={T.GPU_POLICY_ANNOTATION: "spread"}),
    dict(containers=[amd_container(gpu=4, mem=16384, cores=25)],
         annotations={T.GPU_POLICY_ANNOTATION: "topology-aware"}),
    dict(containers=[amd_container(gpu=1, mem=20000, cores=25)], annotations={T.NODE_POLICY_ANNOTATION: "spread"}),
    dict(containers=[amd_container("app", gpu=1, mem=30000, cores=25)],
         init=[amd_container("init", gpu=1, mem=50000, cores=50)]),
]


def _run(memoize: bool, nodes: int = 10, pods: int = 160, seed: int = 7):
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    names = []
    for i in range(nodes):
        devs = mi355x_devices(f"n{i}")
        degraded = {(devs[0].id, devs[1].id): 40} if i % 3 == 0 else None
        c.create("nodes", amd_node(f"n{i}", scores=full_mesh_scores(devs, degraded=degraded)))
        names.append(f"n{i}")
    c.create("resourcequotas", {"metadata": {"name": "q", "namespace": "team-q"},
                                "spec": {"hard": {"limits.amd.com/gpumem": "400000"}}})
    s = Scheduler(c, SchedulerConfig())
    s.memoize = memoize
    s.start()
    s.register()
    rng = random.Random(seed)
    out, live = [], []
    for i in range(pods):
        shape = rng.choice(SHAPES)
        ns = rng.choice(["default", "default", "team-a", "team-q"])
        pod = amd_pod(f"p{i}", namespace=ns, containers=shape["containers"], init=shape.get("init"),
                      annotations=dict(shape.get("annotations") or {}))
        c.create("pods", pod)
        cur = c.get_pod(ns, f"p{i}")
        res = s.filter({"Pod": cur, "NodeNames": names})
        annos = c.get_pod(ns, f"p{i}")["metadata"].get("annotations") or {}
        out.append((res.get("NodeNames"), annos.get(SUPPORT_ANNOS), annos.get(CU_RANGES_ANNOS),
                    sorted((res.get("FailedNodes") or {}).items())))
        if res.get("NodeNames"):
            live.append((ns, f"p{i}"))
        if live and rng.random() < 0.25:           # churn: a placed pod goes away
            ns_, name = live.pop(rng.randrange(len(live)))
            c.delete("pods", name, ns_)
    return out, s


@pytest.fixture(autouse=True)
def _reset():
    yield
    init_devices_with_config()
    get_local_cache().quotas.clear()


def test_memoised_filter_places_exactly_like_a_full_refit():
    ref, _ = _run(memoize=False)
    got, s = _run(memoize=True)
    assert len(ref) == len(got)
    for i, (a, b) in enumerate(zip(ref, got)):
        assert a == b, f"pod p{i}: full refit {a} vs memoised {b}"
    assert s.memo_hits > 300                # the memo actually served repeated pod shapes
    assert sum(1 for r in ref if r[0]) > 50   # and the stream placed plenty of pods


def test_fit_signature_ignores_scheduler_outputs_only():
    p = amd_pod("a", mem=1000, annotations={T.GPU_POLICY_ANNOTATION: "spread"})
    base = fit_signature(p)
    q = amd_pod("b", mem=1000, annotations={T.GPU_POLICY_ANNOTATION: "spread", T.ASSIGNED_NODE_ANNOTATION: "n1",
                                            T.ASSIGNED_TIME_ANNOTATION: "123", SUPPORT_ANNOS: "x"})
    assert fit_signature(q) == base                   # name/uid/outputs do not matter
    r = amd_pod("c", mem=1000, annotations={T.GPU_POLICY_ANNOTATION: "binpack"})
    assert fit_signature(r) != base                   # an input annotation does
    assert fit_signature(amd_pod("d", mem=2000, annotations={T.GPU_POLICY_ANNOTATION: "spread"})) != base
    assert fit_signature(amd_pod("e", namespace="x", mem=1000,
                                 annotations={T.GPU_POLICY_ANNOTATION: "spread"})) != base


def test_node_registration_change_invalidates_cached_usage():
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    c.create("nodes", amd_node("n1", n=1))
    s = Scheduler(c, SchedulerConfig())
    s.start()
    s.register()
    c.create("pods", amd_pod("a", mem=200000))
    assert s.filter({"Pod": c.get_pod("default", "a"), "NodeNames": ["n1"]})["NodeNames"] == ["n1"]
    c.create("pods", amd_pod("b", mem=200000))
    assert s.filter({"Pod": c.get_pod("default", "b"), "NodeNames": ["n1"]})["NodeNames"] is None
    # the device plugin re-registers the node with a second GPU: the same pod shape now fits
    node = amd_node("n1", n=2)
    c.patch("nodes", "n1", {"metadata": {"annotations": node["metadata"]["annotations"]}})
    s.register()
    assert s.filter({"Pod": c.get_pod("default", "b"), "NodeNames": ["n1"]})["NodeNames"] == ["n1"]


def test_filter_latency_at_100_nodes():
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    names = [f"node{i}" for i in range(100)]
    for n in names:
        c.create("nodes", amd_node(n, scores=full_mesh_scores(mi355x_devices(n))))
    s = Scheduler(c, SchedulerConfig())
    s.start()
    s.register()
    rng = random.Random(0)
    lat = []
    for i in range(200):
        shape = rng.choice(SHAPES[:4])
        c.create("pods", amd_pod(f"p{i}", containers=shape["containers"]))
        t0 = time.perf_counter()
        res = s.filter({"Pod": c.get_pod("default", f"p{i}"), "NodeNames": names})
        lat.append(time.perf_counter() - t0)
        assert res["NodeNames"]
    lat.sort()
    # before the usage cache + memo: p50 49-68 ms on this container
    assert lat[len(lat) // 2] < 0.010, f"filter p50 {lat[len(lat) // 2] * 1e3:.1f} ms"
