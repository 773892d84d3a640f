"""Concurrent Filter calls must not over-commit a GPU.

kube-scheduler calls the extender once per scheduling cycle, but the HTTP
server is threaded and several scheduler profiles (or a retried request) can
overlap; the reference serialises through its caches
(pkg/scheduler/scheduler.go Filter).  Here 16 threads filter 16 pods that
each want 40 % of a GPU's HBM onto a 1-node, 4-GPU cluster: at most 2 fit per
GPU, so at most 8 may be placed and no GPU may end above its HBM."""

import sys
import threading
import time
from collections import defaultdict

from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler import scheduler as S
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.testing import MI355X_MEM_MIB, amd_node, amd_pod

from test_score_matrix import devs_of


def test_concurrent_filters_never_overcommit(monkeypatch):
    # widen the read-usage -> commit window so an unserialised Filter races
    # every time (without the lock this places 16 pods, 1.5 TB on one GPU)
    orig = S.score_node_safe

    def slow(*a, **k):
        r = orig(*a, **k)
        time.sleep(0.002)
        return r
    monkeypatch.setattr(S, "score_node_safe", slow)
    cluster = FakeCluster()
    init_global_client(cluster)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    cluster.create("nodes", amd_node("n1", n=4))
    s = Scheduler(cluster, SchedulerConfig())
    s.start()
    s.register()
    mem = MI355X_MEM_MIB * 40 // 100
    names = [f"p{i}" for i in range(16)]
    for n in names:
        cluster.create("pods", amd_pod(n, mem=mem))
    barrier = threading.Barrier(len(names))
    old = sys.getswitchinterval()
    sys.setswitchinterval(1e-6)     # interleave the threads as finely as the GIL allows
    placed, errors = [], []

    def go(n):
        try:
            barrier.wait()
            r = s.filter({"Pod": cluster.get_pod("default", n), "NodeNames": ["n1"]})
            if r.get("NodeNames"):
                placed.append(n)
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    ts = [threading.Thread(target=go, args=(n,)) for n in names]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    sys.setswitchinterval(old)
    assert not errors, errors
    per_gpu = defaultdict(int)
    for n in placed:
        for d in devs_of(cluster, n)[0]:
            per_gpu[d.uuid] += d.usedmem
    assert all(v <= MI355X_MEM_MIB for v in per_gpu.values()), dict(per_gpu)
    assert len(placed) == 8, placed


def _cluster_with(n_gpus=4):
    cluster = FakeCluster()
    init_global_client(cluster)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    cluster.create("nodes", amd_node("n1", n=n_gpus))
    s = Scheduler(cluster, SchedulerConfig())
    s.start()
    s.register()
    return cluster, s


def test_overlapping_filters_of_one_pod_with_a_failing_patch(monkeypatch):
    """two Filters for the SAME pod overlap (an extender
    timeout retry) and the first one's annotation patch fails.  Its rollback
    must not delete the second Filter's reservation, and the quota must not be
    released twice: the pod ends with exactly the reservation whose patch
    landed."""
    from k8s_vgpu_scheduler_amd.utils import util as U

    cluster, s = _cluster_with()
    get_local_cache().add_quota({"metadata": {"name": "q", "namespace": "default"},
                                 "spec": {"hard": {"limits.amd.com/gpumem": str(4 * MI355X_MEM_MIB)}}})
    mem = MI355X_MEM_MIB // 4
    cluster.create("pods", amd_pod("p", mem=mem))
    real = U.patch_pod_annotations
    first = threading.Event()
    calls = []

    def patch(pod, annos):
        calls.append(annos)
        if len(calls) == 1:          # the first Filter's patch: slow, then it fails
            first.set()
            time.sleep(0.05)
            raise RuntimeError("lost patch")
        return real(pod, annos)
    monkeypatch.setattr(U, "patch_pod_annotations", patch)
    pod = cluster.get_pod("default", "p")
    out = {}

    def go(tag):
        out[tag] = s.filter({"Pod": pod, "NodeNames": ["n1"]})
    a = threading.Thread(target=go, args=("a",))
    a.start()
    first.wait(5)
    b = threading.Thread(target=go, args=("b",))
    b.start()
    a.join()
    b.join()
    assert out["a"]["Error"] == "lost patch" and out["b"]["NodeNames"] == ["n1"], out
    pi = s.pod_manager.get_pod(pod)
    assert pi is not None and pi.node_id == "n1"          # the second Filter's reservation survived
    used = get_local_cache().quotas["default"]["amd.com/gpumem"].used
    assert used == mem, used                              # charged exactly once


def test_rollback_keeps_a_reservation_that_replaced_the_decision(monkeypatch):
    """Token check: when the pod manager entry is no longer the failed
    decision's (an informer event re-added the pod from its annotations),
    the rollback leaves it alone."""
    from k8s_vgpu_scheduler_amd.utils import util as U

    cluster, s = _cluster_with()
    cluster.create("pods", amd_pod("p", mem=MI355X_MEM_MIB // 4))
    pod = cluster.get_pod("default", "p")
    other = {"AMD": [[]]}

    def patch(p, annos):
        s.pod_manager.add_pod(p, "n-elsewhere", other)     # replaced while the patch was in flight
        raise RuntimeError("patch failed")
    monkeypatch.setattr(U, "patch_pod_annotations", patch)
    r = s.filter({"Pod": pod, "NodeNames": ["n1"]})
    assert r["Error"] == "patch failed"
    pi = s.pod_manager.get_pod(pod)
    assert pi is not None and pi.node_id == "n-elsewhere"
