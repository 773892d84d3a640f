"""Scheduler cache concurrency (SURVEY.md §4 race tests): register() against
the node-delete callback with a flapping node (register_race_test.go:37-120),
concurrent node-cache readers and writers (Test_ListNodes_Concurrent), and
transactional multi-vendor node locking (Test_lockAllDevices_Transactional)."""

import random
import threading

import pytest

from k8s_vgpu_scheduler_amd.device import devices as D
from k8s_vgpu_scheduler_amd.device.amd.device import REGISTER_ANNOS
from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.device.types import DeviceInfo, NodeInfo
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.nodes import NodeManager
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.testing import amd_node


@pytest.fixture
def cluster():
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    return c


def _run(threads):
    errs = []

    def wrap(fn):
        def go():
            try:
                fn()
            except BaseException as e:  # noqa: BLE001
                errs.append(e)
        return go
    ts = [threading.Thread(target=wrap(f)) for f in threads]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs


def test_register_vs_node_delete_converges(cluster):
    """One node whose GPU health flaps (so every register() pass rewrites the
    cache entry) against 6 threads running the delete callback; afterwards the
    node is really deleted and one more pass must leave no stale entry."""
    cluster.create("nodes", amd_node("gpu-node-0", n=1))
    s = Scheduler(cluster, SchedulerConfig())
    s.start()
    rounds = 600

    def flap_and_register():
        for v in range(rounds):
            node = cluster.get_node("gpu-node-0")
            ann = node["metadata"]["annotations"][REGISTER_ANNOS]
            healthy, sick = '"health":true', '"health":false'
            ann = ann.replace(healthy, sick) if v % 2 else ann.replace(sick, healthy)
            cluster.patch("nodes", "gpu-node-0", {"metadata": {"annotations": {REGISTER_ANNOS: ann}}})
            s.register()

    def deleter():
        n = cluster.get_node("gpu-node-0")
        for _ in range(rounds):
            s.on_del_node(n)
    _run([flap_and_register] + [deleter] * 6)
    # the node is still in the API: one pass brings it back
    s.register()
    assert "gpu-node-0" in s.nodes.node_ids()
    # a delete that lands while register() is between list and add_node
    real_list = s.nodes_inf.list

    def list_then_delete(*a, **kw):
        out = real_list(*a, **kw)
        cluster.delete("nodes", "gpu-node-0")          # informer event -> on_del_node
        return out
    s.nodes_inf.list = list_then_delete
    s.register()                                       # re-adds from the stale list
    s.nodes_inf.list = real_list
    s.register()                                       # ...and the next pass drops it
    assert s.nodes.node_ids() == [] and "gpu-node-0" not in s.inspect_all_nodes_usage()


def test_node_manager_concurrent_readers_and_writers():
    nm = NodeManager()
    names = [f"n{i}" for i in range(16)]

    def info(n):
        return NodeInfo(id=n, node={"metadata": {"name": n}},
                        devices={"AMD": [DeviceInfo(id=f"{n}-gpu0", index=0, count=8, devmem=294912,
                                                    devcore=256, type="AMD Instinct MI355X", numa=0,
                                                    mode="hami-core", health=True, devicevendor="AMD")]})

    def writer():
        rng = random.Random()
        for _ in range(2000):
            n = rng.choice(names)
            if rng.random() < 0.5:
                nm.add_node(n, info(n))
            else:
                nm.rm_node(n)

    def reader():
        for _ in range(2000):
            for k, v in nm.list_nodes().items():
                assert v.id == k and len(v.devices["AMD"]) == 1
    _run([writer] * 4 + [reader] * 4)
    for n in names:
        nm.add_node(n, info(n))
    assert sorted(nm.node_ids()) == sorted(names)


class _Vendor:
    def __init__(self, fail=False):
        self.fail, self.locked, self.released = fail, 0, 0

    def lock_node(self, node, pod):
        if self.fail:
            raise RuntimeError("lock conflict")
        self.locked += 1

    def release_node_lock(self, node, pod):
        self.released += 1


def test_lock_all_devices_is_transactional(cluster, monkeypatch):
    s = Scheduler(cluster, SchedulerConfig())
    a, b = _Vendor(), _Vendor(fail=True)
    monkeypatch.setattr(D, "get_devices", lambda: {"A": a, "B": b})
    with pytest.raises(RuntimeError):
        s.lock_all_devices({"metadata": {"name": "n1"}}, {"metadata": {"name": "p"}})
    assert a.locked == 1 and a.released == 1 and b.released == 0     # A rolled back
