"""Filter vs a brute-force feasibility oracle (property test).

The reference pins its fit engine with hand tables (pkg/scheduler/score_test.go
Test_calcScore, ~3.2k lines; tests/test_score_matrix.py re-casts those).  This
test complements them: hypothesis generates small clusters and sequences of
single-container pods (1-2 GPUs, HBM in MiB, gpucores 0/25/50/100), each pod
is filtered and bound in turn, and after every step

* soundness: no GPU holds more HBM than it has, more tasks than its split
  count, or two grants whose CU ranges overlap; every CU grant is
  XCD-balanced (device/amd/cu_alloc.py);
* completeness: when Filter refuses a pod, the oracle (AMDDevices.fit's rules
  applied to the bookkept usage: free slot, free HBM, free CUs in whole
  granules, an exclusive 100 % request only on an idle GPU, no time-shared
  request on a GPU whose CUs are all granted) finds no node with enough
  eligible GPUs either; when Filter accepts, the oracle agrees.
"""

from __future__ import annotations

from hypothesis import HealthCheck, given, settings, strategies as st

from k8s_vgpu_scheduler_amd.device.amd import cu_alloc
from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.testing import amd_node, amd_pod
from k8s_vgpu_scheduler_amd.utils import nodelock
from k8s_vgpu_scheduler_amd.utils import types as T

from test_score_matrix import devs_of

MEM, CUS, SPLIT = 294912, 256, 4
TOPO = cu_alloc.CUTopology()

pod_spec = st.tuples(st.integers(1, 2),                                     # GPUs
                     st.sampled_from([1000, 50000, 100000, 150000, 290000]),  # MiB per GPU
                     st.sampled_from([0, 0, 25, 50, 100]))                   # gpucores %


class Book:
    def __init__(self, nodes):
        self.gpus = {f"{n}-gpu{i}": {"node": n, "mem": 0, "cu": 0, "tasks": 0, "bitmap": 0}
                     for n, k in nodes.items() for i in range(k)}

    def eligible(self, uuid, mem, cores):
        g = self.gpus[uuid]
        cu = CUS if cores >= 100 else (cu_alloc.round_up_cus(CUS * cores // 100, TOPO) if cores else 0)
        if g["tasks"] >= SPLIT or MEM - g["mem"] < mem or CUS - g["cu"] < cu:
            return False
        if cores >= 100 and g["tasks"] > 0:
            return False
        if g["cu"] >= CUS and cu == 0:
            return False
        return True

    def feasible_nodes(self, n_gpu, mem, cores):
        out = set()
        for node in {g["node"] for g in self.gpus.values()}:
            ok = sum(1 for u, g in self.gpus.items() if g["node"] == node and self.eligible(u, mem, cores))
            if ok >= n_gpu:
                out.add(node)
        return out


@settings(max_examples=80, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.dictionaries(st.sampled_from(["a", "b", "c"]), st.integers(1, 3), min_size=1, max_size=3),
       st.lists(pod_spec, min_size=1, max_size=10),
       st.sampled_from([T.GPU_POLICY_BINPACK, T.GPU_POLICY_SPREAD]))
def test_filter_agrees_with_oracle(nodes, pods, gpu_policy):
    cluster = FakeCluster()
    init_global_client(cluster)
    init_devices_with_config(gpu_policy=gpu_policy)
    get_local_cache().quotas.clear()
    for name, k in nodes.items():
        cluster.create("nodes", amd_node(name, n=k, split=SPLIT))
    s = Scheduler(cluster, SchedulerConfig(gpu_scheduler_policy=gpu_policy))
    s.start()
    s.register()
    book = Book(nodes)
    for i, (n_gpu, mem, cores) in enumerate(pods):
        name = f"p{i}"
        kw = dict(gpu=n_gpu, mem=mem)
        if cores:
            kw["cores"] = cores
        cluster.create("pods", amd_pod(name, **kw))
        want = book.feasible_nodes(n_gpu, mem, cores)
        res = s.filter({"Pod": cluster.get_pod("default", name), "NodeNames": sorted(nodes)})
        got = res.get("NodeNames") or []
        if not want:
            assert not got, (i, pods[: i + 1], res)
            continue
        assert got and got[0] in want, (i, pods[: i + 1], want, res)
        node = got[0]
        p = cluster.get_pod("default", name)
        assert s.bind({"PodName": name, "PodNamespace": "default", "PodUID": p["metadata"]["uid"],
                       "Node": node})["Error"] == ""
        nodelock.release_node_lock(node, T.NODE_LOCK_KEY, cluster.get_pod("default", name))
        devs = devs_of(cluster, name)[0]
        assert len(devs) == n_gpu and len({d.uuid for d in devs}) == n_gpu
        for d in devs:
            g = book.gpus[d.uuid]
            assert g["node"] == node and book.eligible(d.uuid, mem, cores)
            g["mem"] += d.usedmem
            g["cu"] += d.usedcores
            g["tasks"] += 1
            ranges = (d.custominfo or {}).get("cu_ranges") or []
            if ranges:
                bm = cu_alloc.bitmap_from_ranges(ranges)
                assert bm & g["bitmap"] == 0, "CU grants overlap"
                assert cu_alloc.is_balanced(ranges, TOPO)
                assert bin(bm).count("1") == d.usedcores
                g["bitmap"] |= bm
            assert g["mem"] <= MEM and g["cu"] <= CUS and g["tasks"] <= SPLIT


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.dictionaries(st.sampled_from(["a", "b"]), st.integers(1, 2), min_size=1, max_size=2),
       st.lists(st.one_of(st.tuples(st.just("add"), pod_spec),
                          st.tuples(st.sampled_from(["delete", "succeed"]), st.integers(0, 50))),
                min_size=1, max_size=14))
def test_usage_released_by_delete_and_completion(nodes, ops):
    """Interleave placements with pod deletions and completions: freed capacity
    must become schedulable again at once (the usage cache and the Filter memo
    are invalidated by the pod events), and the oracle still agrees."""
    cluster = FakeCluster()
    init_global_client(cluster)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    for name, k in nodes.items():
        cluster.create("nodes", amd_node(name, n=k, split=SPLIT))
    s = Scheduler(cluster, SchedulerConfig())
    s.start()
    s.register()
    book = Book(nodes)
    live = {}                       # pod name -> devices
    for i, (kind, arg) in enumerate(ops):
        if kind != "add":
            if not live:
                continue
            name = sorted(live)[arg % len(live)]
            if kind == "delete":
                cluster.delete("pods", name, "default")
            else:
                p = cluster.get_pod("default", name)
                p["status"] = {"phase": "Succeeded"}
                cluster.update("pods", p)
            for d in live.pop(name):
                g = book.gpus[d.uuid]
                g["mem"] -= d.usedmem
                g["cu"] -= d.usedcores
                g["tasks"] -= 1
                g["bitmap"] &= ~cu_alloc.bitmap_from_ranges((d.custominfo or {}).get("cu_ranges") or [])
            continue
        n_gpu, mem, cores = arg
        name = f"p{i}"
        kw = dict(gpu=n_gpu, mem=mem)
        if cores:
            kw["cores"] = cores
        cluster.create("pods", amd_pod(name, **kw))
        want = book.feasible_nodes(n_gpu, mem, cores)
        res = s.filter({"Pod": cluster.get_pod("default", name), "NodeNames": sorted(nodes)})
        got = res.get("NodeNames") or []
        assert bool(got) == bool(want), (i, ops[: i + 1], want, res)
        if not got:
            cluster.delete("pods", name, "default")
            continue
        assert got[0] in want
        devs = devs_of(cluster, name)[0]
        for d in devs:
            g = book.gpus[d.uuid]
            assert book.eligible(d.uuid, mem, cores)
            g["mem"] += d.usedmem
            g["cu"] += d.usedcores
            g["tasks"] += 1
            bm = cu_alloc.bitmap_from_ranges((d.custominfo or {}).get("cu_ranges") or [])
            assert bm & g["bitmap"] == 0
            g["bitmap"] |= bm
        live[name] = devs


@settings(max_examples=50, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.integers(0, 600000), st.integers(0, 400),
       st.lists(st.tuples(st.integers(1, 2), st.sampled_from([1000, 50000, 150000]), st.sampled_from([0, 25, 50])),
                min_size=1, max_size=10))
def test_namespace_quota_is_never_exceeded(mem_quota, core_quota, pods):
    """Filter under a namespace ResourceQuota (limits.amd.com/gpumem / gpucores,
    pkg/device/quota.go): a pod is placed only if the namespace's usage plus its
    request stays within both limits (cores in % per GPU), on top of fitting."""
    cluster = FakeCluster()
    init_global_client(cluster)
    init_devices_with_config()
    q = get_local_cache()
    q.quotas.clear()
    q.add_quota({"metadata": {"name": "q", "namespace": "default"},
                 "spec": {"hard": {"limits.amd.com/gpumem": str(mem_quota),
                                   "limits.amd.com/gpucores": str(core_quota)}}})
    cluster.create("nodes", amd_node("a", n=4, split=SPLIT))
    s = Scheduler(cluster, SchedulerConfig())
    s.start()
    s.register()
    book = Book({"a": 4})
    used_mem = used_core = 0
    try:
        for i, (n_gpu, mem, cores) in enumerate(pods):
            name = f"p{i}"
            kw = dict(gpu=n_gpu, mem=mem)
            if cores:
                kw["cores"] = cores
            cluster.create("pods", amd_pod(name, **kw))
            fits_quota = used_mem + mem * n_gpu <= mem_quota and used_core + cores * n_gpu <= core_quota
            want = fits_quota and bool(book.feasible_nodes(n_gpu, mem, cores))
            res = s.filter({"Pod": cluster.get_pod("default", name), "NodeNames": ["a"]})
            got = bool(res.get("NodeNames"))
            assert got == want, (i, pods[: i + 1], mem_quota, core_quota, used_mem, used_core, res)
            if not got:
                cluster.delete("pods", name, "default")
                continue
            used_mem += mem * n_gpu
            used_core += cores * n_gpu
            for d in devs_of(cluster, name)[0]:
                g = book.gpus[d.uuid]
                g["mem"] += d.usedmem
                g["cu"] += d.usedcores
                g["tasks"] += 1
    finally:
        q.quotas.clear()


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.dictionaries(st.sampled_from(["a", "b", "c"]), st.integers(1, 3), min_size=1, max_size=3),
       st.lists(pod_spec, min_size=1, max_size=8))
def test_simulation_filter_matches_the_real_one_without_side_effects(nodes, pods):
    """Cluster-Autoscaler simulation (``Nodes`` given): the nodes are
    transient templates, fitted empty as in the reference
    (scheduler.go:865-893 getSimulationNodesUsage -> buildNodeUsage without
    pod usage).  On an empty cluster it picks the node the real Filter picks;
    it never patches a pod nor caches one, and it ignores the cached usage."""
    cluster = FakeCluster()
    init_global_client(cluster)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    for name, k in nodes.items():
        cluster.create("nodes", amd_node(name, n=k, split=SPLIT))
    s = Scheduler(cluster, SchedulerConfig())
    s.start()
    s.register()
    node_objs = [cluster.get_node(n) for n in sorted(nodes)]
    for i, (n_gpu, mem, cores) in enumerate(pods):
        name = f"p{i}"
        kw = dict(gpu=n_gpu, mem=mem)
        if cores:
            kw["cores"] = cores
        cluster.create("pods", amd_pod(name, **kw))
        pod = cluster.get_pod("default", name)
        cached, patches = len(s.pod_manager), cluster.count("patch", "pods")
        sim = s.filter({"Pod": pod, "Nodes": {"items": node_objs}})
        assert len(s.pod_manager) == cached and cluster.count("patch", "pods") == patches
        sim_node = [n["metadata"]["name"] for n in (sim.get("Nodes") or {}).get("items", [])]
        real = s.filter({"Pod": pod, "NodeNames": sorted(nodes)})
        assert sim_node == (real.get("NodeNames") or []), (i, pods[: i + 1], sim, real)
        cluster.delete("pods", name, "default")      # back to an empty cluster
        assert len(s.pod_manager) == 0
