"""Scheduler event handlers, Bind failure paths and Filter outcomes
(pkg/scheduler/scheduler_test.go counterparts: onAddPod/onUpdatePod/onDelPod,
onDelNode, Bind with lock contention and API failures, PodGroup lock retry,
FilteringFailed/Succeed events), on the fake API server."""

import threading
import time

import pytest

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device.amd.device import SUPPORT_ANNOS
from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.k8s.client import Conflict, init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster, make_pod
from k8s_vgpu_scheduler_amd.scheduler import events as E
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.testing import amd_container, amd_node, amd_pod
from k8s_vgpu_scheduler_amd.utils import nodelock
from k8s_vgpu_scheduler_amd.utils import types as T


@pytest.fixture
def cluster():
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    return c


def make_sched(cluster, nodes, **cfg):
    for n in nodes:
        cluster.create("nodes", n)
    s = Scheduler(cluster, SchedulerConfig(**cfg))
    s.start()
    s.register()
    assert s.synced
    return s


def filt(s, cluster, pod, nodes):
    cluster.create("pods", pod)
    return s.filter({"Pod": cluster.get_pod("default", pod["metadata"]["name"]), "NodeNames": nodes})


def used_mem(s, node="n1", idx=0):
    _, overall, _ = s.get_nodes_usage([node], None)
    return overall[node].devices.device_lists[idx].device.usedmem


def events(cluster, reason):
    return [e for e in cluster.list("events", "default") if e.get("reason") == reason]


# -------------------------------------------------------------- filter
def test_pod_without_device_requests_passes_through(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])
    pod = make_pod("cpu-only")
    cluster.create("pods", pod)
    res = s.filter({"Pod": cluster.get_pod("default", "cpu-only"), "NodeNames": ["n1", "n2"]})
    assert res["NodeNames"] == ["n1", "n2"] and res["Error"] == ""
    assert cluster.count("patch", "pods") == 0


def test_filter_events_success_and_failure(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])
    filt(s, cluster, amd_pod("ok", mem=1000), ["n1"])
    ok = events(cluster, E.FILTERING_SUCCEED)
    assert ok and "find fit node(n1)" in ok[-1]["message"]
    filt(s, cluster, amd_pod("no", mem=10 ** 7), ["n1"])
    bad = [e["message"] for e in events(cluster, E.FILTERING_FAILED)]
    assert any("CardInsufficientMemory" in m for m in bad)
    assert any(m.startswith("no available node") for m in bad)


def test_filter_picks_best_node_by_policy(cluster):
    s = make_sched(cluster, [amd_node("n1", n=2), amd_node("n2", n=2)], node_scheduler_policy="binpack")
    assert filt(s, cluster, amd_pod("a", mem=200000), ["n1"])["NodeNames"] == ["n1"]
    # binpack: the busier node wins
    assert filt(s, cluster, amd_pod("b", mem=1000), ["n1", "n2"])["NodeNames"] == ["n1"]


def test_filter_spread_node_policy_prefers_the_idle_node(cluster):
    s = make_sched(cluster, [amd_node("n1", n=2), amd_node("n2", n=2)], node_scheduler_policy="spread")
    filt(s, cluster, amd_pod("a", mem=200000), ["n1"])
    assert filt(s, cluster, amd_pod("b", mem=1000), ["n1", "n2"])["NodeNames"] == ["n2"]


def test_pod_annotation_overrides_node_policy(cluster):
    s = make_sched(cluster, [amd_node("n1", n=2), amd_node("n2", n=2)], node_scheduler_policy="spread")
    filt(s, cluster, amd_pod("a", mem=200000), ["n1"])
    pod = amd_pod("b", mem=1000, annotations={T.NODE_POLICY_ANNOTATION: "binpack"})
    assert filt(s, cluster, pod, ["n1", "n2"])["NodeNames"] == ["n1"]


def test_two_containers_two_allocations(cluster):
    s = make_sched(cluster, [amd_node("n1", n=2)])
    pod = amd_pod("p", containers=[amd_container("a", mem=1000), amd_container("b", mem=2000)])
    assert filt(s, cluster, pod, ["n1"])["NodeNames"] == ["n1"]
    parts = cluster.get_pod("default", "p")["metadata"]["annotations"][SUPPORT_ANNOS].split(";")
    a, b = codec.decode_container_devices(parts[0]), codec.decode_container_devices(parts[1])
    assert (a[0].usedmem, b[0].usedmem) == (1000, 2000)


def test_patch_failure_rolls_back_the_cache(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])

    def boom(verb, kind, name, ns, payload):
        if name == "p":
            raise Conflict("injected")
    r = cluster.add_reactor("patch", "pods", boom)
    res = filt(s, cluster, amd_pod("p", mem=1000), ["n1"])
    cluster.remove_reactor(r)
    assert "injected" in res["Error"]
    assert len(s.pod_manager) == 0 and used_mem(s) == 0


# ------------------------------------------------------------- handlers
def test_terminated_pod_releases_usage(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])
    filt(s, cluster, amd_pod("a", mem=5000), ["n1"])
    assert used_mem(s) == 5000
    p = cluster.get_pod("default", "a")
    p["status"] = {"phase": "Succeeded"}
    cluster.update("pods", p)
    assert used_mem(s) == 0 and len(s.pod_manager) == 0


def test_terminating_pod_keeps_usage(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])
    filt(s, cluster, amd_pod("a", mem=5000), ["n1"])
    p = cluster.get_pod("default", "a")
    p["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
    cluster.update("pods", p)
    assert used_mem(s) == 5000


def test_init_containers_done_shrinks_usage_and_quota(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])
    cluster.create("resourcequotas", {"metadata": {"name": "q", "namespace": "default"},
                                      "spec": {"hard": {"limits.amd.com/gpumem": "500000"}}})
    pod = amd_pod("p", containers=[amd_container("app", mem=1000)], init=[amd_container("init", mem=9000)])
    filt(s, cluster, pod, ["n1"])
    assert used_mem(s) == 9000
    assert get_local_cache().get_resource_quota()["default"]["amd.com/gpumem"].used == 9000
    p = cluster.get_pod("default", "p")
    p["status"] = {"phase": "Running", "initContainerStatuses": [{"state": {"terminated": {"exitCode": 0}}}]}
    cluster.update("pods", p)
    assert used_mem(s) == 1000
    assert get_local_cache().get_resource_quota()["default"]["amd.com/gpumem"].used == 1000


def test_failed_init_container_keeps_peak(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])
    filt(s, cluster, amd_pod("p", containers=[amd_container("app", mem=1000)],
                             init=[amd_container("init", mem=9000)]), ["n1"])
    p = cluster.get_pod("default", "p")
    p["status"] = {"phase": "Pending", "initContainerStatuses": [{"state": {"terminated": {"exitCode": 1}}}]}
    cluster.update("pods", p)
    assert used_mem(s) == 9000


def test_malformed_allocation_annotation_is_ignored(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])
    pod = amd_pod("bad", annotations={T.ASSIGNED_NODE_ANNOTATION: "n1", SUPPORT_ANNOS: "n1-gpu0,AMD,xx,1:;"})
    cluster.create("pods", pod)
    assert len(s.pod_manager) == 0 and used_mem(s) == 0


def test_pod_added_with_existing_allocation_counts(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])
    pod = amd_pod("adopted", annotations={T.ASSIGNED_NODE_ANNOTATION: "n1",
                                          SUPPORT_ANNOS: "n1-gpu0,AMD,7000,0:;"})
    cluster.create("pods", pod)
    assert used_mem(s) == 7000


def test_node_deletion_drops_node_and_lock(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1), amd_node("n2", n=1)])
    filt(s, cluster, amd_pod("a", mem=1000), ["n1"])
    cluster.delete("nodes", "n1")
    res = filt(s, cluster, amd_pod("b", mem=1000), ["n1", "n2"])
    assert res["NodeNames"] == ["n2"] and res["FailedNodes"]["n1"] == "node unregistered"


# ------------------------------------------------------------------ bind
def test_bind_failure_releases_lock_and_records_event(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])
    filt(s, cluster, amd_pod("a", mem=1000), ["n1"])

    def refuse(verb, kind, name, ns, payload):
        raise Conflict("apiserver says no")
    r = cluster.add_reactor("create", "bindings", refuse)
    res = s.bind({"PodName": "a", "PodNamespace": "default", "Node": "n1"})
    cluster.remove_reactor(r)
    assert "apiserver says no" in res["Error"]
    assert T.NODE_LOCK_KEY not in (cluster.get_node("n1")["metadata"].get("annotations") or {})
    assert events(cluster, E.BINDING_FAILED)
    # and the next bind works
    assert s.bind({"PodName": "a", "PodNamespace": "default", "Node": "n1"})["Error"] == ""
    assert events(cluster, E.BINDING_SUCCEED)


def test_bind_unknown_node_cleans_stale_allocation(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])
    filt(s, cluster, amd_pod("a", mem=1000), ["n1"])
    res = s.bind({"PodName": "a", "PodNamespace": "default", "Node": "ghost"})
    assert res["Error"] and len(s.pod_manager) == 0


def test_bind_deleted_pod_cleans_stale_allocation(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)])
    filt(s, cluster, amd_pod("a", mem=1000), ["n1"])
    uid = cluster.get_pod("default", "a")["metadata"]["uid"]
    cluster._store("pods").clear()          # the API server lost it; the informer still caches it
    res = s.bind({"PodName": "a", "PodNamespace": "default", "PodUID": uid, "Node": "n1"})
    assert res["Error"]


def test_pod_group_member_waits_for_the_lock(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)], node_lock_retry_timeout=5.0)
    holder = amd_pod("holder", mem=1)
    cluster.create("pods", holder)
    nodelock.lock_node("n1", T.NODE_LOCK_KEY, cluster.get_pod("default", "holder"))
    filt(s, cluster, amd_pod("member", mem=1000, labels={T.POD_GROUP_LABEL: "g1"}), ["n1"])

    def release():
        time.sleep(0.4)
        nodelock.release_node_lock("n1", T.NODE_LOCK_KEY, cluster.get_pod("default", "holder"))
    t = threading.Thread(target=release)
    t.start()
    t0 = time.time()
    res = s.bind({"PodName": "member", "PodNamespace": "default", "Node": "n1"})
    t.join()
    assert res["Error"] == "" and time.time() - t0 >= 0.3


def test_pod_group_member_times_out(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)], node_lock_retry_timeout=0.3)
    holder = amd_pod("holder", mem=1)
    cluster.create("pods", holder)
    nodelock.lock_node("n1", T.NODE_LOCK_KEY, cluster.get_pod("default", "holder"))
    filt(s, cluster, amd_pod("member", mem=1000, labels={T.POD_GROUP_LABEL: "g1"}), ["n1"])
    res = s.bind({"PodName": "member", "PodNamespace": "default", "Node": "n1"})
    assert "timed out" in res["Error"]


def test_plain_pod_does_not_wait_for_the_lock(cluster):
    s = make_sched(cluster, [amd_node("n1", n=1)], node_lock_retry_timeout=5.0)
    holder = amd_pod("holder", mem=1)
    cluster.create("pods", holder)
    nodelock.lock_node("n1", T.NODE_LOCK_KEY, cluster.get_pod("default", "holder"))
    filt(s, cluster, amd_pod("solo", mem=1000), ["n1"])
    t0 = time.time()
    res = s.bind({"PodName": "solo", "PodNamespace": "default", "Node": "n1"})
    assert res["Error"] and time.time() - t0 < 2.0
