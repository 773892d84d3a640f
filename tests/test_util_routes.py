"""pkg/util (util_test.go), pkg/util/nodelock (nodelock_test.go) and
pkg/scheduler/routes (route_test.go) counterparts, CPU only, on the fake API
server."""

import datetime as dt
import http.client
import json

import pytest

from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster, make_node, make_pod
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.routes import MAX_BODY, ExtenderServer
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.scheduler.webhook import Webhook
from k8s_vgpu_scheduler_amd.testing import amd_node, amd_pod
from k8s_vgpu_scheduler_amd.utils import nodelock, util
from k8s_vgpu_scheduler_amd.utils import types as T


@pytest.fixture
def cluster():
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    return c


# ---------------------------------------------------------------- util.go
def _pending(name, node, phase="Pending", bind_phase=T.DEVICE_BIND_ALLOCATING, assigned=None, bind_time=True):
    annos = {T.DEVICE_BIND_PHASE: bind_phase, T.ASSIGNED_NODE_ANNOTATION: assigned or node}
    if bind_time:
        annos[T.BIND_TIME_ANNOTATION] = "123"
    p = make_pod(name, annotations=annos)
    p["spec"]["nodeName"] = node
    p["status"] = {"phase": phase}
    return p


def test_get_pending_pod_prefers_the_lock_holder(cluster):
    cluster.create("nodes", make_node("n1"))
    holder = make_pod("holder")
    cluster.create("pods", holder)
    cluster.create("pods", _pending("other", "n1"))
    nodelock.lock_node("n1", T.NODE_LOCK_KEY, cluster.get_pod("default", "holder"))
    assert util.get_pending_pod("n1")["metadata"]["name"] == "holder"


@pytest.mark.parametrize("kw,found", [
    ({}, True),
    ({"bind_phase": T.DEVICE_BIND_SUCCESS}, True),
    ({"bind_phase": T.DEVICE_BIND_FAILED}, False),
    ({"phase": "Running"}, False),
    ({"bind_time": False}, False),
    ({"assigned": "n2"}, False),
])
def test_get_pending_pod_filters(cluster, kw, found):
    cluster.create("nodes", make_node("n1"))
    cluster.create("pods", _pending("p", "n1", **kw))
    if found:
        assert util.get_pending_pod("n1")["metadata"]["name"] == "p"
    else:
        with pytest.raises(LookupError):
            util.get_pending_pod("n1")


def test_patch_pod_annotations_mirrors_assigned_node_label(cluster):
    cluster.create("pods", make_pod("p"))
    util.patch_pod_annotations(cluster.get_pod("default", "p"), {T.ASSIGNED_NODE_ANNOTATION: "n1", "x": "y"})
    p = cluster.get_pod("default", "p")
    assert p["metadata"]["annotations"]["x"] == "y"
    assert p["metadata"]["labels"][T.ASSIGNED_NODE_ANNOTATION] == "n1"


def test_remove_node_annotation(cluster):
    cluster.create("nodes", make_node("n1", annotations={"a": "1", "b": "2"}))
    util.remove_node_annotation("n1", "a")
    assert cluster.get_node("n1")["metadata"]["annotations"] == {"b": "2"}
    with pytest.raises(ValueError):
        util.get_node("")


@pytest.mark.parametrize("annos,expect", [({}, "spread"), ({T.GPU_POLICY_ANNOTATION: "binpack"}, "binpack")])
def test_gpu_policy_by_pod(annos, expect):
    assert util.get_gpu_scheduler_policy_by_pod("spread", make_pod("p", annotations=annos)) == expect
    assert util.get_gpu_scheduler_policy_by_pod("spread", None) == "spread"


@pytest.mark.parametrize("policy,name,hit", [("binpack,topology-aware", "topology-aware", True),
                                             ("binpack, numa", "numa", True), ("binpack", "bin", False),
                                             ("", "binpack", False)])
def test_policy_contains(policy, name, hit):
    assert util.policy_contains(policy, name) is hit


def test_pod_state_predicates():
    p = make_pod("p")
    assert not util.is_pod_terminated(p) and not util.is_pod_terminating(p)
    p["status"] = {"phase": "Succeeded"}
    assert util.is_pod_terminated(p)
    p["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
    assert util.is_pod_terminating(p)
    p["status"]["containerStatuses"] = [{}] * len(p["spec"]["containers"])
    assert util.all_containers_created(p)
    assert not util.all_init_containers_succeeded(p)
    p["status"]["initContainerStatuses"] = [{"state": {"terminated": {"exitCode": 0}}}]
    assert util.all_init_containers_succeeded(p)
    p["status"]["initContainerStatuses"].append({"state": {"terminated": {"exitCode": 2}}})
    assert not util.all_init_containers_succeeded(p)


def test_pod_group_member():
    assert not util.is_pod_group_member(make_pod("p"))
    assert util.is_pod_group_member(make_pod("p", labels={T.POD_GROUP_LABEL: "g"}))
    sg = make_pod("p")
    sg["spec"]["schedulingGroup"] = {"podGroupName": "g"}
    assert util.is_pod_group_member(sg)
    assert not util.is_pod_group_member(None)


def test_node_warning_event_dedup(cluster):
    node = make_node("n1")
    cluster.create("nodes", node)
    node = cluster.get_node("n1")
    util.emit_node_warning_event(node, "AsymmetricXGMI", "first")
    util.emit_node_warning_event(node, "AsymmetricXGMI", "second")
    util.emit_node_warning_event(node, "OtherReason", "x")
    evs = cluster.list("events", "default")
    mine = [e for e in evs if e["reason"] == "AsymmetricXGMI"]
    assert len(mine) == 1 and mine[0]["count"] == 2 and mine[0]["message"] == "second"
    assert len(evs) == 2


# ------------------------------------------------------------ nodelock.go
def test_parse_node_lock_formats():
    ts = dt.datetime(2026, 10, 16, 8, 30, 0, tzinfo=dt.timezone.utc)
    t, ns, name = nodelock.parse_node_lock(ts.strftime("%Y-%m-%dT%H:%M:%SZ") + ",ns1,pod1")
    assert (t, ns, name) == (ts, "ns1", "pod1")
    t, ns, name = nodelock.parse_node_lock(ts.strftime("%Y-%m-%dT%H:%M:%SZ"))   # legacy: time only
    assert t == ts and ns == "" and name == ""
    with pytest.raises(ValueError):
        nodelock.parse_node_lock("not-a-time,ns,pod")


def test_lock_by_other_pod_is_refused_then_released(cluster):
    cluster.create("nodes", make_node("n1"))
    a, b = make_pod("a"), make_pod("b")
    cluster.create("pods", a)
    cluster.create("pods", b)
    nodelock.lock_node("n1", T.NODE_LOCK_KEY, cluster.get_pod("default", "a"))
    with pytest.raises(Exception):
        nodelock.lock_node("n1", T.NODE_LOCK_KEY, cluster.get_pod("default", "b"))
    # a non-owner cannot release it
    nodelock.release_node_lock("n1", T.NODE_LOCK_KEY, cluster.get_pod("default", "b"))
    assert T.NODE_LOCK_KEY in cluster.get_node("n1")["metadata"]["annotations"]
    nodelock.release_node_lock("n1", T.NODE_LOCK_KEY, cluster.get_pod("default", "a"))
    assert T.NODE_LOCK_KEY not in cluster.get_node("n1")["metadata"]["annotations"]
    nodelock.lock_node("n1", T.NODE_LOCK_KEY, cluster.get_pod("default", "b"))


# --------------------------------------------------------------- route.go
@pytest.fixture
def server(cluster):
    cluster.create("nodes", amd_node("n1", n=1))
    s = Scheduler(cluster, SchedulerConfig())
    s.start()
    s.register()
    srv = ExtenderServer(s, Webhook("hami-scheduler"), "127.0.0.1:0", profiling=True).start()
    yield srv
    srv.stop()


def _req(port, method, path, body=None, headers=None):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    c.request(method, path, body=body, headers=headers or {})
    r = c.getresponse()
    data = r.read()
    c.close()
    return r.status, data


def test_route_empty_body_is_400(server):
    code, data = _req(server.port, "POST", "/filter")
    assert code == 400 and b"request body" in data


@pytest.mark.parametrize("path", ["/filter", "/bind"])
def test_route_invalid_json_reports_error(server, path):
    code, data = _req(server.port, "POST", path, body=b"{not json", headers={"Content-Type": "application/json"})
    assert code == 200 and json.loads(data)["Error"]


def test_route_body_over_one_mib_is_refused(server):
    big = b'{"Pod": "' + b"x" * (MAX_BODY + 10) + b'"}'
    code, data = _req(server.port, "POST", "/filter", body=big)
    assert code == 413
    # the server is still healthy for the next client
    assert _req(server.port, "GET", "/healthz")[0] == 200


def test_route_unknown_paths_and_pprof(server):
    assert _req(server.port, "GET", "/nope")[0] == 404
    assert _req(server.port, "POST", "/nope", body=b"{}")[0] == 404
    code, data = _req(server.port, "GET", "/debug/pprof/goroutine")
    assert code == 200 and b"thread" in data


def test_route_filter_reports_scheduling_failure(server, cluster):
    pod = amd_pod("huge", mem=10 ** 7)
    cluster.create("pods", pod)
    code, data = _req(server.port, "POST", "/filter",
                      body=json.dumps({"Pod": cluster.get_pod("default", "huge"), "NodeNames": ["n1"]}))
    res = json.loads(data)
    assert code == 200 and not res.get("NodeNames") and res["FailedNodes"]["n1"]


def test_route_bind_unknown_pod(server):
    code, data = _req(server.port, "POST", "/bind",
                      body=json.dumps({"PodName": "ghost", "PodNamespace": "default", "PodUID": "u", "Node": "n1"}))
    assert code == 200 and json.loads(data)["Error"]


def test_route_webhook_roundtrip(server):
    review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
              "request": {"uid": "r1", "object": amd_pod("w", gpu=1)}}
    code, data = _req(server.port, "POST", "/webhook", body=json.dumps(review))
    resp = json.loads(data)["response"]
    assert code == 200 and resp["uid"] == "r1" and resp["allowed"] and resp["patchType"] == "JSONPatch"
