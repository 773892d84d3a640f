"""RestClient (the client every binary uses in a cluster) against the HTTP
API server of the e2e tier: CRUD, merge patch, optimistic concurrency,
bind, selectors, watch replay/streaming/re-watch, 410 Gone, Status errors."""

import threading
import time

import pytest
import requests

from k8s_vgpu_scheduler_amd.e2e.apiserver import FakeApiServer
from k8s_vgpu_scheduler_amd.k8s.client import AlreadyExists, ApiError, Conflict, NotFound
from k8s_vgpu_scheduler_amd.k8s.fake import make_node, make_pod
from k8s_vgpu_scheduler_amd.k8s.informer import Informer
from k8s_vgpu_scheduler_amd.k8s.rest import RestClient


@pytest.fixture
def srv(tmp_path):
    s = FakeApiServer(bookmark_s=0.2, max_watch_s=1.0).start()
    cli = RestClient.from_env(s.write_kubeconfig(str(tmp_path / "kubeconfig")), qps=0)
    yield s, cli
    s.stop()


def _until(cond, timeout=5.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if cond():
            return True
        time.sleep(0.02)
    return False


def test_crud_patch_conflict_and_errors(srv):
    s, c = srv
    c.create("nodes", make_node("n1", labels={"gpu": "mi355x"}))
    c.create("nodes", make_node("n2"))
    with pytest.raises(AlreadyExists):
        c.create("nodes", make_node("n1"))
    assert [n["metadata"]["name"] for n in c.list("nodes", label_selector={"gpu": "mi355x"})] == ["n1"]
    n1 = c.get("nodes", "n1")
    c.patch("nodes", "n1", {"metadata": {"annotations": {"a": "1"}}})
    with pytest.raises(Conflict):        # stale resourceVersion
        c.patch("nodes", "n1", {"metadata": {"resourceVersion": n1["metadata"]["resourceVersion"],
                                             "annotations": {"a": "2"}}})
    cur = c.get("nodes", "n1")
    assert cur["metadata"]["annotations"] == {"a": "1"}
    c.patch("nodes", "n1", {"metadata": {"annotations": {"a": None}}})      # null deletes
    assert "a" not in (c.get("nodes", "n1")["metadata"].get("annotations") or {})
    with pytest.raises(Conflict):
        c.update("nodes", n1)
    c.delete("nodes", "n2")
    with pytest.raises(NotFound):
        c.get("nodes", "n2")
    with pytest.raises(ApiError) as e:
        c._req("PATCH", c._url("nodes", "n1"), data="{}", headers={"Content-Type": "application/json-patch+json"})
    assert e.value.code == 415


def test_pods_bind_and_field_selector(srv):
    s, c = srv
    c.create("pods", make_pod("p", namespace="ns1"))
    p = c.get_pod("ns1", "p")
    c.bind("ns1", "p", "n1", p["metadata"]["uid"])
    assert c.get_pod("ns1", "p")["spec"]["nodeName"] == "n1"
    with pytest.raises(Conflict):
        c.bind("ns1", "p", "n2")
    c.create("pods", make_pod("q", namespace="ns2"))
    assert [x["metadata"]["name"] for x in c.list_pods(field_selector={"spec.nodeName": "n1"})] == ["p"]
    assert [x["metadata"]["name"] for x in c.list_pods("ns2")] == ["q"]


def test_watch_streams_and_rewatches(srv):
    s, c = srv
    c.create("pods", make_pod("a"))
    seen = []
    stop = c.watch("pods", lambda t, o, old: seen.append((t, o["metadata"]["name"])))
    try:
        assert _until(lambda: ("ADDED", "a") in seen)
        c.create("pods", make_pod("b"))
        time.sleep(1.3)                                   # the stream ends; the client re-watches
        c.patch_pod("default", "b", {"metadata": {"labels": {"x": "y"}}})
        c.delete("pods", "a", "default")
        assert _until(lambda: ("MODIFIED", "b") in seen and ("DELETED", "a") in seen)
        assert seen.count(("ADDED", "b")) == 1
    finally:
        stop()


def test_watch_from_compacted_version_is_gone(srv):
    s, c = srv
    c.create("nodes", make_node("n1"))
    c.patch("nodes", "n1", {"metadata": {"labels": {"k": "v"}}})
    s.compact("nodes")
    r = requests.get(f"{s.url}/api/v1/nodes", params={"watch": "1", "resourceVersion": "1"}, timeout=5)
    assert r.status_code == 410 and r.json()["reason"] == "Expired"
    # a list gives a current version a watch can resume from
    rv = c._req("GET", c._url("nodes"))["metadata"]["resourceVersion"]
    r = requests.get(f"{s.url}/api/v1/nodes", params={"watch": "1", "resourceVersion": rv, "timeoutSeconds": "1"},
                     timeout=5, stream=True)
    assert r.status_code == 200


def test_informer_over_http(srv):
    s, c = srv
    inf = Informer(c, "nodes")
    inf.start()
    try:
        c.create("nodes", make_node("n9"))
        assert _until(lambda: any(n["metadata"]["name"] == "n9" for n in inf.list()))
        c.delete("nodes", "n9")
        assert _until(lambda: not inf.list())
    finally:
        inf.stop()


def test_eviction_api(srv):
    """POST pods/<name>/eviction (policy/v1): the monitor's --over-grant-action=evict."""
    s, c = srv
    c.create("pods", make_pod("victim", "ns1"))
    c.evict("ns1", "victim")
    assert s.cluster.evictions == [("ns1", "victim")]
    with pytest.raises(NotFound):
        c.get_pod("ns1", "victim")
    assert ("POST", "/api/v1/namespaces/ns1/pods/victim/eviction") in s.requests
    with pytest.raises(NotFound):
        c.evict("ns1", "victim")
