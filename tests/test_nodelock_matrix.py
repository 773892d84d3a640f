"""Node-lock tables (model: pkg/util/nodelock/nodelock_test.go — Test_LockNode,
TestReleaseNodeLock, TestGeneratePodNamespaceName, the conflict-preservation
cases and TestSetupNodeLockTimeout), against utils/nodelock.py."""

import datetime as dt

import pytest

from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.k8s.client import Conflict, init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster, make_node, make_pod
from k8s_vgpu_scheduler_amd.scheduler.config import init_devices_with_config
from k8s_vgpu_scheduler_amd.utils import nodelock
from k8s_vgpu_scheduler_amd.utils import types as T

KEY = T.NODE_LOCK_KEY


@pytest.fixture
def cluster(monkeypatch):
    monkeypatch.setattr(nodelock, "BACKOFF_BASE", 0.001)
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    return c


def _lock(cluster, node="n"):
    return (cluster.get_node(node)["metadata"].get("annotations") or {}).get(KEY)


def _ts(minutes_ago=0):
    t = dt.datetime.now().astimezone() - dt.timedelta(minutes=minutes_ago)
    return t.replace(microsecond=0).isoformat()


@pytest.mark.parametrize("s,want", [
    ("5m", 300.0), ("30s", 30.0), ("1h30m", 5400.0), ("250ms", 0.25), ("1.5s", 1.5),
    ("100us", 1e-4), ("2h0m0s", 7200.0),
])
def test_parse_go_duration(s, want):
    assert nodelock.parse_go_duration(s) == pytest.approx(want)


@pytest.mark.parametrize("s", ["", "5", "m", "5x", "5m junk", "-5m", "5 m"])
def test_parse_go_duration_rejects(s):
    with pytest.raises(ValueError):
        nodelock.parse_go_duration(s)


@pytest.mark.parametrize("env,want", [(None, 300.0), ("90s", 90.0), ("bogus", 300.0), ("10m", 600.0)])
def test_timeout_from_env(monkeypatch, env, want):
    if env is None:
        monkeypatch.delenv("HAMI_NODELOCK_EXPIRE", raising=False)
    else:
        monkeypatch.setenv("HAMI_NODELOCK_EXPIRE", env)
    assert nodelock._timeout_from_env() == want


@pytest.mark.parametrize("pod,sep,want", [
    (make_pod("a", "ns1"), ",", "ns1,a"),
    (make_pod("a", "ns1"), "", "ns1a"),
    (make_pod("a", "ns1"), "/#", "ns1/#a"),
    (None, ",", ""),
])
def test_pod_ns_name(pod, sep, want):
    assert nodelock.pod_ns_name(pod, sep) == want


def test_parse_node_lock_forms():
    t, ns, name = nodelock.parse_node_lock(f"{_ts()},ns1,p")
    assert (ns, name) == ("ns1", "p") and t.tzinfo is not None
    t, ns, name = nodelock.parse_node_lock("2026-01-02T03:04:05Z")
    assert (ns, name) == ("", "") and t.year == 2026 and t.utcoffset() == dt.timedelta(0)
    with pytest.raises(nodelock.NodeLockError, match="3 parts"):
        nodelock.parse_node_lock(f"{_ts()},ns1")
    with pytest.raises(ValueError):
        nodelock.parse_node_lock("not-a-time")


def test_generate_lock_value_round_trips():
    p = make_pod("a", "ns1")
    t, ns, name = nodelock.parse_node_lock(nodelock.generate_lock_value(p))
    assert (ns, name) == ("ns1", "a")
    assert abs((dt.datetime.now(t.tzinfo) - t).total_seconds()) < 5
    legacy = nodelock.generate_lock_value(None)
    assert "," not in legacy


# --------------------------------------------------------------- lock_node --

def test_lock_missing_node_raises(cluster):
    with pytest.raises(Exception):
        nodelock.lock_node("absent", "x", make_pod("a"))


def test_lock_held_by_live_pod_same_namespace(cluster):
    cluster.create("pods", make_pod("owner"))
    cluster.create("nodes", make_node("n", annotations={KEY: f"{_ts()},default,owner"}))
    with pytest.raises(nodelock.NodeLockContention):
        nodelock.lock_node("n", "x", make_pod("other"))
    assert _lock(cluster).endswith(",default,owner")


def test_malformed_lock_is_an_error(cluster):
    cluster.create("nodes", make_node("n", annotations={KEY: f"{_ts()},only-two"}))
    with pytest.raises(nodelock.NodeLockError):
        nodelock.lock_node("n", "x", make_pod("a"))


def test_fresh_legacy_lock_blocks(cluster):
    """A bare-timestamp lock names no owner to check: it blocks until it expires."""
    cluster.create("nodes", make_node("n", annotations={KEY: _ts()}))
    with pytest.raises(nodelock.NodeLockContention):
        nodelock.lock_node("n", "x", make_pod("a"))


def test_expired_legacy_lock_taken_over(cluster):
    cluster.create("nodes", make_node("n", annotations={KEY: _ts(minutes_ago=10)}))
    p = make_pod("a")
    cluster.create("pods", p)
    nodelock.lock_node("n", "x", p)
    assert _lock(cluster).endswith(",default,a")


def test_lock_sets_owner_value(cluster):
    cluster.create("nodes", make_node("n"))
    p = make_pod("a", "team")
    nodelock.lock_node("n", "x", p)
    _, ns, name = nodelock.parse_node_lock(_lock(cluster))
    assert (ns, name) == ("team", "a")


# ------------------------------------------------------- release_node_lock --

def test_release_nil_pod_is_an_error(cluster):
    cluster.create("nodes", make_node("n"))
    with pytest.raises(nodelock.NodeLockError, match="nil"):
        nodelock.release_node_lock("n", "x", None)


def test_release_unlocked_node_is_a_no_op(cluster):
    cluster.create("nodes", make_node("n"))
    nodelock.release_node_lock("n", "x", make_pod("a"))
    assert _lock(cluster) is None


def test_release_legacy_lock_by_any_pod(cluster):
    cluster.create("nodes", make_node("n", annotations={KEY: _ts()}))
    nodelock.release_node_lock("n", "x", make_pod("a"))
    assert _lock(cluster) is None


def test_release_skip_owner_check_releases_foreign_lock(cluster):
    cluster.create("nodes", make_node("n", annotations={KEY: f"{_ts()},default,b"}))
    nodelock.release_node_lock("n", "x", make_pod("a"), skip_owner_check=True)
    assert _lock(cluster) is None


def test_release_preserves_lock_taken_by_another_pod_after_conflict(cluster):
    """Our release PATCH conflicts; meanwhile another pod's lock replaced ours.
    The retry must leave the new owner's lock in place."""
    cluster.create("nodes", make_node("n", annotations={KEY: f"{_ts()},default,a"}))
    fired = []

    def swap_then_conflict(verb, kind, name, ns, payload):
        if not fired:
            fired.append(1)
            cluster.patch_node("n", {"metadata": {"annotations": {KEY: f"{_ts()},default,b"}}})
            raise Conflict("stale")
    r = cluster.add_reactor("patch", "nodes", swap_then_conflict)
    nodelock.release_node_lock("n", "x", make_pod("a"))
    cluster.remove_reactor(r)
    assert fired and _lock(cluster).endswith(",default,b")


def test_release_restamped_lock_of_same_pod(cluster):
    """The same pod re-stamped its lock between read and PATCH: still ours, released."""
    cluster.create("nodes", make_node("n", annotations={KEY: f"{_ts(1)},default,a"}))
    fired = []

    def restamp_then_conflict(verb, kind, name, ns, payload):
        if not fired:
            fired.append(1)
            cluster.patch_node("n", {"metadata": {"annotations": {KEY: f"{_ts()},default,a"}}})
            raise Conflict("stale")
    r = cluster.add_reactor("patch", "nodes", restamp_then_conflict)
    nodelock.release_node_lock("n", "x", make_pod("a"))
    cluster.remove_reactor(r)
    assert fired and _lock(cluster) is None


def test_set_preserves_concurrent_lock_after_conflict(cluster):
    """Our acquire PATCH conflicts because another pod locked first: we must see
    contention, not overwrite its lock."""
    cluster.create("nodes", make_node("n"))
    fired = []

    def lock_then_conflict(verb, kind, name, ns, payload):
        if not fired:
            fired.append(1)
            cluster.patch_node("n", {"metadata": {"annotations": {KEY: f"{_ts()},default,b"}}})
            raise Conflict("stale")
    r = cluster.add_reactor("patch", "nodes", lock_then_conflict)
    with pytest.raises(nodelock.NodeLockContention):
        nodelock.set_node_lock("n", "x", make_pod("a"))
    cluster.remove_reactor(r)
    assert _lock(cluster).endswith(",default,b")


def test_persistent_errors_surface_as_node_lock_error(cluster):
    cluster.create("nodes", make_node("n"))

    def always(verb, kind, name, ns, payload):
        raise Conflict("stale")
    cluster.add_reactor("patch", "nodes", always)
    with pytest.raises(nodelock.NodeLockError):
        nodelock.set_node_lock("n", "x", make_pod("a"))


def test_cleanup_node_lock_drops_the_mutex():
    m = nodelock._node_mutex("gone-node")
    assert nodelock._node_mutex("gone-node") is m
    nodelock.cleanup_node_lock("gone-node")
    assert nodelock._node_mutex("gone-node") is not m
