"""Leader-election edge tables (utils/leaderelection.py; reference
pkg/util/leaderelection/leaderelection_test.go)."""

import pytest

from k8s_vgpu_scheduler_amd.utils.leaderelection import DummyLeaderManager, LeaderManager


def lease(holder="sched-0_x", dur=15, name="hami-scheduler", ns="kube-system", rv="1"):
    spec = {"holderIdentity": holder}
    if dur is not None:
        spec["leaseDurationSeconds"] = dur
    return {"metadata": {"name": name, "namespace": ns, "resourceVersion": rv}, "spec": spec}


def mgr(clock, events=None):
    ev = events if events is not None else []
    return LeaderManager("sched-0", "kube-system", "hami-scheduler", on_started=lambda: ev.append("up"),
                         on_stopped=lambda: ev.append("down"), clock=lambda: clock[0])


@pytest.mark.parametrize("name,l,want", [
    ("holder is this pod", lease(), True),
    ("holder is another pod", lease(holder="sched-1_x"), False),
    ("empty holder", lease(holder=""), False),
    ("no lease duration", lease(dur=None), False),
    ("zero lease duration", lease(dur=0), False),
    ("hostname prefix match (kube-scheduler appends a suffix)", lease(holder="sched-0"), True),
])
def test_is_leader(name, l, want):
    clock = [10.0]
    m = mgr(clock)
    m.on_add(l)
    assert m.is_leader() == want, name


@pytest.mark.parametrize("l", [lease(name="other-lease"), lease(ns="default")])
def test_foreign_leases_ignored(l):
    clock = [10.0]
    m = mgr(clock)
    m.on_add(l)
    assert not m.is_leader()


def test_delete_stops_leading():
    clock, ev = [10.0], []
    m = mgr(clock, ev)
    m.on_add(lease())
    m.on_delete(lease())
    assert not m.is_leader() and ev == ["up", "down"]


def test_started_fires_once_per_term():
    clock, ev = [10.0], []
    m = mgr(clock, ev)
    m.on_add(lease(rv="1"))
    m.on_update(lease(rv="1"), lease(rv="2"))
    m.on_update(lease(rv="2"), lease(rv="3"))
    assert ev == ["up"]
    m.on_update(lease(rv="3"), lease(holder="sched-9_x", rv="4"))
    m.on_update(lease(holder="sched-9_x", rv="4"), lease(rv="5"))
    assert ev == ["up", "down", "up"]


def test_explicit_now_argument():
    clock = [100.0]
    m = mgr(clock)
    m.on_add(lease(dur=15))
    assert m.is_leader(now=114.9) and not m.is_leader(now=115.0)


@pytest.mark.parametrize("flag", [True, False])
def test_dummy_manager(flag):
    d = DummyLeaderManager(flag)
    d.on_lease({"anything": 1})
    assert d.is_leader() is flag
