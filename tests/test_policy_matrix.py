"""Table-driven GPU/node policy tests (model: pkg/scheduler/policy/gpu_policy_test.go,
node_policy_test.go and pkg/util/weights tests of the reference).

Conventions under test (scheduler/policy.py): devices sort ascending by
``less`` and Fit walks from the END, so the last element is the preferred one;
binpack prefers the fullest device, spread the emptiest, mutex the least-used.
"""

import pytest
from hypothesis import given, settings, strategies as st

from k8s_vgpu_scheduler_amd.device.types import ContainerDeviceRequest, DeviceUsage
from k8s_vgpu_scheduler_amd.scheduler.policy import (DeviceListsScore, DeviceUsageList, NodeScore,
                                                     NodeScoreList, sort_key_chain)
from k8s_vgpu_scheduler_amd.utils import types as T
from k8s_vgpu_scheduler_amd.utils.weights import DEFAULT_WEIGHTS, DeviceScoringWeights, parse_weights

GIB = 1024


def dev(i, used=0, count=10, usedmem=0, totalmem=288 * GIB, usedcores=0, totalcore=256,
        numa=0, typ="MI355X"):
    return DeviceUsage(id=f"GPU-{i}", index=i, used=used, count=count, usedmem=usedmem,
                       totalmem=totalmem, usedcores=usedcores, totalcore=totalcore, numa=numa, type=typ)


def req(nums=1, typ="MI355X", memreq=0, pct=101, cores=0):
    return ContainerDeviceRequest(nums=nums, type=typ, memreq=memreq, mem_percentage_req=pct, coresreq=cores)


def ordered(policy, devices, numa_bind=False, scores=None):
    lst = DeviceUsageList([DeviceListsScore(d, s) for d, s in zip(devices, scores or [0.0] * len(devices))],
                          policy, numa_bind)
    lst.sort()
    return [d.device.index for d in lst.device_lists]


# ------------------------------------------------------------ compute_score --

@pytest.mark.parametrize("name,d,reqs,weights,want", [
    ("empty device, no request", dev(0), {}, DEFAULT_WEIGHTS, 0.0),
    ("one slot of ten", dev(0), {"a": req()}, DEFAULT_WEIGHTS, 10 * (1 / 10)),
    ("used slots add to the request", dev(0, used=4), {"a": req()}, DEFAULT_WEIGHTS, 10 * (5 / 10)),
    ("memory in MiB", dev(0), {"a": req(memreq=144 * GIB)}, DEFAULT_WEIGHTS, 10 * (0.1 + 0.5)),
    ("memory percentage", dev(0), {"a": req(pct=25)}, DEFAULT_WEIGHTS, 10 * (0.1 + 0.25)),
    ("percentage 0 falls back to memreq", dev(0), {"a": req(memreq=72 * GIB, pct=0)}, DEFAULT_WEIGHTS,
     10 * (0.1 + 0.25)),
    ("core percent converted to CUs", dev(0), {"a": req(cores=50)}, DEFAULT_WEIGHTS, 10 * (0.1 + 0.5)),
    ("used CUs", dev(0, usedcores=64), {"a": req(cores=25)}, DEFAULT_WEIGHTS, 10 * (0.1 + 0.5)),
    ("all three", dev(0, used=1, usedmem=72 * GIB, usedcores=128), {"a": req(memreq=72 * GIB, cores=25)},
     DEFAULT_WEIGHTS, 10 * (0.2 + 0.75 + 0.5)),
    ("slot weight only", dev(0, used=4), {"a": req(memreq=144 * GIB)}, DeviceScoringWeights(1, 0, 0),
     10 * 0.5),
    ("memory weight doubled", dev(0), {"a": req(memreq=144 * GIB)}, DeviceScoringWeights(0, 0, 2),
     10 * 1.0),
    ("other family ignored", dev(0), {"a": req(typ="NVIDIA", memreq=144 * GIB)}, DEFAULT_WEIGHTS, 0.0),
    ("family matched case-insensitively", dev(0, typ="AMD-MI355X"), {"a": req(typ="mi355x")},
     DEFAULT_WEIGHTS, 10 * 0.1),
    ("zero-capacity device scores 0", dev(0, count=0), {"a": req()}, DEFAULT_WEIGHTS, 0.0),
    ("zero memory scores 0", dev(0, totalmem=0), {"a": req()}, DEFAULT_WEIGHTS, 0.0),
    ("percent-style cores (totalcore 100) not converted", dev(0, totalcore=100), {"a": req(cores=30)},
     DEFAULT_WEIGHTS, 10 * (0.1 + 0.3)),
])
def test_device_score(name, d, reqs, weights, want):
    s = DeviceListsScore(d)
    s.compute_score(reqs, weights)
    assert s.score == pytest.approx(want), name


def test_device_score_of_none_device():
    s = DeviceListsScore(None, 5.0)
    s.compute_score({"a": req()}, DEFAULT_WEIGHTS)
    assert s.score == 0.0


# ------------------------------------------------------------------- ordering --

@pytest.mark.parametrize("policy,scores,numas,numa_bind,want", [
    # binpack: highest score last; ties broken by numa ascending
    (T.GPU_POLICY_BINPACK, [1, 3, 2], [0, 0, 0], False, [0, 2, 1]),
    (T.GPU_POLICY_BINPACK, [2, 2, 2], [1, 0, 1], False, [1, 0, 2]),
    # spread: lowest score last
    (T.GPU_POLICY_SPREAD, [1, 3, 2], [0, 0, 0], False, [1, 2, 0]),
    (T.GPU_POLICY_SPREAD, [5, 5], [1, 0], False, [1, 0]),
    # numa bind groups by node first: binpack puts the lower numa last
    (T.GPU_POLICY_BINPACK, [1, 9, 2, 8], [0, 1, 0, 1], True, [3, 1, 0, 2]),
    # numa bind + spread: higher numa last, lowest score last within it
    (T.GPU_POLICY_SPREAD, [1, 9, 2, 8], [0, 1, 0, 1], True, [2, 0, 1, 3]),
    # chains: binpack then numa
    ("binpack,numa", [1, 1, 2], [1, 0, 0], False, [1, 0, 2]),
    # numa alone ascending; ties on index
    (T.GPU_POLICY_NUMA, [3, 1, 2], [1, 0, 1], False, [1, 0, 2]),
    # spread,numa
    ("spread,numa", [2, 2, 1], [1, 0, 0], False, [1, 0, 2]),
    # unknown keys ignored: "foo,binpack" is binpack
    ("foo,binpack", [1, 3, 2], [0, 0, 0], False, [0, 2, 1]),
    # chain of only unknown keys defaults to spread
    ("foo,bar", [1, 3, 2], [0, 0, 0], False, [1, 2, 0]),
    # numa bind forces numa first in a chain
    ("binpack,spread", [9, 1], [0, 1], True, [0, 1]),
])
def test_device_ordering(policy, scores, numas, numa_bind, want):
    devices = [dev(i, numa=n) for i, n in enumerate(numas)]
    assert ordered(policy, devices, numa_bind, [float(s) for s in scores]) == want


def test_mutex_prefers_least_used_device():
    devices = [dev(0, used=2), dev(1, used=0), dev(2, used=1)]
    assert ordered(T.GPU_POLICY_MUTEX, devices) == [0, 2, 1]


def test_mutex_ties_broken_by_numa():
    devices = [dev(0, used=1, numa=1), dev(1, used=1, numa=0)]
    assert ordered(T.GPU_POLICY_MUTEX, devices) == [1, 0]


@pytest.mark.parametrize("policy,want", [
    ("binpack", ["binpack"]),
    ("binpack,numa", ["binpack", "numa"]),
    (" spread , numa ,spread", ["spread", "numa"]),
    ("topology-aware", []),
    ("mutex,binpack", ["binpack"]),
    ("", []),
    (None, []),
])
def test_sort_key_chain(policy, want):
    assert sort_key_chain(policy) == want


def test_deepcopy_is_independent():
    lst = DeviceUsageList([DeviceListsScore(dev(0, used=1), 2.0)], T.GPU_POLICY_BINPACK, True)
    cp = lst.deepcopy()
    cp.device_lists[0].device.used = 7
    cp.device_lists[0].score = 9.0
    assert lst.device_lists[0].device.used == 1 and lst.device_lists[0].score == 2.0
    assert cp.policy == lst.policy and cp.numa_bind


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 50), st.integers(0, 3)), min_size=1, max_size=12),
       st.sampled_from([T.GPU_POLICY_BINPACK, T.GPU_POLICY_SPREAD]))
def test_preferred_device_is_extreme(items, policy):
    """Whatever the inputs, Fit's first pick (the last element) is the max-score
    device for binpack and the min-score device for spread."""
    devices = [dev(i, numa=n) for i, (_, n) in enumerate(items)]
    scores = [float(s) for s, _ in items]
    order = ordered(policy, devices, scores=scores)
    last = scores[order[-1]]
    assert last == (max(scores) if policy == T.GPU_POLICY_BINPACK else min(scores))
    assert sorted(order) == list(range(len(items)))


# --------------------------------------------------------------- node policy --

def _usage_list(*devices):
    return DeviceUsageList([DeviceListsScore(d) for d in devices])


@pytest.mark.parametrize("devices,want", [
    ([], 0.0),
    ([dev(0)], 0.0),
    ([dev(0, used=5, usedcores=128, usedmem=144 * GIB)], 10 * (0.5 + 0.5 + 0.5)),
    ([dev(0, used=10), dev(1)], 10 * 0.5),
    ([dev(0, usedcores=256), dev(1, usedcores=0)], 10 * 0.5),
])
def test_node_default_score(devices, want):
    ns = NodeScore("n", None)
    ns.compute_default_score(_usage_list(*devices))
    assert ns.score == pytest.approx(want)


@pytest.mark.parametrize("policy,scores,want_last", [
    (T.NODE_POLICY_BINPACK, {"a": 1.0, "b": 5.0, "c": 3.0}, "b"),
    (T.NODE_POLICY_SPREAD, {"a": 1.0, "b": 5.0, "c": 3.0}, "a"),
    (T.NODE_POLICY_BINPACK, {"a": 2.0}, "a"),
])
def test_node_ordering(policy, scores, want_last):
    nl = NodeScoreList([NodeScore(k, None, score=v) for k, v in scores.items()], policy)
    nl.sort()
    assert nl.node_list[-1].node_id == want_last


def test_snapshot_device_copies():
    lst = _usage_list(dev(0, used=3))
    snap = NodeScore.snapshot_device(lst)
    snap[0].used = 0
    assert lst.device_lists[0].device.used == 3


# ------------------------------------------------------------------- weights --

@pytest.mark.parametrize("value,want", [
    ("slot=1,core=1,memory=1", (1, 1, 1)),
    ("memory=3, slot=0 ,core=2", (0, 2, 3)),
    ("slot=10,core=0,memory=0", (10, 0, 0)),
])
def test_parse_weights(value, want):
    w = parse_weights(value)
    assert (w.slot, w.core, w.memory) == want


@pytest.mark.parametrize("value,msg", [
    ("slot=1,core=1", "expected slot, core, and memory"),
    ("slot=1,core=1,memory=1,extra=1", "expected slot, core, and memory"),
    ("slot=1,core,memory=1", "key=value"),
    ("slot=1,slot=2,memory=1", "duplicate"),
    ("slot=x,core=1,memory=1", "integer"),
    ("slot=-1,core=1,memory=1", "negative"),
    ("slot=1,core=1,disk=1", "unknown weight"),
])
def test_parse_weights_rejects(value, msg):
    with pytest.raises(ValueError, match=msg):
        parse_weights(value)
