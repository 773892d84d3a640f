"""xGMI pair-score and combination tables (device/amd/topology.py; reference
pkg/device/nvidia/calculate_score.go:177-286 and device.go:887-978)."""

from dataclasses import dataclass

import pytest
from hypothesis import given, settings, strategies as st

from k8s_vgpu_scheduler_amd.device.amd import topology as TP


@pytest.mark.parametrize("args,kw,want", [
    (("xgmi",), {}, 100),
    (("XGMI",), {"bw_gbps": 76.0}, 100),
    (("xgmi",), {"bw_gbps": 38.0}, 50),
    (("xgmi",), {"bw_gbps": 152.0}, 100),          # capped at nominal
    (("xgmi",), {"bw_gbps": 0.0}, 0),
    (("xgmi",), {"hops": 2}, 50),
    (("xgmi",), {"links": 2}, 200),
    (("xgmi",), {"hops": 0, "links": 0}, 100),     # degenerate counts clamp to 1
    (("pcie",), {"same_numa": True}, 20),
    (("PCIE",), {"same_numa": False}, 10),
    (("",), {}, 0), ((None,), {}, 0), (("nvlink",), {}, 0),
])
def test_pair_score(args, kw, want):
    assert TP.pair_score(*args, **kw) == want


def test_asymmetric_pairs_reported_once():
    scores = {"a": {"b": 100, "c": 20}, "b": {"a": 50, "c": 100}, "c": {"a": 20, "b": 100}}
    assert TP.is_asymmetric(scores) == [("a", "b")]
    assert TP.is_asymmetric({"a": {"b": 1}, "b": {"a": 1}}) == []


@dataclass
class Dev:
    uuid: str


def test_combination_and_single_choice():
    s = {"a": {"b": 100, "c": 10, "d": 10}, "b": {"a": 100, "c": 10, "d": 10},
         "c": {"a": 10, "b": 10, "d": 100}, "d": {"a": 10, "b": 10, "c": 100}}
    cands = [Dev(u) for u in "abcd"]
    assert sorted(d.uuid for d in TP.best_combination(cands, 2, s)) in (["a", "b"], ["c", "d"])
    assert TP.combination_score(["a", "b", "c"], s) == 120
    assert TP.mean_pair_score(["a", "b", "c"], s) == 40.0
    assert TP.mean_pair_score(["a"], s) == 0.0
    assert TP.worst_single([], s) == [] and TP.best_combination([], 2, s) == []


@settings(max_examples=60, deadline=None)
@given(st.integers(3, 6).flatmap(lambda n: st.tuples(
    st.just(n), st.lists(st.integers(0, 100), min_size=n * (n - 1) // 2, max_size=n * (n - 1) // 2))),
    st.integers(1, 3))
def test_worst_single_keeps_the_best_connected_free(nv, k):
    n, vals = nv
    ids = [f"g{i}" for i in range(n)]
    s = {u: {} for u in ids}
    it = iter(vals)
    for i in range(n):
        for j in range(i + 1, n):
            v = next(it)
            s[ids[i]][ids[j]] = s[ids[j]][ids[i]] = v
    cands = [Dev(u) for u in ids]
    (w,) = TP.worst_single(cands, s)
    tot = {u: sum(s[u].values()) for u in ids}
    assert tot[w.uuid] == min(tot.values())
    k = min(k, n)
    best = TP.best_combination(cands, k, s)
    from itertools import combinations
    assert TP.combination_score([d.uuid for d in best], s) == max(
        TP.combination_score(list(c), s) for c in combinations(ids, k))
