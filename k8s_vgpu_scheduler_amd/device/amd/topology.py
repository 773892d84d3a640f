"""xGMI topology scoring for multi-GPU placement on MI355X nodes.

Reference: NVLink/P2P pair scoring (pkg/device/nvidia/calculate_score.go:177-286,
links.go:411-481) and the combination search of nvidia/device.go:887-978.

MI355X: every GPU of an 8-GPU node has 7 xGMI links, one to each peer
(fully connected, 1 hop), so healthy nodes score every intra-node pair the
same and the scorer's job is to (a) prefer xGMI over PCIe peers (mixed or
partitioned systems) and (b) steer around degraded links, measured as the
min/max xGMI bandwidth amd-smi reports.  Pair score:

    xGMI:  100 * links * min(1, bw_GBps / nominal_GBps) / hops
           (nominal 76 GB/s per link per direction: KFD io_link min = max
           bandwidth 76000 MB/s on every GPU pair of a healthy 8 x MI355X
           node, = amd-smi link_metrics 608 Gb/s; tests/fixtures/mi355x_8gpu_kfd_links.json)
    PCIe:  20 same NUMA node, 10 cross-socket
    none:  0
"""

from __future__ import annotations

from itertools import combinations

XGMI_NOMINAL_GBPS = 76.0


def pair_score(link_type: str, hops: int = 1, links: int = 1, bw_gbps: float | None = None,
               same_numa: bool = True) -> int:
    lt = (link_type or "").upper()
    if lt == "XGMI":
        frac = 1.0 if bw_gbps is None else max(0.0, min(1.0, bw_gbps / XGMI_NOMINAL_GBPS))
        return int(round(100 * max(1, links) * frac / max(1, hops)))
    if lt == "PCIE":
        return 20 if same_numa else 10
    return 0


def is_asymmetric(scores: dict[str, dict[str, int]]) -> list[tuple[str, str]]:
    """Pairs whose two directions disagree (reference emits a node warning and scores 0)."""
    bad = []
    for a, row in scores.items():
        for b, s in row.items():
            if scores.get(b, {}).get(a, s) != s and (b, a) not in bad:
                bad.append((a, b))
    return bad


def combination_score(uuids, scores: dict[str, dict[str, int]]) -> int:
    return sum(scores.get(a, {}).get(b, 0) for a, b in combinations(uuids, 2))


def worst_single(candidates: list, scores: dict[str, dict[str, int]]):
    """For a 1-GPU request keep well-connected GPUs free: pick the candidate
    with the LOWEST total score to the other candidates (device.go:927-951)."""
    best, best_s = None, None
    for d in candidates:
        s = sum(scores.get(d.uuid, {}).get(o.uuid, 0) for o in candidates if o.uuid != d.uuid)
        if best is None or s < best_s:
            best, best_s = d, s
    return [best] if best is not None else []


def best_combination(candidates: list, k: int, scores: dict[str, dict[str, int]]):
    """Highest total pair score among all C(n, k) subsets (device.go:953-978);
    C(8, 4) = 70 on an 8-GPU node."""
    best, best_s = None, -1
    for combo in combinations(candidates, k):
        s = combination_score([d.uuid for d in combo], scores)
        if s > best_s:
            best, best_s = list(combo), s
    return best or []


def mean_pair_score(uuids, scores: dict[str, dict[str, int]]) -> float:
    pairs = list(combinations(uuids, 2))
    if not pairs:
        return 0.0
    return sum(scores.get(a, {}).get(b, 0) for a, b in pairs) / len(pairs)
