"""XCD-balanced CU-range allocator for ``HSA_CU_MASK`` partitions on MI355X.

The reference only converts ``amd.com/gpucores`` % into a CU *count*
(pkg/device/amd/device.go:333-344) and leaves choosing non-overlapping CU
ranges to an unimplemented device-plugin step (docs/develop/amd-vgpu.md:74-90).
Here the scheduler owns a per-GPU CU bitmap (rebuilt from pod annotations, so
it survives restarts) and picks the concrete CUs at Fit time.

Measured on MI355X (``python -m k8s_vgpu_scheduler_amd.shim.probe --hwid``,
profiles/cu_mask_placement.md):
  * mask index i lives on XCD ``i % 8`` ("interleaved" layout): indices
    0..7 are CU 0 of XCD 0..7, 8..15 the next CU of each XCD, ...;
  * an XCD left with NO enabled CU is silently run with ALL its CUs
    (mask ``0,8,16,24`` -> 228 active CUs), because every dispatch is dealt
    round-robin to all 8 XCDs.
So a partition must be XCD-*balanced*: the unit is a granule of one CU on
each XCD (8 CUs, mask indices ``[8k, 8k+8)``), requests round up to whole
granules, and a tenant's granules are chosen contiguous (best fit) so its
CUs stay adjacent within each XCD's shader engines.  Per-XCD L2 isolation
between tenants is not available through CU masking (it needs CPX partition
mode, i.e. one HIP device per XCD), which is why the planner never promises it.
"""

from __future__ import annotations

import functools
from dataclasses import dataclass


@dataclass(frozen=True)
class CUTopology:
    total: int = 256
    xcds: int = 8
    layout: str = "interleaved"   # "interleaved" (measured on MI355X) | "blocked"

    @property
    def per_xcd(self) -> int:
        return max(1, self.total // max(1, self.xcds))

    @property
    def granules(self) -> int:
        return self.per_xcd

    def granule_cus(self, k: int) -> list[int]:
        """CU mask indices of granule k (one CU on every XCD)."""
        if self.layout == "blocked":
            return [x * self.per_xcd + k for x in range(self.xcds)]
        return list(range(k * self.xcds, (k + 1) * self.xcds))

    def xcd_of(self, cu: int) -> int:
        return cu // self.per_xcd if self.layout == "blocked" else cu % self.xcds


def bitmap_from_ranges(ranges) -> int:
    m = 0
    for a, b in ranges:
        m |= ((1 << (b - a + 1)) - 1) << a
    return m


def ranges_from_cus(cus) -> list[tuple[int, int]]:
    out: list[list[int]] = []
    for c in sorted(set(cus)):
        if out and c == out[-1][1] + 1:
            out[-1][1] = c
        else:
            out.append([c, c])
    return [(a, b) for a, b in out]


def round_up_cus(n: int, topo: CUTopology) -> int:
    """CU count actually granted for a request of n (whole granules)."""
    if n <= 0:
        return 0
    g = -(-n // topo.xcds)
    return min(topo.total, g * topo.xcds)


def free_cus(used_bitmap: int, topo: CUTopology) -> int:
    return topo.total - bin(used_bitmap & ((1 << topo.total) - 1)).count("1")


@functools.lru_cache(maxsize=64)
def _granule_masks(topo: CUTopology) -> tuple[int, ...]:
    return tuple(sum(1 << c for c in topo.granule_cus(k)) for k in range(topo.granules))


def _granule_free(used_bitmap: int, topo: CUTopology, k: int) -> bool:
    return not used_bitmap & _granule_masks(topo)[k]


def pick(used_bitmap: int, n: int, topo: CUTopology) -> list[tuple[int, int]] | None:
    """Choose ceil(n / xcds) free granules, contiguous if possible (best-fit
    run), else the lowest free ones.  None if not enough granules are free."""
    if n <= 0:
        return []
    need = -(-n // topo.xcds)
    if need > topo.granules:
        return None
    free = [k for k, m in enumerate(_granule_masks(topo)) if not used_bitmap & m]
    if len(free) < need:
        return None
    # runs of consecutive free granules
    runs: list[list[int]] = []
    for k in free:
        if runs and k == runs[-1][-1] + 1:
            runs[-1].append(k)
        else:
            runs.append([k])
    fitting = [r for r in runs if len(r) >= need]
    if fitting:
        r = min(fitting, key=lambda r: (len(r), r[0]))   # best fit keeps big runs whole
        chosen = r[:need]
    else:
        chosen = free[:need]
    cus = [c for k in chosen for c in topo.granule_cus(k)]
    return ranges_from_cus(cus)


# ------------------------------------------------------------ shared ranges --
# Hybrid layout for small slices.  Measured on MI355X: 8
# decode tenants on disjoint 32-CU masks ran 4 % below the same 8 processes
# unmasked (8551 vs 8921 tok/s) -- a tenant's latency-bound phases leave its
# CUs idle where unmasked neighbours would fill them -- while 4 tenants on
# 64-CU quarters ran 4.7 % ABOVE native.  So a request below one quarter of
# the GPU does not get a range of its own: it shares a quarter-sized range
# with other small requests (their CU counts summing to at most the range),
# and the temporal governor splits the range among them (the grant's core
# limit is the request's share of the GPU, below the mask's width, so the
# shim time-slices it: mivgpu_shim.cpp gate_wanted).  The quarters still
# isolate the pairs from each other spatially.  Round 5 makes the unit the
# whole GPU by default (AMDConfig.cu_share_unit = WHOLE_GPU): 8 pooled slices ran at
# native (8889 vs 8887 tok/s, fairness 0.996) against 8502 on disjoint ranges;
# device.py falls back to a disjoint range where no pool range is free.


WHOLE_GPU = -1     # cuShareUnit: the whole device, whatever its CU count


def share_unit(topo: CUTopology, cus: int = 0) -> int:
    """CUs of one shared range: ``cus`` rounded down to whole granules (at
    least one, at most the GPU), the whole GPU when negative (``WHOLE_GPU``)
    or at least the GPU's CU count, a quarter of the GPU when 0."""
    if cus < 0 or cus >= topo.total:
        return topo.total
    if cus > 0:
        return max(topo.xcds, min(topo.total, cus // topo.xcds * topo.xcds))
    return max(topo.xcds, topo.total // 4 // topo.xcds * topo.xcds)


def is_shared(ranges, usedcores: int) -> bool:
    """A container's range is shared when it is wider than its CU grant."""
    return bool(ranges) and sum(b - a + 1 for a, b in ranges) > usedcores > 0


def range_key(ranges) -> tuple:
    return tuple((int(a), int(b)) for a, b in ranges)


def charge(custominfo: dict, ranges, usedcores: int) -> None:
    """Charge a container's CU grant to its device's usage: the range's bits,
    and for a shared range its CUs against that range's load.  Values are
    replaced, never mutated in place (usage copies share them, types.py)."""
    custominfo["cu_used"] = custominfo.get("cu_used", 0) | bitmap_from_ranges(ranges)
    if is_shared(ranges, usedcores):
        load = dict(custominfo.get("cu_shared") or {})
        key = range_key(ranges)
        load[key] = load.get(key, 0) + usedcores
        custominfo["cu_shared"] = load


def merge_shared(a: dict | None, b: dict | None) -> dict:
    """Per-range maximum of two shared-load maps (init-container peaks)."""
    out = dict(a or {})
    for k, v in (b or {}).items():
        out[k] = max(out.get(k, 0), v)
    return out


def pick_shared(used_bitmap: int, shared_load: dict, n: int, topo: CUTopology,
                unit_cus: int = 0) -> list[tuple[int, int]] | None:
    """Range for a small request of ``n`` CUs (n < share_unit): the most loaded
    existing shared range it still fits in (best fit packs the ranges), else
    a new range of ``share_unit(topo, unit_cus)`` CUs from the free granules.
    ``shared_load``: ``{range_key: CUs granted on it}``."""
    unit = share_unit(topo, unit_cus)
    if not 0 < n < unit:
        return None
    fits = [(load, key) for key, load in shared_load.items()
            if load + n <= sum(b - a + 1 for a, b in key)]
    if fits:
        return [tuple(r) for r in max(fits)[1]]
    return pick(used_bitmap, unit, topo)


def per_xcd_counts(ranges, topo: CUTopology) -> list[int]:
    counts = [0] * topo.xcds
    for a, b in ranges:
        for c in range(a, b + 1):
            counts[topo.xcd_of(c)] += 1
    return counts


def is_balanced(ranges, topo: CUTopology) -> bool:
    c = per_xcd_counts(ranges, topo)
    return len(set(c)) == 1 and c[0] > 0
