"""XCD-aware CU-range allocator for ``HSA_CU_MASK`` partitions on MI355X.

The reference only converts ``amd.com/gpucores`` % into a CU *count*
(pkg/device/amd/device.go:333-344) and leaves choosing non-overlapping CU
ranges to an unimplemented device-plugin step (docs/develop/amd-vgpu.md:74-90).
Here the scheduler owns a per-GPU CU bitmap (rebuilt from pod annotations, so
it survives restarts) and picks the concrete CUs at Fit time, XCD-first:

  * MI355X = 8 XCDs x 32 CUs; each XCD has its own 4 MiB L2, so a tenant
    confined to whole XCDs does not share L2 with its neighbours
    (MI355X_MICROARCH.md, XCD row);
  * a request of >= 32 CUs takes whole free XCDs first, the remainder by
    best-fit in the least-free XCD that can hold it (keeps other XCDs whole);
  * a request < 32 CUs is best-fit into one XCD (never split across L2s unless
    no single XCD has room).

``layout`` says how ``HSA_CU_MASK`` logical CU indices map to XCDs:
"blocked" (index // cus_per_xcd) or "interleaved" (index % n_xcd); it is
measured on hardware by ``shim.probe --hwid`` and set in the device config.
"""

from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class CUTopology:
    total: int = 256
    xcds: int = 8
    layout: str = "interleaved"   # "interleaved" | "blocked"

    @property
    def per_xcd(self) -> int:
        return max(1, self.total // max(1, self.xcds))

    def xcd_cus(self, x: int) -> list[int]:
        if self.layout == "blocked":
            return list(range(x * self.per_xcd, (x + 1) * self.per_xcd))
        return list(range(x, self.total, self.xcds))

    def groups(self) -> list[list[int]]:
        return [self.xcd_cus(x) for x in range(self.xcds)]


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


def free_cus(used_bitmap: int, topo: CUTopology) -> int:
    return topo.total - bin(used_bitmap & ((1 << topo.total) - 1)).count("1")


def pick(used_bitmap: int, n: int, topo: CUTopology) -> list[tuple[int, int]] | None:
    """Choose n free CUs (XCD-first); None if fewer than n are free."""
    if n <= 0:
        return []
    if n > topo.total:
        return None
    free_by_xcd = []
    for x, cus in enumerate(topo.groups()):
        free_by_xcd.append((x, [c for c in cus if not (used_bitmap >> c) & 1]))
    if sum(len(f) for _, f in free_by_xcd) < n:
        return None
    chosen: list[int] = []
    need = n
    per = topo.per_xcd
    # 1) whole free XCDs
    if need >= per:
        for x, f in free_by_xcd:
            if need < per:
                break
            if len(f) == per:
                chosen.extend(f)
                need -= per
        taken = {x for x, f in free_by_xcd if f and set(f) <= set(chosen)}
    else:
        taken = set()
    # 2) remainder: best fit into a single partially free XCD (least free that fits)
    if need > 0:
        cands = [(len(f), x, f) for x, f in free_by_xcd if x not in taken and len(f) >= need]
        partial = [c for c in cands if c[0] < per]
        pool = partial or cands
        if pool:
            _, x, f = min(pool)
            chosen.extend(f[:need])
            need = 0
    # 3) still short: spill across XCDs, fullest-first to minimise L2 sharing
    if need > 0:
        for _, x, f in sorted(((len(f), x, f) for x, f in free_by_xcd if x not in taken), reverse=True):
            rest = [c for c in f if c not in chosen]
            take = rest[:need]
            chosen.extend(take)
            need -= len(take)
            if need == 0:
                break
    if need > 0:
        return None
    return ranges_from_cus(chosen)


def xcds_touched(ranges, topo: CUTopology) -> int:
    cus = set()
    for a, b in ranges:
        cus.update(range(a, b + 1))
    return sum(1 for g in topo.groups() if cus & set(g))
