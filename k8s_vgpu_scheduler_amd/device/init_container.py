"""Init-container-aware usage accounting (pkg/device/initContainer.go:36-157).

Init containers run sequentially before app containers, so a pod's effective
footprint on a device is ``max(peak over init containers, sum over app
containers)`` with slots ``max(1 if any init, #app occurrences)``; once every
init container has succeeded the usage shrinks to the app-only sum.
Design note: docs/develop/initContainer-design.md in the reference.
"""

from __future__ import annotations

from k8s_vgpu_scheduler_amd.k8s.client import init_containers

from .codec import merge_ranges
from .types import ContainerDevice


def _ranges_of(d) -> list:
    return list((d.custominfo or {}).get("cu_ranges") or [])


def _with_ranges(cd: ContainerDevice, ranges: list) -> ContainerDevice:
    if ranges:
        cd.custominfo = {"cu_ranges": merge_ranges(ranges)}
    return cd


def collapse_init_container_usage(pod: dict, raw: dict | None) -> dict | None:
    if raw is None:
        return None
    n_init = len(init_containers(pod))
    init_peak: dict = {}
    app_sum: dict = {}
    cu: dict = {}  # (type, uuid) -> union of CU ranges (init + app)
    for dev_type, single in raw.items():
        for cidx, ctr in enumerate(single):
            for d in ctr:
                key = (dev_type, d.uuid)
                cu.setdefault(key, []).extend(_ranges_of(d))
                if cidx < n_init:
                    m, c, s = init_peak.get(key, (0, 0, 0))
                    init_peak[key] = (max(m, d.usedmem), max(c, d.usedcores), 1)
                else:
                    m, c, s = app_sum.get(key, (0, 0, 0))
                    app_sum[key] = (m + d.usedmem, c + d.usedcores, s + 1)
    out = {}
    for dev_type in raw:
        uuids = sorted({u for (t, u) in list(init_peak) + list(app_sum) if t == dev_type})
        devs = []
        for u in uuids:
            im, ic, is_ = init_peak.get((dev_type, u), (0, 0, 0))
            am, ac, as_ = app_sum.get((dev_type, u), (0, 0, 0))
            devs.append(_with_ranges(ContainerDevice(uuid=u, type=dev_type, usedmem=max(im, am),
                                                     usedcores=max(ic, ac), slots=max(is_, as_, 1)),
                                     cu.get((dev_type, u), [])))
        out[dev_type] = [devs]
    return out


def app_containers_only_device_usage(pod: dict, raw: dict | None) -> dict | None:
    if raw is None:
        return None
    n_init = len(init_containers(pod))
    out = {}
    for dev_type, single in raw.items():
        sums: dict = {}
        cu: dict = {}
        for cidx, ctr in enumerate(single):
            if cidx < n_init:
                continue
            for d in ctr:
                m, c, s = sums.get(d.uuid, (0, 0, 0))
                sums[d.uuid] = (m + d.usedmem, c + d.usedcores, s + 1)
                cu.setdefault(d.uuid, []).extend(_ranges_of(d))
        out[dev_type] = [[_with_ranges(ContainerDevice(uuid=u, type=dev_type, usedmem=m, usedcores=c, slots=s),
                                       cu.get(u, []))
                          for u, (m, c, s) in sorted(sums.items())]]
    return out
