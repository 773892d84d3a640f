"""Priority feedback loop over the shared regions (cmd/vGPUmonitor/feedback.go:40-165).

Every 5 s: decay each container's ``recent_kernel`` activity counter (the shim
sets it to 2 on every launch); count, per GPU uuid and priority level, how
many containers launched recently.  Then per container:
  * blocking  -- a HIGHER-priority (numerically lower) task is active on one of
    its GPUs -> ``recent_kernel = -1`` (the shim parks launches), else 0;
  * util switch -- a higher-priority task, or another task of the SAME priority,
    is active -> ``utilization_switch = 1`` (enforce the core limit with the
    governor even when a CU mask exists), else 0.
"""

from __future__ import annotations

import logging
import threading

from .hostpid import fill_host_pids
from .lister import ContainerLister

log = logging.getLogger(__name__)


def _uuids(c) -> list[str]:
    r = c.region
    return [r.uuid(i) for i in range(r.device_num()) if r.is_valid_uuid(i)]


def check_blocking(ut: dict, p: int, c) -> bool:
    for u in _uuids(c):
        lst = ut.get(u)
        if lst and any(lst[i] > 0 for i in range(min(p, len(lst)))):
            return True
    return False


def check_priority(ut: dict, p: int, c) -> bool:
    for u in _uuids(c):
        lst = ut.get(u)
        if not lst:
            continue
        if any(lst[i] > 0 for i in range(min(p, len(lst)))):
            return True
        if 0 <= p < len(lst) and lst[p] > 1:
            return True
    return False


def observe(lister: ContainerLister):
    ut: dict[str, list[int]] = {}
    cs = lister.list_containers()
    for c in cs:
        rk = c.region.recent_kernel()
        if rk > 0:
            rk -= 1
            if rk > 0:
                p = c.region.priority()
                if p >= 0:
                    for u in _uuids(c):
                        lst = ut.setdefault(u, [])
                        while p >= len(lst):
                            lst.append(0)
                        lst[p] += 1
            c.region.set_recent_kernel(rk)
    for c in cs:
        p = c.region.priority()
        rk = c.region.recent_kernel()
        sw = c.region.utilization_switch()
        if check_blocking(ut, p, c):
            if rk >= 0:
                c.region.set_recent_kernel(-1)
        elif rk < 0:
            c.region.set_recent_kernel(0)
        if check_priority(ut, p, c):
            if sw != 1:
                c.region.set_utilization_switch(1)
        elif sw != 0:
            c.region.set_utilization_switch(0)
    return ut


def watch_and_feedback(lister: ContainerLister, stop: threading.Event, period: float = 5.0,
                       pause: threading.Event | None = None):
    while not stop.wait(period):
        if pause is not None and pause.is_set():
            continue
        try:
            lister.update()
            fill_host_pids(lister.list_containers())
            observe(lister)
        except Exception:  # noqa: BLE001
            log.exception("feedback iteration failed")
