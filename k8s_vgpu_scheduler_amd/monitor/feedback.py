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
from .region import MAX_DEVICES

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


def observe(lister: ContainerLister, over: set | None = None):
    """``over``: (pod_uid, container) keys the host-truth pass found over
    their HBM grant (hosttruth.py): they stay blocked whatever the
    priorities say."""
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
        if over and (c.pod_uid, c.container) in over:
            if rk >= 0:
                c.region.set_recent_kernel(-1)
        elif check_blocking(ut, p, c):
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


_SIZE_MULT = {"k": 1 << 10, "m": 1 << 20, "g": 1 << 30, "t": 1 << 40}


def parse_size(v: str | None) -> int:
    """The shim's parse_size: ``4096m`` -> bytes (plain numbers are bytes)."""
    if not v:
        return 0
    v = v.strip()
    mult = _SIZE_MULT.get(v[-1:].lower(), 1)
    try:
        return int(float(v[:-1] if mult > 1 else v) * mult)
    except ValueError:
        return 0


def mask_count(mask: str | None, idx: int) -> int:
    """CUs granted to local device ``idx`` by an HSA_CU_MASK value."""
    for part in (mask or "").split(";"):
        dev, sep, ranges = part.partition(":")
        if not sep or dev.strip() != str(idx):
            continue
        n = 0
        for r in ranges.split(","):
            a, _, b = r.partition("-")
            try:
                n += int(b or a) - int(a) + 1
            except ValueError:
                return 0
        return n
    return 0


def expected_region(grant: dict) -> dict:
    """Region fields a grant file (deviceplugin/allocate.py) implies."""
    allmem = parse_size(grant.get("HIP_DEVICE_MEMORY_LIMIT"))
    try:
        core = int(grant.get("HIP_DEVICE_CORE_LIMIT", "100"))
    except ValueError:
        core = 100
    core = core if 1 <= core <= 100 else 100
    pol = {"force": 1, "disable": 2}.get(grant.get("GPU_CORE_UTILIZATION_POLICY", "").lower(), 0)
    try:
        prio = int(grant.get("HIP_TASK_PRIORITY", "1"))
    except ValueError:
        prio = 1
    cores = []
    for i in range(MAX_DEVICES):
        try:
            ci = int(grant.get(f"HIP_DEVICE_CORE_LIMIT_{i}", "0"))
        except ValueError:
            ci = 0
        cores.append(ci if 1 <= ci <= 100 else core)
    return {"mem_limit": [parse_size(grant.get(f"HIP_DEVICE_MEMORY_LIMIT_{i}")) or allmem
                          for i in range(MAX_DEVICES)],
            "cu_limit": cores, "cu_mask": [mask_count(grant.get("HSA_CU_MASK"), i) for i in range(MAX_DEVICES)],
            "core_policy": pol, "priority": prio}


def reconcile_limits(lister: ContainerLister) -> int:
    """Put every region's limits back to the container's grant.

    The region file sits in a directory the container mounts read-write, so a
    tenant can rewrite ``mem_limit``/``cu_limit``/``cu_mask_count``/policy in
    it; the grant file (written by Allocate on the host, mounted read-only)
    is the authority.  Returns the number of fields corrected."""
    from k8s_vgpu_scheduler_amd.deviceplugin.allocate import parse_grant
    fixed = 0
    limits_dir = lister.base.parent / "limits"
    for c in lister.list_containers():
        path = limits_dir / f"{c.pod_uid}_{c.container}.conf"
        try:
            grant = parse_grant(path.read_text())
        except OSError:
            continue
        want = expected_region(grant)
        r = c.region.r
        for i in range(c.region.device_num()):
            for field, val in (("mem_limit", want["mem_limit"][i]), ("cu_limit", want["cu_limit"][i]),
                               ("cu_mask_count", want["cu_mask"][i])):
                arr = getattr(r, field)
                if int(arr[i]) != val:
                    log.warning("%s/%s: region %s[%d]=%d differs from the grant %d; restored",
                                c.pod_uid, c.container, field, i, int(arr[i]), val)
                    arr[i] = val
                    fixed += 1
        for field in ("core_policy", "priority"):
            if int(getattr(r, field)) != want[field]:
                log.warning("%s/%s: region %s=%d differs from the grant %d; restored", c.pod_uid, c.container,
                            field, int(getattr(r, field)), want[field])
                setattr(r, field, want[field])
                fixed += 1
    return fixed


def feedback_pass(lister: ContainerLister, truth=None) -> dict:
    """One pass: map host pids, restore the limits from the grants, restore
    the usage from host truth (hosttruth.HostTruth, optional), then the
    priority feedback."""
    lister.update()
    fill_host_pids(lister.list_containers())
    fixed = reconcile_limits(lister)
    over = set()
    if truth is not None:
        from .hosttruth import grants_from_files
        truth.enforce(lister, grants_from_files(lister))
        over = truth.snapshot()[1]
    ut = observe(lister, over)
    return {"limits_fixed": fixed, "over": over, "util": ut}


def watch_and_feedback(lister: ContainerLister, stop: threading.Event, period: float = 5.0,
                       pause: threading.Event | None = None, truth=None):
    """The 5 s loop; skipped while ``pause`` is set (a compute-partition apply
    is in progress, cmd/vGPUmonitor/main.go:79-109)."""
    while not stop.wait(period):
        if pause is not None and pause.is_set():
            continue
        try:
            feedback_pass(lister, truth)
        except Exception:  # noqa: BLE001
            log.exception("feedback iteration failed")
