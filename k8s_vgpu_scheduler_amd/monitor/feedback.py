"""Priority feedback loop over the shared regions (cmd/vGPUmonitor/feedback.go:40-165).

Every 5 s: decay each container's ``recent_kernel`` activity counter (the shim
sets it to 2 while it launches); count, per GPU uuid and priority level, how
many containers launched recently.  Then per container:
  * blocking  -- a HIGHER-priority (numerically lower) task is active on one of
    its GPUs -> ``recent_kernel = -1`` (the shim parks launches), else 0;
  * util switch -- a higher-priority task, or another task of the SAME priority,
    is active -> ``utilization_switch = 1`` (enforce the core limit with the
    governor even when a CU mask exists), else 0.

Both verdicts go into the shared region (the reference's channel) AND into the
container's host-owned, read-only control file (control.py), which is what the
shim obeys when it has one: a tenant rewriting its region cannot clear them.
"""

from __future__ import annotations

import logging
import os
import re
import threading

from .control import DEFAULT_LEASE_S
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


def observe(lister: ContainerLister, over: set | None = None, decisions: dict | None = None):
    """``over``: (pod_uid, container) keys the host-truth pass found over
    their HBM grant (hosttruth.py): they stay blocked whatever the
    priorities say.  ``decisions``: filled with ``{(pod_uid, container):
    (block, switch)}`` for the control files."""
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
        block = bool(over and (c.pod_uid, c.container) in over) or check_blocking(ut, p, c)
        switch = check_priority(ut, p, c)
        if block:
            if rk >= 0:
                c.region.set_recent_kernel(-1)
        elif rk < 0:
            c.region.set_recent_kernel(0)
        if switch:
            if sw != 1:
                c.region.set_utilization_switch(1)
        elif sw != 0:
            c.region.set_utilization_switch(0)
        if decisions is not None:
            decisions[(c.pod_uid, c.container)] = (block, switch)
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


def core_limit_ppm(s: str | None) -> int:
    """A grant's core limit in percent with up to four decimals ("25", "12.5")
    -> parts per million of the device; 0 when absent or outside (0, 100].
    Integer arithmetic, the shim's parse_pct_ppm digit for digit."""
    m = re.fullmatch(r"([0-9]{0,3})(?:\.([0-9]*))?", s or "")
    if not m or not (m.group(1) or m.group(2)):
        return 0
    ppm = int(m.group(1) or "0") * 10000 + int((m.group(2) or "")[:4].ljust(4, "0"))
    return ppm if 0 < ppm <= 1_000_000 else 0


def pct_of_ppm(ppm: int) -> int:
    """The region's whole-percent core limit of a ppm share (half up, >= 1)."""
    return 0 if ppm == 0 else max(1, (ppm + 5000) // 10000)


def expected_region(grant: dict) -> dict:
    """Region fields a grant file (deviceplugin/allocate.py) implies."""
    allmem = parse_size(grant.get("HIP_DEVICE_MEMORY_LIMIT"))
    core = pct_of_ppm(core_limit_ppm(grant.get("HIP_DEVICE_CORE_LIMIT")) or 1000000)
    pol = {"force": 1, "disable": 2}.get(grant.get("GPU_CORE_UTILIZATION_POLICY", "").lower(), 0)
    try:
        prio = int(grant.get("HIP_TASK_PRIORITY", "1"))
    except ValueError:
        prio = 1
    cores = []
    for i in range(MAX_DEVICES):
        ci = core_limit_ppm(grant.get(f"HIP_DEVICE_CORE_LIMIT_{i}"))
        cores.append(pct_of_ppm(ci) if ci else core)
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


def publish_controls(lister: ContainerLister, grants: dict, decisions: dict, verdicts: dict,
                     lease_s: float = DEFAULT_LEASE_S) -> int:
    """Write every granted container's verdicts into its host-owned control
    file (monitor/control.py) and renew the lease.  Returns files written."""
    n = 0
    for key, g in grants.items():
        cf = lister.controls.get(key)
        if cf is None:
            continue
        v = verdicts.get((g.pod_uid, g.container))
        over = bool(v is not None and v.over)
        block, switch = decisions.get((g.pod_uid, g.container), (over, False))
        cf.publish(block=block or over, switch=switch, over=over,
                   excess=v.excess if v is not None else None, lease_s=lease_s)
        n += 1
    lister.controls.retain(set(grants))
    return n


def feedback_pass(lister: ContainerLister, truth=None, escalation=None, lease_s: float = DEFAULT_LEASE_S,
                  board_dir: str | None = None) -> dict:
    """One pass: map host pids, restore the region mirrors of the limits from
    the grants, enforce HBM from host truth (hosttruth.HostTruth, optional:
    over grant, shim not loaded, excess), the priority feedback, the
    verdicts into the read-only control files, then the over-grant
    escalation (escalate.OverGrantPolicy, optional).  With host truth and a
    share-board directory, each GPU's node-written core limits (board.py
    write_limits: the grant's limit of every process host truth attributes)."""
    from .hosttruth import load_grants

    lister.update()
    fill_host_pids(lister.list_containers())
    fixed = reconcile_limits(lister)
    grants = load_grants(lister.base.parent / "limits")
    verdicts: dict = {}
    if truth is not None:
        verdicts = truth.enforce(lister, grants, lister.pod)
        if board_dir and os.path.isdir(board_dir):
            from .board import write_limits, write_owners
            for gid, w in getattr(truth, "weights", {}).items():
                try:
                    write_limits(board_dir, gid, w)
                    write_owners(board_dir, gid, getattr(truth, "owners", {}).get(gid, {}))
                except OSError as e:
                    log.warning("share board limits for gpu %d: %s", gid, e)
    over = {k for k, v in verdicts.items() if v.over}
    decisions: dict = {}
    ut = observe(lister, over, decisions)
    published = publish_controls(lister, grants, decisions, verdicts, lease_s)
    taken = escalation.step(verdicts, lister.pod) if escalation is not None else []
    return {"limits_fixed": fixed, "over": over, "util": ut, "controls": published, "actions": taken,
            "no_shim": {k for k, v in verdicts.items() if not v.shim_loaded}}


def watch_and_feedback(lister: ContainerLister, stop: threading.Event, period: float = 5.0,
                       pause: threading.Event | None = None, truth=None, escalation=None,
                       board_dir: str | None = None, state_file: str | None = None, board=None):
    """The 5 s loop; skipped while ``pause`` is set (a compute-partition apply
    is in progress, cmd/vGPUmonitor/main.go:79-109).  The control-file lease
    covers four periods, so a paused or dead monitor releases its verdicts.
    ``state_file``: each pass's host-truth state as JSON (``write_state``)."""
    n = 0
    while not stop.wait(period):
        if pause is not None and pause.is_set():
            continue
        n += 1
        res = None
        if board is not None:
            board.ensure()      # the node's share-board sampler (monitor/board.py), restarted if it died
        try:
            res = feedback_pass(lister, truth, escalation, lease_s=max(DEFAULT_LEASE_S, 4 * period),
                                board_dir=board_dir)
        except Exception:  # noqa: BLE001
            log.exception("feedback iteration failed")
        if state_file:
            write_state(state_file, n, res, truth, escalation)


def write_state(path: str, n: int, res: dict | None, truth=None, escalation=None):
    """Atomically replace ``path`` with this pass's state as JSON (the
    monitor's ``--state-file``: what host truth saw and decided, readable
    by an operator or a failed e2e test)."""
    import json
    import time as _t

    st = {"pass": n, "time": _t.time(), "ok": res is not None}
    if res is not None:
        st["no_shim"] = sorted("/".join(k) for k in res.get("no_shim", ()))
        st["over"] = sorted("/".join(k) for k in res.get("over", ()))
        st["actions"] = [[str(x) for x in a] for a in res.get("actions", ())]
    if truth is not None and hasattr(truth, "debug_state"):
        st["host_truth"] = truth.debug_state()
    if escalation is not None:
        st["escalation"] = {"shimless": {"/".join(k): v for k, v in escalation.shimless.items()},
                            "over": {"/".join(k): v for k, v in escalation.count.items()},
                            "evicted": sorted(escalation.evicted), "actions": dict(escalation.actions)}
    tmp = f"{path}.{os.getpid()}.tmp"
    try:
        with open(tmp, "w") as f:
            json.dump(st, f, default=str)
        os.replace(tmp, path)
    except OSError as e:
        log.debug("state file %s: %s", path, e)
