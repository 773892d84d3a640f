"""Map shared-region process slots to host pids.

A slot records the pid the shim saw inside the container (``getpid()`` in the
container's pid namespace).  Two consumers need the host pid:

* the shim's runtime-VRAM accounting reads KFD's per-process total from
  ``/sys/class/kfd/kfd/proc/<host pid>/vram_<gpu_id>`` (KFD names the
  directory by the host pid), see ``csrc/shim/mivgpu_shim.cpp:refresh_context``;
* per-process metrics joined with amd-smi's process list (host pids).

The reference carries the same field (``hostpid`` of the v1 proc slot,
pkg/monitor/nvidia/v1/spec.go:26-50) and fills it host-side.  Here the monitor
(hostPID DaemonSet) scans ``/proc/<pid>/status`` once per feedback pass: a
host process belongs to the slot when the last entry of its ``NSpid`` line
(the pid in its innermost namespace) equals the slot's pid and its cgroup path
names the slot's pod UID (cgroupfs ``pod<uid>`` or systemd
``pod<uid with _>``).  A slot is only filled when exactly one process matches.
"""

from __future__ import annotations

import os
from pathlib import Path


def _ns_pid(status_text: str) -> int | None:
    for line in status_text.splitlines():
        if line.startswith("NSpid:"):
            parts = line.split()[1:]
            return int(parts[-1]) if parts else None
    return None


def scan(proc_root: str = "/proc") -> list[tuple[int, int, str]]:
    """(host pid, innermost-namespace pid, cgroup text) of every process that
    runs in a nested pid namespace (NSpid with more than one entry) or not."""
    out = []
    root = Path(proc_root)
    try:
        entries = os.listdir(root)
    except OSError:
        return out
    for name in entries:
        if not name.isdigit():
            continue
        try:
            status = (root / name / "status").read_text()
            cgroup = (root / name / "cgroup").read_text()
        except OSError:
            continue
        nsp = _ns_pid(status)
        if nsp is not None:
            out.append((int(name), nsp, cgroup))
    return out


def _uid_forms(pod_uid: str) -> tuple[str, str]:
    return pod_uid, pod_uid.replace("-", "_")


def fill_host_pids(containers, proc_root: str = "/proc", procs=None) -> int:
    """Write ``hostpid`` into every active slot that lacks one; returns how
    many slots were filled.  ``containers``: ContainerUsage-like objects with
    ``pod_uid`` and ``region``."""
    pending = []
    for c in containers:
        r = c.region.r
        for i in range(min(r.procnum, len(r.procs))):
            s = r.procs[i]
            if s.status == 1 and s.pid > 0 and s.hostpid == 0:
                pending.append((c, s, s.pid, s.start_ns))
    if not pending:
        return 0
    procs = scan(proc_root) if procs is None else procs
    filled = 0
    for c, s, pid, start in pending:
        forms = _uid_forms(c.pod_uid)
        hits = [hp for hp, nsp, cg in procs if nsp == pid and any(f"pod{f}" in cg for f in forms)]
        # the slot may have been freed and reused by another process during the
        # /proc scan: write only if it still holds the process that was matched
        # (same pid and start time, still active, still unmapped)
        if len(hits) == 1 and s.status == 1 and s.pid == pid and s.start_ns == start and s.hostpid == 0:
            s.hostpid = hits[0]
            filled += 1
    return filled
