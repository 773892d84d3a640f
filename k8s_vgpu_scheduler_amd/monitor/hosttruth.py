"""Host-truth HBM accounting for the shared regions (VERDICT r2 weak #3a).

The shared region sits in a directory the container mounts read-write.  The
shim's O(1) quota counter (``dev_used``) and the per-process slot totals live
there, so a tenant that zeroes them -- or raises ``mem_limit`` -- allocates
past its grant: the shim's verdict is only as good as the counter.
``reconcile_limits`` (feedback.py) already restores the limits from the
read-only grant file; this pass restores the USAGE from host truth.

Every monitor pass (the reference's 5 s feedback period,
cmd/vGPUmonitor/feedback.go:136-165) recomputes each container's VRAM from
what the kernel driver itself counts: KFD's ``vram_<gpu_id>`` of every host
process of the container's pod (the cgroup names the pod UID -- the same
``/proc`` scan that maps slot pids to host pids, hostpid.py), which a tenant
cannot write.  Then, per container and device:

  * ``dev_used`` is raised to the truth (never below it); slot totals whose
    host pid is known are raised to that process's KFD total (the excess is
    runtime memory, charged as context), so the metrics stay honest;
  * a container whose truth exceeds its GRANT (the grant file, not the
    region) by more than ``slack`` is blocked -- ``recent_kernel = -1``, the
    shim parks its launches -- gets a ``VGPUMemoryOverGrant`` Warning event
    and ``mivgpu_container_memory_over_grant 1``, until it is back under;
    the raised ``dev_used`` makes its next allocation fail in the shim.

Multi-container pods: a device used by one container of the pod gets the
pod's total; otherwise each container is charged the KFD totals of its own
slots' (validated) host pids, and VRAM held by pod processes outside every
slot is charged to the pod as a whole: over the sum of the grants, every
container of the pod on that device is blocked.
"""

from __future__ import annotations

import logging
import threading
from pathlib import Path
from typing import Callable

from .hostpid import scan as scan_procs
from .occupancy import KFD_ROOT

log = logging.getLogger(__name__)

OVER_GRANT_REASON = "VGPUMemoryOverGrant"


def _uid_forms(pod_uid: str) -> tuple[str, str]:
    return pod_uid, pod_uid.replace("-", "_")


class HostTruth:
    """``gpu_ids``: callable returning ``{device uuid: KFD gpu_id}``.
    ``pod_pids``: optional callable ``pod_uid -> [host pids]`` (default: a
    ``/proc`` cgroup scan per pass).  ``events``: an EventRecorder-like object
    (``event(obj, type, reason, message)``) or None."""

    def __init__(self, gpu_ids: Callable[[], dict], kfd_root: Path | str = KFD_ROOT, proc_root: str = "/proc",
                 pod_pids: Callable[[str], list] | None = None, events=None, slack_bytes: int = 64 << 20):
        self.gpu_ids = gpu_ids
        self.kfd_root = Path(kfd_root)
        self.proc_root = proc_root
        self._pod_pids = pod_pids
        self.events = events
        self.slack = slack_bytes
        self._mu = threading.Lock()
        self.truth: dict[tuple, int] = {}      # (pod_uid, container, dev index) -> bytes
        self.over: set[tuple] = set()          # (pod_uid, container) currently over their grant
        self.corrections = 0

    # ------------------------------------------------------------ sources
    def vram(self, host_pid: int, gpu_id: int) -> int:
        try:
            return int((self.kfd_root / "proc" / str(host_pid) / f"vram_{gpu_id}").read_text().strip() or 0)
        except (OSError, ValueError):
            return 0

    def _pids_by_pod(self, uids: set) -> dict[str, list[int]]:
        if self._pod_pids is not None:
            return {u: list(self._pod_pids(u) or []) for u in uids}
        procs = scan_procs(self.proc_root)
        out: dict[str, list[int]] = {u: [] for u in uids}
        for hp, _nsp, cg in procs:
            for u in uids:
                if any(f"pod{f}" in cg for f in _uid_forms(u)):
                    out[u].append(hp)
                    break
        return out

    # ------------------------------------------------------------- a pass
    def enforce(self, lister, grants: dict | None = None) -> dict:
        """One pass over every container of ``lister``.  ``grants``: optional
        ``{(pod_uid, container): [limit bytes per device]}`` (the grant
        files); absent -> the region's mem_limit.  Returns the truth map."""
        containers = lister.list_containers()
        if not containers:
            with self._mu:
                self.truth, self.over = {}, set()
            return {}
        ids = self.gpu_ids() or {}
        pods = self._pids_by_pod({c.pod_uid for c in containers})
        # (pod, uuid) -> [(container, device index)]
        users: dict[tuple, list] = {}
        for c in containers:
            r = c.region
            for i in range(r.device_num()):
                if r.is_valid_uuid(i) and r.uuid(i) in ids:
                    users.setdefault((c.pod_uid, r.uuid(i)), []).append((c, i))
        truth: dict[tuple, int] = {}
        over: set[tuple] = set()
        for (uid, dev_uuid), lst in users.items():
            gid = ids[dev_uuid]
            pids = set(pods.get(uid, []))
            per_pid = {hp: self.vram(hp, gid) for hp in pids}
            pod_total = sum(per_pid.values())
            attributed = 0
            charged = []
            for c, i in lst:
                if len(lst) == 1:
                    t = pod_total
                else:
                    t = sum(per_pid.get(p.hostpid, 0) for p in c.region.active_procs() if p.hostpid in pids)
                attributed += t
                charged.append((c, i, t))
            grant_sum = 0
            for c, i, t in charged:
                key = (c.pod_uid, c.container)
                g = self._grant(c, i, grants)
                grant_sum += g
                truth[(c.pod_uid, c.container, i)] = t
                self._correct(c, i, t, per_pid if len(lst) == 1 else
                              {p: v for p, v in per_pid.items()
                               if p in {s.hostpid for s in c.region.active_procs()}})
                if g and t > g + self.slack:
                    over.add(key)
                    self._report(c, i, t, g)
            # pod processes outside every slot (a hidden tenant process)
            if len(lst) > 1 and grant_sum and pod_total - attributed > self.slack and pod_total > grant_sum + self.slack:
                for c, i, _ in charged:
                    over.add((c.pod_uid, c.container))
                    self._report(c, i, pod_total, grant_sum)
        with self._mu:
            newly_clear = self.over - over
            self.truth, self.over = truth, over
        for c in containers:
            key = (c.pod_uid, c.container)
            if key in over:
                c.region.set_recent_kernel(-1)
            elif key in newly_clear:
                log.info("%s/%s: back under its grant; unblocked", c.pod_uid, c.container)
                if c.region.recent_kernel() < 0:
                    c.region.set_recent_kernel(0)
        return truth

    def _grant(self, c, i: int, grants: dict | None) -> int:
        if grants is not None:
            g = grants.get((c.pod_uid, c.container))
            if g is not None and i < len(g):
                return int(g[i])
        return int(c.region.r.mem_limit[i])

    def _correct(self, c, i: int, t: int, per_pid: dict):
        r = c.region.r
        if int(r.dev_used[i]) < t:
            log.warning("%s/%s dev %d: region counts %d B in use, KFD %d B; corrected", c.pod_uid, c.container, i,
                        int(r.dev_used[i]), t)
            r.dev_used[i] = t
            self.corrections += 1
        for s in c.region.active_procs():
            v = per_pid.get(s.hostpid) if s.hostpid > 0 else None
            if v is None:
                continue
            m = s.used[i]
            if int(m.total) < v:
                m.context = int(m.context) + (v - int(m.total))
                m.total = v
                self.corrections += 1

    def _report(self, c, i: int, t: int, g: int):
        key = (c.pod_uid, c.container)
        with self._mu:
            was = key in self.over
        msg = (f"container {c.container} holds {t >> 20} MiB of HBM on device {i} (KFD), over its grant of "
               f"{g >> 20} MiB: launches blocked until it is back under")
        if not was:
            log.warning("%s/%s: %s", c.pod_uid, c.container, msg)
            if self.events is not None:
                self.events.event({"kind": "Pod", "metadata": {"name": c.pod_name or c.pod_uid,
                                                               "namespace": c.namespace or "default",
                                                               "uid": c.pod_uid}},
                                  "Warning", OVER_GRANT_REASON, msg)

    def snapshot(self) -> tuple[dict, set]:
        with self._mu:
            return dict(self.truth), set(self.over)


def grants_from_files(lister) -> dict:
    """``{(pod_uid, container): [limit bytes per device]}`` from the grant
    files next to the containers directory (deviceplugin/allocate.py)."""
    from k8s_vgpu_scheduler_amd.deviceplugin.allocate import parse_grant

    from .feedback import expected_region

    out = {}
    limits_dir = lister.base.parent / "limits"
    for c in lister.list_containers():
        try:
            grant = parse_grant((limits_dir / f"{c.pod_uid}_{c.container}.conf").read_text())
        except OSError:
            continue
        out[(c.pod_uid, c.container)] = expected_region(grant)["mem_limit"]
    return out


def kfd_gpu_ids(backend, kfd_root: Path | str = KFD_ROOT) -> Callable[[], dict]:
    """``{uuid: gpu_id}`` of the node's GPUs (by PCI location, like the
    occupancy sampler), refreshed when a uuid is missing."""
    from .occupancy import gpu_ids_by_bdf

    cache: dict = {}

    def get() -> dict:
        if not cache and backend is not None:
            by_bdf = gpu_ids_by_bdf(Path(kfd_root))
            for g in backend.gpus():
                if g.bdf in by_bdf:
                    cache[g.uuid] = by_bdf[g.bdf]
        return cache
    return get


def single_gpu_ids(uuid: str, kfd_root: Path | str = KFD_ROOT) -> dict:
    """Test helper for a one-GPU box: ``{uuid: the only GPU's gpu_id}``."""
    nodes = Path(kfd_root) / "topology" / "nodes"
    for n in sorted(nodes.iterdir(), key=lambda p: int(p.name) if p.name.isdigit() else -1):
        try:
            gid = int((n / "gpu_id").read_text().strip() or 0)
        except (OSError, ValueError):
            continue
        if gid:
            return {uuid: gid}
    return {}


__all__ = ["HostTruth", "grants_from_files", "kfd_gpu_ids", "single_gpu_ids", "OVER_GRANT_REASON"]
