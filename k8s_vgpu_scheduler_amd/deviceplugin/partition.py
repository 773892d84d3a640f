"""Compute-partition manager: the MI355X counterpart of the reference's MIG
instance manager and MIG apply lock.

Reference: plugin/migmgr.go:65-556 (reconcile GPU instances every 5 s, adopt
on restart, only touch idle GPUs), plugin/lock.go:28-136 + util.go:237-279
(`/tmp/hami/hami-mig-apply.lock` pauses every NVML user while a
reconfiguration runs).

MI355X has no per-instance carving: a physical GPU is in one compute-partition
mode at a time: SPX (1 x 8 XCDs), DPX (2 x 4), QPX (4 x 2), CPX (8 x 1).
Partitions surface as separate ROCm devices, and the registrar publishes them
with ``mode`` = dpx/qpx/cpx (pods pick them with ``amd.com/vgpu-mode``).  So the
manager reconciles a *desired mode per physical GPU* against the current one:

  desired   node annotation ``mivgpu.io/partition-request`` = ``"0=CPX,3=DPX"``
            (set by an operator or a higher-level controller), or the node's
            ``partitions`` entry in the device-plugin node config;
  busy      a GPU is only reconfigured when none of its logical devices has a
            process (smi) or a non-terminated pod allocated on this node;
  apply     under the apply lock file (registration and health checks pause
            while it exists), via the smi backend (amd-smi / sysfs), then the
            device plugin re-registers and restarts its kubelet endpoint;
  status    ``mivgpu.io/partition-status`` = ``"0=CPX,1=SPX,3=SPX>DPX:busy"``.
"""

from __future__ import annotations

import contextlib
import logging
import os
import threading
import time
from pathlib import Path

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device.amd.device import SUPPORT_ANNOS
from k8s_vgpu_scheduler_amd.smi import PARTITION_MODES, Backend, PartitionError
from k8s_vgpu_scheduler_amd.utils import util

log = logging.getLogger("mivgpu.partition")

REQUEST_ANNOS = "mivgpu.io/partition-request"
STATUS_ANNOS = "mivgpu.io/partition-status"
APPLY_LOCK = os.environ.get("MIVGPU_PARTITION_LOCK", "/tmp/mivgpu/partition-apply.lock")
_TERMINAL = ("Succeeded", "Failed")


def parse_request(value: str) -> dict[int, str]:
    out = {}
    for part in (value or "").replace(";", ",").split(","):
        part = part.strip()
        if not part:
            continue
        idx, _, mode = part.partition("=")
        mode = mode.strip().upper()
        if mode not in PARTITION_MODES:
            raise ValueError(f"unknown compute partition {mode!r} in {value!r}")
        out[int(idx)] = mode
    return out


def is_applying(lock_path: str = APPLY_LOCK) -> bool:
    return Path(lock_path).exists()


@contextlib.contextmanager
def apply_lock(lock_path: str = APPLY_LOCK):
    p = Path(lock_path)
    p.parent.mkdir(parents=True, exist_ok=True)
    fd = os.open(p, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o644)   # fails if another apply runs
    try:
        os.write(fd, str(os.getpid()).encode())
        os.close(fd)
        yield p
    finally:
        with contextlib.suppress(FileNotFoundError):
            p.unlink()


class PartitionManager:
    def __init__(self, backend: Backend, node: str, lock_path: str = APPLY_LOCK, static: dict | None = None):
        self.backend, self.node, self.lock_path = backend, node, lock_path
        self.static = dict(static or {})
        self._stop = threading.Event()

    # ------------------------------------------------------------- inputs
    def desired(self) -> dict[int, str]:
        want = dict(self.static)
        node = util.get_node(self.node)
        ann = ((node.get("metadata") or {}).get("annotations") or {}).get(REQUEST_ANNOS, "")
        try:
            want.update(parse_request(ann))
        except ValueError as e:
            log.error("ignoring %s: %s", REQUEST_ANNOS, e)
        return want

    def current(self) -> dict[int, str]:
        return {g.physical: g.compute_partition.upper() or "SPX" for g in self.backend.gpus()}

    def _allocated_uuids(self) -> set[str]:
        from k8s_vgpu_scheduler_amd.k8s.client import get_client

        used = set()
        for p in get_client().list_pods(field_selector={"spec.nodeName": self.node}):
            if ((p.get("status") or {}).get("phase")) in _TERMINAL:
                continue
            ann = ((p.get("metadata") or {}).get("annotations") or {}).get(SUPPORT_ANNOS)
            if not ann:
                continue
            try:
                for ctr in codec.decode_pod_devices({"AMD": SUPPORT_ANNOS}, {SUPPORT_ANNOS: ann}).get("AMD", []):
                    used.update(d.uuid for d in ctr)
            except codec.CodecError:
                continue
        return used

    def busy(self, physical: int, allocated: set[str] | None = None) -> str | None:
        allocated = self._allocated_uuids() if allocated is None else allocated
        for g in self.backend.gpus():
            if g.physical != physical:
                continue
            if self.backend.processes(g):
                return "processes"
            if g.uuid in allocated:
                return "pods"
        return None

    # ---------------------------------------------------------- reconcile
    def reconcile(self) -> bool:
        """Apply every pending mode change whose GPU is idle; returns True if
        anything changed (the caller re-registers and restarts the plugin)."""
        want, cur = self.desired(), self.current()
        allocated = self._allocated_uuids()
        status, changed = {}, False
        for phys in sorted(cur):
            target = want.get(phys, cur[phys])
            if target == cur[phys]:
                status[phys] = cur[phys]
                continue
            why = self.busy(phys, allocated)
            if why:
                status[phys] = f"{cur[phys]}>{target}:busy"
                continue
            try:
                with apply_lock(self.lock_path):
                    log.info("GPU %d: compute partition %s -> %s", phys, cur[phys], target)
                    self.backend.set_compute_partition(phys, target)
                status[phys] = target
                changed = True
            except FileExistsError:
                status[phys] = f"{cur[phys]}>{target}:locked"
            except PartitionError as e:
                log.error("GPU %d: %s", phys, e)
                status[phys] = f"{cur[phys]}>{target}:error"
        value = ",".join(f"{k}={v}" for k, v in sorted(status.items()))
        try:
            util.patch_node_annotations(self.node, {STATUS_ANNOS: value})
        except Exception as e:  # noqa: BLE001
            log.warning("could not publish %s: %s", STATUS_ANNOS, e)
        return changed

    def watch(self, on_change, interval: float = 5.0):
        while not self._stop.is_set():
            try:
                if self.reconcile():
                    on_change()
            except Exception as e:  # noqa: BLE001
                log.error("partition reconcile failed: %s", e)
            self._stop.wait(interval)

    def stop(self):
        self._stop.set()


def wait_until_applied(lock_path: str = APPLY_LOCK, timeout: float = 120.0, poll: float = 0.5) -> bool:
    """Block while a reconfiguration holds the apply lock (health/registration users)."""
    deadline = time.time() + timeout
    while is_applying(lock_path):
        if time.time() > deadline:
            return False
        time.sleep(poll)
    return True
