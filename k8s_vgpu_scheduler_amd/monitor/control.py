"""Host-owned control files: the monitor's verdicts, read-only to the tenant.

ctypes mirror of ``mivgpu_control_t`` (csrc/include/mivgpu/shared_region.h).
The shared region a container's shim writes sits in a directory the container
mounts read-write, so a verdict the monitor writes there -- the reference's
``recent_kernel = -1`` block and ``utilization_switch`` (feedback.go:74-134,
written into the same shared memory in HAMi-core) -- is one store away from
being cleared by the tenant.  Here:

* the device plugin's Allocate creates ``$HOOK_PATH/vgpu/control/<pod>_<ctr>.ctl``
  on the host and bind-mounts it READ-ONLY into the container; the grant names
  it (``MIVGPU_CONTROL_FILE``), so only the plugin can point the shim at it;
* the shim maps it ``PROT_READ`` and honours ``block`` (parks launches),
  ``utilization_switch`` and ``host_excess`` (KFD-measured VRAM beyond the
  region's own counter, added to the quota check);
* the monitor maps it on the host and writes it in place every pass (never a
  rename: the container's bind mount pins the inode), renewing a lease.  The
  verdicts hold only while the lease is live, so a dead monitor cannot leave a
  tenant parked.
"""

from __future__ import annotations

import ctypes as C
import mmap
import os
import stat
import threading
import time

from .region import MAX_DEVICES

CTL_MAGIC = 0x4D495643
CTL_VERSION = 1
CONTAINER_CONTROL_PATH = "/etc/mivgpu/control"     # the grant's MIVGPU_CONTROL_FILE
DEFAULT_LEASE_S = 20.0                             # 4 monitor periods (5 s)


class Control(C.Structure):
    _fields_ = [("magic", C.c_uint32), ("version", C.c_int32), ("seq", C.c_uint64),
                ("lease_until_ns", C.c_int64), ("block", C.c_int32), ("utilization_switch", C.c_int32),
                ("over_grant", C.c_int32), ("reserved0", C.c_int32),
                ("host_excess", C.c_uint64 * MAX_DEVICES), ("unused", C.c_uint64 * 43)]


CTL_SIZE = C.sizeof(Control)
assert CTL_SIZE == 512


def control_host_path(hook_path: str, pod_uid: str, ctr_name: str) -> str:
    return f"{hook_path}/vgpu/control/{pod_uid}_{ctr_name}.ctl"


def create(path: str) -> None:
    """Write an initialised control file (no verdicts, no lease), 0644: the
    container gets it through a read-only bind mount."""
    os.makedirs(os.path.dirname(path), exist_ok=True)
    c = Control()
    c.magic, c.version = CTL_MAGIC, CTL_VERSION
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(bytes(c))
    os.chmod(tmp, 0o644)
    os.replace(tmp, path)


class ControlFile:
    """A control file mapped read-write on the host (the monitor's side)."""

    def __init__(self, path: str):
        self.path = path
        # host-owned directory, but be as careful as with the region files
        self.fd = os.open(path, os.O_RDWR | os.O_NOFOLLOW | os.O_NONBLOCK | os.O_CLOEXEC)
        st = os.fstat(self.fd)
        if not stat.S_ISREG(st.st_mode) or st.st_size < CTL_SIZE:
            os.close(self.fd)
            raise ValueError(f"{path}: not a control file")
        self.mm = mmap.mmap(self.fd, CTL_SIZE, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        self.c = Control.from_buffer(self.mm)
        if int(self.c.magic) != CTL_MAGIC:
            self.close()
            raise ValueError(f"{path}: bad magic")

    def close(self):
        try:
            del self.c
            self.mm.close()
        except (BufferError, ValueError, AttributeError):
            pass
        try:
            os.close(self.fd)
        except OSError:
            pass

    # aligned 4/8-byte stores, matching the shim's relaxed loads
    def publish(self, *, block: bool, switch: bool, over: bool, excess: list[int] | None = None,
                lease_s: float = DEFAULT_LEASE_S, now_ns: int | None = None):
        c = self.c
        for i in range(MAX_DEVICES):
            v = int(excess[i]) if excess is not None and i < len(excess) else 0
            if int(c.host_excess[i]) != v:
                c.host_excess[i] = v
        c.over_grant = 1 if over else 0
        c.utilization_switch = 1 if switch else 0
        c.block = 1 if block else 0
        now = time.time_ns() if now_ns is None else now_ns
        c.lease_until_ns = now + int(lease_s * 1e9)
        c.seq = int(c.seq) + 1

    def snapshot(self) -> dict:
        c = self.c
        return {"seq": int(c.seq), "lease_until_ns": int(c.lease_until_ns), "block": int(c.block),
                "utilization_switch": int(c.utilization_switch), "over_grant": int(c.over_grant),
                "host_excess": [int(v) for v in c.host_excess]}


class ControlSet:
    """The monitor's open control files, keyed ``<pod uid>_<container>``,
    under ``$HOOK_PATH/vgpu/control`` (files of gone containers are closed)."""

    def __init__(self, base: str):
        self.base = base
        self._open: dict[str, ControlFile] = {}
        self._mu = threading.Lock()

    def get(self, key: str) -> ControlFile | None:
        with self._mu:
            cf = self._open.get(key)
            if cf is not None:
                return cf
            path = os.path.join(self.base, f"{key}.ctl")
            try:
                cf = ControlFile(path)
            except (OSError, ValueError):
                return None
            self._open[key] = cf
            return cf

    def retain(self, keys: set):
        with self._mu:
            for k in [k for k in self._open if k not in keys]:
                self._open.pop(k).close()

    def close(self):
        self.retain(set())


def offsets() -> dict:
    """Python-side offsets keyed like MIVGPU_F_CTL_* (shared_region.h)."""
    K = Control
    return {19: K.seq.offset, 20: K.lease_until_ns.offset, 21: K.block.offset, 22: K.utilization_switch.offset,
            23: K.over_grant.offset, 24: K.host_excess.offset, 25: CTL_SIZE}


__all__ = ["Control", "ControlFile", "ControlSet", "create", "control_host_path", "offsets",
           "CONTAINER_CONTROL_PATH", "CTL_MAGIC"]
