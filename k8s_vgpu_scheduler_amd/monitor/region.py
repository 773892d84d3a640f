"""ctypes mirror of ``mivgpu_shared_region_t`` (csrc/include/mivgpu/shared_region.h).

Counterpart of the reference's Go mirror pkg/monitor/nvidia/v1/spec.go:24-240:
aggregated per-device usage over active process slots, limits, and atomic-width
setters for the feedback loop (``recent_kernel``, ``utilization_switch``,
limits).  Offsets are pinned against the C layout by
tests/test_shared_region_abi.py through ``mivgpu_abi_offsetof``.
"""

from __future__ import annotations

import ctypes as C
import mmap
import stat
import os

MAGIC = 0x4D495647
MAX_DEVICES = 16
MAX_PROCS = 1024
UUID_LEN = 96
SLOT_ACTIVE = 1


class MemT(C.Structure):
    _fields_ = [("context", C.c_uint64), ("module", C.c_uint64), ("buffer", C.c_uint64), ("vmm", C.c_uint64),
                ("total", C.c_uint64), ("peak", C.c_uint64), ("unused", C.c_uint64 * 2)]


class UtilT(C.Structure):
    _fields_ = [("launches", C.c_uint64), ("busy_ns", C.c_uint64), ("throttled_ns", C.c_uint64),
                ("gates", C.c_uint64), ("util_pct", C.c_uint64), ("share_ns", C.c_uint64),
                ("occupancy", C.c_uint64), ("share_ppm", C.c_uint64)]


class ProcSlot(C.Structure):
    _fields_ = [("pid", C.c_int32), ("hostpid", C.c_int32), ("status", C.c_int32), ("priority", C.c_int32),
                ("start_ns", C.c_uint64), ("heartbeat_ns", C.c_uint64), ("unused", C.c_uint64 * 5),
                ("used", MemT * MAX_DEVICES), ("util", UtilT * MAX_DEVICES)]


class Region(C.Structure):
    _fields_ = [("magic", C.c_uint32), ("major_version", C.c_int32), ("minor_version", C.c_int32),
                ("initialized", C.c_int32), ("owner_pid", C.c_uint64), ("lock", C.c_uint8 * 64),
                ("num_devices", C.c_uint64), ("procnum", C.c_int32), ("utilization_switch", C.c_int32),
                ("recent_kernel", C.c_int32), ("priority", C.c_int32), ("last_kernel_time", C.c_int64),
                ("core_policy", C.c_int32), ("oversubscribe", C.c_int32), ("unused0", C.c_uint64 * 2),
                ("uuids", (C.c_char * UUID_LEN) * MAX_DEVICES), ("mem_limit", C.c_uint64 * MAX_DEVICES),
                ("cu_limit", C.c_uint64 * MAX_DEVICES), ("cu_mask_count", C.c_uint64 * MAX_DEVICES),
                ("dev_used", C.c_uint64 * MAX_DEVICES), ("unused1", C.c_uint64 * 16),
                ("procs", ProcSlot * MAX_PROCS)]


REGION_SIZE = C.sizeof(Region)


class SharedRegion:
    """A mapped shared-region file (read-mostly; setters are naturally atomic
    aligned 4/8-byte stores, matching the C side's relaxed atomics)."""

    def __init__(self, path: str, writable: bool = True):
        self.path = path
        # The file sits in a directory the container writes: never follow a
        # planted symlink (the privileged monitor would map and write a host
        # file), never block on a FIFO, accept only a regular file.
        flags = (os.O_RDWR if writable else os.O_RDONLY) | os.O_NOFOLLOW | os.O_NONBLOCK | os.O_CLOEXEC
        self.fd = os.open(path, flags)
        st = os.fstat(self.fd)
        if not stat.S_ISREG(st.st_mode):
            os.close(self.fd)
            raise ValueError(f"{path}: not a regular file")
        size = st.st_size
        if size < REGION_SIZE:
            os.close(self.fd)
            raise ValueError(f"{path}: {size} bytes < region size {REGION_SIZE}")
        self.mm = mmap.mmap(self.fd, REGION_SIZE, mmap.MAP_SHARED,
                            mmap.PROT_READ | (mmap.PROT_WRITE if writable else 0))
        self.r = Region.from_buffer(self.mm) if writable else Region.from_buffer_copy(self.mm)
        self.writable = writable
        magic = int(self.r.magic)
        if magic != MAGIC:
            self.close()   # drops self.r: report the value read before
            raise ValueError(f"{path}: bad magic {magic:#x}")

    @classmethod
    def create(cls, path: str, num_devices: int = 1, mem_limit: int = 0, cu_limit: int = 100) -> "SharedRegion":
        """Initialise a region file the way the shim does (tests / tooling)."""
        with open(path, "wb") as f:
            f.truncate(REGION_SIZE)
        fd = os.open(path, os.O_RDWR)
        mm = mmap.mmap(fd, REGION_SIZE, mmap.MAP_SHARED)
        r = Region.from_buffer(mm)
        r.major_version, r.minor_version, r.initialized = 1, 1, 1
        r.num_devices = num_devices
        for d in range(MAX_DEVICES):
            r.mem_limit[d] = mem_limit
            r.cu_limit[d] = cu_limit
        r.magic = MAGIC
        del r
        mm.close()
        os.close(fd)
        return cls(path)

    def close(self):
        try:
            if self.writable:
                del self.r
            self.mm.close()
        except (BufferError, ValueError, AttributeError):
            pass
        try:
            os.close(self.fd)
        except OSError:
            pass

    # --------------------------------------------------------------- reads
    def device_num(self) -> int:
        return min(int(self.r.num_devices), MAX_DEVICES)

    def active_procs(self):
        n = max(0, min(int(self.r.procnum), MAX_PROCS))
        return [p for p in self.r.procs[:n] if p.status == SLOT_ACTIVE]

    def uuid(self, idx: int) -> str:
        return bytes(self.r.uuids[idx]).split(b"\0", 1)[0].decode(errors="replace")

    def is_valid_uuid(self, idx: int) -> bool:
        return bytes(self.r.uuids[idx])[:1] not in (b"", b"\0")

    def memory_total(self, idx: int) -> int:
        return sum(p.used[idx].total for p in self.active_procs())

    def memory_field(self, idx: int, field: str) -> int:
        return sum(getattr(p.used[idx], field) for p in self.active_procs())

    def memory_limit(self, idx: int) -> int:
        return int(self.r.mem_limit[idx])

    def dev_used(self, idx: int) -> int:
        return int(self.r.dev_used[idx])

    def busy_ns(self, idx: int) -> int:
        return sum(p.util[idx].busy_ns for p in self.active_procs())

    def launches(self, idx: int) -> int:
        return sum(p.util[idx].launches for p in self.active_procs())

    def pids(self) -> list[int]:
        return [p.pid for p in self.active_procs()]

    def priority(self) -> int:
        return int(self.r.priority)

    def recent_kernel(self) -> int:
        return int(self.r.recent_kernel)

    def utilization_switch(self) -> int:
        return int(self.r.utilization_switch)

    def last_kernel_time(self) -> int:
        return int(self.r.last_kernel_time)

    def refresh(self):
        if not self.writable:
            self.r = Region.from_buffer_copy(self.mm)

    # -------------------------------------------------------------- writes
    def set_recent_kernel(self, v: int):
        self.r.recent_kernel = v

    def set_utilization_switch(self, v: int):
        self.r.utilization_switch = v

    def set_memory_limit(self, limit_bytes: int):
        for d in range(self.device_num()):
            self.r.mem_limit[d] = limit_bytes

    def set_cu_limit(self, pct: int):
        for d in range(self.device_num()):
            self.r.cu_limit[d] = pct


def offsets() -> dict:
    """Python-side offsets, keyed like MIVGPU_F_* (shared_region.h)."""
    R = Region
    return {0: R.magic.offset, 1: R.lock.offset, 2: R.num_devices.offset, 3: R.procnum.offset,
            4: R.utilization_switch.offset, 5: R.recent_kernel.offset, 6: R.priority.offset,
            7: R.last_kernel_time.offset, 8: R.core_policy.offset, 9: R.uuids.offset, 10: R.mem_limit.offset,
            11: R.cu_limit.offset, 12: R.cu_mask_count.offset, 13: R.dev_used.offset, 14: R.procs.offset,
            15: C.sizeof(Region), 16: C.sizeof(ProcSlot), 17: ProcSlot.used.offset, 18: ProcSlot.util.offset}
