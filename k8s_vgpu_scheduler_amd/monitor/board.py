"""Share boards: one wave-occupancy sampler per GPU (monitor side).

ctypes mirror of ``mivgpu_board_t`` (csrc/include/mivgpu/shared_region.h,
owner logic in csrc/shim/board.h) plus the node sampler's process.

The governor charges a tenant the GPU time it receives: its share of the
resident wavefronts KFD reports per process.  When each tenant sampled that
on its own clock, four symmetric 25 % tenants were charged 100 / 33 / 100 /
100 % of their busy time.  The reference serialises
utilisation sampling across containers through the host lock directory
``/tmp/vgpulock`` (pkg/device-plugin/nvidiadevice/nvinternal/plugin/
server.go:853-864); here ONE owner per GPU reads every process's
``cu_occupancy`` in the same pass and publishes per-pid integrals in
``<board dir>/gpu-<kfd gpu_id>.board``:

* production: the monitor runs ``mivgpu-boardd`` (``BoardSampler``) on
  ``$HOOK_PATH/vgpu/board``, which the device plugin mounts READ-ONLY into
  every vGPU container (``deviceplugin/allocate.py``) -- no tenant can write
  the share it is charged -- and one read-write flags directory per
  container (``flags/<pod uid>_<container>/``, mounted at
  ``MIVGPU_BOARD_FLAGS_DIR`` in that container only) where its shim publishes
  whether it is held in its governor gate, whether it owes work, whether it
  gates at all and its core limit; the owner reads a pid's flags only from
  the directory of the container host truth attributes it to
  (``gpu-<id>.owners``, written by the monitor) and weighs it with the
  node-written limit (``gpu-<id>.limits``) -- ADVICE r5;
* without a node sampler (hand-run slices, the bench), a shim that governs
  the GPU takes the owner role with ``flock`` on ``gpu-<id>.owner``.

The monitor also reads the boards for per-process utilisation (``recv_ns``).
"""

from __future__ import annotations

import ctypes as C
import logging
import mmap
import os
import subprocess
import time
from pathlib import Path

BOARD_MAGIC = 0x4D495642
BOARD_VERSION = 2
BOARD_SLOTS = 64
OWNER_NONE, OWNER_NODE, OWNER_SHIM = 0, 1, 2
CONTAINER_BOARD_DIR = "/var/run/mivgpu/board"    # the grant's MIVGPU_BOARD_DIR (read-only mount)

log = logging.getLogger("mivgpu.board")


class BoardSlot(C.Structure):
    _fields_ = [("pid", C.c_int32), ("occupancy", C.c_int32), ("seen_ns", C.c_uint64), ("obs_ns", C.c_uint64),
                ("frac_ns", C.c_uint64), ("recv_ns", C.c_uint64), ("busy_ns", C.c_uint64),
                ("vt_ns", C.c_uint64), ("lead_ns", C.c_int64)]


class BoardHeader(C.Structure):
    _fields_ = [("magic", C.c_uint32), ("version", C.c_int32), ("gpu_id", C.c_int32), ("owner_kind", C.c_int32),
                ("owner_pid", C.c_int32), ("nslots", C.c_int32), ("seq", C.c_uint64), ("beat_ns", C.c_uint64),
                ("period_ns", C.c_uint64), ("passes", C.c_uint64), ("want_fast_ns", C.c_uint64),
                ("busy_ns", C.c_uint64), ("pass_ns", C.c_uint64), ("sub_passes", C.c_uint64),
                ("fair_passes", C.c_uint64), ("unused", C.c_uint64 * 4),
                ("slots", BoardSlot * BOARD_SLOTS)]


BOARD_SIZE = C.sizeof(BoardHeader)
assert C.sizeof(BoardSlot) == 64 and BOARD_SIZE == 128 + 64 * BOARD_SLOTS

FLAGS_MAGIC = 0x4D495646
FLAGS_VERSION = 2
FLAGS_SLOTS = 256
FLAG_HELD, FLAG_OWES, FLAG_GATED = 1, 2, 4


class Flag(C.Structure):
    _fields_ = [("pid", C.c_int32), ("state", C.c_int32), ("stamp_ns", C.c_uint64), ("limit_ppm", C.c_uint32),
                ("reserved", C.c_uint32), ("unused", C.c_uint64)]


class Flags(C.Structure):
    _fields_ = [("magic", C.c_uint32), ("version", C.c_int32), ("gpu_id", C.c_int32), ("reserved", C.c_int32),
                ("unused", C.c_uint64 * 6), ("flags", Flag * FLAGS_SLOTS)]


FLAGS_SIZE = C.sizeof(Flags)
assert FLAGS_SIZE == 64 + 32 * FLAGS_SLOTS


def offsets() -> dict:
    """Field offsets for the ABI test against mivgpu_abi_offsetof()."""
    # MIVGPU_F_BOARD_SEQ .. MIVGPU_F_SIZEOF_FLAGS (enum order in shared_region.h)
    return {26: BoardHeader.seq.offset, 27: BoardHeader.beat_ns.offset, 28: BoardHeader.slots.offset,
            29: BOARD_SIZE, 30: C.sizeof(BoardSlot), 31: Flags.flags.offset, 32: FLAGS_SIZE}


def flags_path(board_dir: str, gpu_id: int) -> Path:
    return Path(board_dir) / "flags" / f"gpu-{gpu_id}.flags"


class FlagsFile:
    """The tenant-written flags of one GPU mapped read-write (tests stand in
    for tenants with it; the owner reads it in its pass)."""

    def __init__(self, board_dir: str, gpu_id: int, create: bool = True, flags_dir: str | None = None):
        p = Path(flags_dir) / f"gpu-{gpu_id}.flags" if flags_dir else flags_path(board_dir, gpu_id)
        if create and not p.exists():
            p.parent.mkdir(parents=True, exist_ok=True)
            f = Flags()
            f.magic, f.version, f.gpu_id = FLAGS_MAGIC, FLAGS_VERSION, gpu_id
            tmp = p.with_name(p.name + f".{os.getpid()}")
            tmp.write_bytes(bytes(f))
            try:
                os.link(tmp, p)
            except FileExistsError:
                pass
            tmp.unlink()
        fd = os.open(p, os.O_RDWR | os.O_CLOEXEC)
        try:
            self.mm = mmap.mmap(fd, FLAGS_SIZE, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self.f = Flags.from_buffer(self.mm)

    def publish(self, pid: int, state: int, limit_ppm: int = 0):
        slot = next((e for e in self.f.flags if e.pid == pid), None) or next(e for e in self.f.flags if e.pid == 0)
        slot.pid, slot.state, slot.limit_ppm, slot.stamp_ns = pid, state, limit_ppm, time.monotonic_ns()

    def entries(self) -> dict[int, tuple[int, int]]:
        return {e.pid: (e.state, e.stamp_ns) for e in self.f.flags if e.pid}

    def close(self):
        del self.f
        self.mm.close()


def board_path(board_dir: str, gpu_id: int) -> Path:
    return Path(board_dir) / f"gpu-{gpu_id}.board"


LIMITS_MAGIC = 0x4D49564C
LIMITS_VERSION = 1
LIMITS_MAX = 1024


def limits_path(board_dir: str, gpu_id: int) -> Path:
    return Path(board_dir) / f"gpu-{gpu_id}.limits"


def write_limits(board_dir: str, gpu_id: int, limits: dict[int, int]) -> Path:
    """The node-written core limits of one GPU (``mivgpu_board_limits_t``):
    ``{host pid: limit ppm}``; the owner pass weighs each process with this
    limit whenever there is one (its flags' limit is ignored then).  Written under a private name and
    renamed into place (the owner re-reads it every 100 ms)."""
    import struct
    items = sorted((int(p), int(v)) for p, v in limits.items() if p > 0 and 0 < v < 1_000_000)[:LIMITS_MAX]
    blob = struct.pack("<IiiI", LIMITS_MAGIC, LIMITS_VERSION, gpu_id, len(items))
    blob += b"".join(struct.pack("<iI", p, v) for p, v in items)
    path = limits_path(board_dir, gpu_id)
    tmp = path.with_name(f".{path.name}.{os.getpid()}")
    tmp.write_bytes(blob)
    os.chmod(tmp, 0o644)
    os.replace(tmp, path)
    return path


def owners_path(board_dir: str, gpu_id: int) -> Path:
    return Path(board_dir) / f"gpu-{gpu_id}.owners"


_KEY_OK = set("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_.-")


def valid_key(key: str) -> bool:
    """A container key (``<pod uid>_<container>``) as the node sampler
    accepts it (board.h ``valid_key``)."""
    return 0 < len(key) < 128 and key not in (".", "..") and set(key) <= _KEY_OK


def write_owners(board_dir: str, gpu_id: int, owners: dict[int, str]) -> Path:
    """Host truth's ``{host pid: container key}`` of one GPU
    (``<dir>/gpu-<id>.owners``): the node sampler reads a pid's flags only
    from ``<dir>/flags/<key>/``, so no tenant can speak for a neighbour
    (ADVICE r5).  Written under a private name and renamed into place."""
    lines = [f"MIVGPU-OWNERS 1 {gpu_id}"]
    lines += [f"{int(p)} {k}" for p, k in sorted(owners.items()) if int(p) > 0 and valid_key(k)][:1024]
    path = owners_path(board_dir, gpu_id)
    tmp = path.with_name(f".{path.name}.{os.getpid()}")
    tmp.write_text("\n".join(lines) + "\n")
    os.chmod(tmp, 0o644)
    os.replace(tmp, path)
    return path


def container_flags_dir(board_dir: str, key: str) -> str:
    """The host directory of one container's flags (mounted read-write at
    ``CONTAINER_FLAGS_DIR`` in that container only)."""
    return os.path.join(board_dir, "flags", key)


CONTAINER_FLAGS_DIR = "/var/run/mivgpu/board-flags"    # the grant's MIVGPU_BOARD_FLAGS_DIR


def board_host_dir(hook_path: str) -> str:
    return f"{hook_path}/vgpu/board"


class Board:
    """One GPU's board mapped read-only (monitor, tests)."""

    def __init__(self, path):
        self.path = str(path)
        fd = os.open(self.path, os.O_RDONLY | os.O_CLOEXEC)
        try:
            if os.fstat(fd).st_size < BOARD_SIZE:
                raise ValueError(f"{path}: not a share board")
            self.mm = mmap.mmap(fd, BOARD_SIZE, mmap.MAP_SHARED, mmap.PROT_READ)
        finally:
            os.close(fd)
        h = BoardHeader.from_buffer_copy(self.mm)
        if h.magic != BOARD_MAGIC or h.version != BOARD_VERSION:
            self.mm.close()
            raise ValueError(f"{path}: bad board magic/version")

    def close(self):
        self.mm.close()

    def snapshot(self, tries: int = 50) -> BoardHeader:
        """A consistent copy (seqlock: retried while the owner writes)."""
        off = BoardHeader.seq.offset
        for _ in range(tries):
            s1 = int.from_bytes(self.mm[off:off + 8], "little")
            if s1 & 1:
                time.sleep(0.0001)
                continue
            h = BoardHeader.from_buffer_copy(self.mm)
            if h.seq == s1:
                return h
        return BoardHeader.from_buffer_copy(self.mm)

    def slots(self) -> dict[int, BoardSlot]:
        h = self.snapshot()
        return {s.pid: s for s in h.slots if s.pid}

    def live(self, max_age_s: float = 0.05) -> bool:
        h = self.snapshot()
        return h.beat_ns > 0 and time.monotonic_ns() - h.beat_ns < max_age_s * 1e9


def shares(before: BoardHeader, after: BoardHeader) -> dict[int, dict]:
    """Per pid between two snapshots: the mean share charged while not held
    (frac / obs) and the share of the window received (recv / wall)."""
    b = {s.pid: s for s in before.slots if s.pid}
    wall = max(1, after.beat_ns - before.beat_ns)
    out = {}
    for s in after.slots:
        if not s.pid:
            continue
        p = b.get(s.pid)
        obs = s.obs_ns - (p.obs_ns if p else 0)
        frac = s.frac_ns - (p.frac_ns if p else 0)
        recv = s.recv_ns - (p.recv_ns if p else 0)
        out[s.pid] = {"charged_share": frac / obs if obs > 0 else None, "received": recv / wall,
                      "obs_ms": obs / 1e6, "occupancy": s.occupancy,
                      "lead_ms": s.lead_ns / 1e6 if s.lead_ns >= 0 else None}
    return out


def boardd_path() -> Path:
    return Path(__file__).resolve().parents[1] / "lib" / "mivgpu-boardd"


class BoardSampler:
    """The node sampler process (``mivgpu-boardd``), owned by the monitor."""

    def __init__(self, board_dir: str, kfd_sysfs: str | None = None, period_us: int = 2000,
                 idle_period_us: int = 20000, binary: str | None = None, extra_args: list | None = None):
        self.dir = board_dir
        self.kfd = kfd_sysfs or os.environ.get("MIVGPU_KFD_SYSFS", "/sys/class/kfd/kfd")
        self.args = ["--period-us", str(period_us), "--idle-period-us", str(idle_period_us), *(extra_args or [])]
        self.binary = binary or str(boardd_path())
        self.proc: subprocess.Popen | None = None

    def available(self) -> bool:
        return os.access(self.binary, os.X_OK) and os.path.isdir(os.path.join(self.kfd, "proc"))

    def start(self) -> "BoardSampler":
        if self.proc is not None or not self.available():
            if self.proc is None:
                log.warning("share-board sampler not started (binary %s, KFD %s)", self.binary, self.kfd)
            return self
        os.makedirs(os.path.join(self.dir, "flags"), exist_ok=True)
        try:
            # containers read the board through a read-only mount, and write
            # their flags only in their own flags/<key>/ (deviceplugin/
            # allocate.py); no tenant can create, replace or unlink anything
            # the root sampler opens here
            os.chmod(self.dir, 0o755)
            os.chmod(os.path.join(self.dir, "flags"), 0o755)
        except OSError:
            pass
        self.proc = subprocess.Popen([self.binary, "--dir", self.dir, "--kfd-sysfs", self.kfd, *self.args,
                                      "--exit-with-parent"], stdout=subprocess.DEVNULL, stderr=None)
        log.info("share-board sampler pid %d on %s", self.proc.pid, self.dir)
        return self

    def alive(self) -> bool:
        return self.proc is not None and self.proc.poll() is None

    def ensure(self, now: float | None = None) -> bool:
        """Restart the sampler if it exited (no tenant can take
        the owner role over a read-only board, so a dead sampler would leave
        every tenant on its own local estimate).  Backs off 1 s, 2 s, ... up
        to 60 s between attempts; returns whether a sampler runs now."""
        if self.alive():
            self._backoff = 0.0
            return True
        if self.proc is None and not self.available():
            return False
        t = time.monotonic() if now is None else now
        if t < getattr(self, "_next_try", 0.0):
            return False
        rc = self.proc.poll() if self.proc is not None else None
        self.restarts = getattr(self, "restarts", 0) + 1
        self._backoff = min(60.0, max(1.0, 2 * getattr(self, "_backoff", 0.0)))
        self._next_try = t + self._backoff
        log.warning("share-board sampler exited (rc %s): restarting (attempt %d, next retry in %.0f s)",
                    rc, self.restarts, self._backoff)
        self.proc = None
        self.start()
        return self.alive()

    def stop(self):
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(timeout=5)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
