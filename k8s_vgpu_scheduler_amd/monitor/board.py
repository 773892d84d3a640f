"""Reader of the shims' per-GPU share boards (monitor side).

Every shimmed process stamps its launches into
``$MIVGPU_LOCK_DIR/mivgpu-board-<domain>-<bus>-<device>-<function>`` (64 x
``{u64 token, u64 last_ns}``, CLOCK_MONOTONIC_COARSE; docs/protocol.md "Share
board").  The governor refills at limit x active tenants; the monitor exports
the same count per GPU as ``mivgpu_host_gpu_active_tenants``.
"""

from __future__ import annotations

import os
import struct
import time
from pathlib import Path

SLOTS = 64
# Linux CLOCK_MONOTONIC_COARSE (the shim's clock); Python 3.10 has no constant for it
_COARSE = getattr(time, "CLOCK_MONOTONIC_COARSE", 6)


def now_ns() -> int:
    return time.clock_gettime_ns(_COARSE)


def lock_dir() -> Path:
    return Path(os.environ.get("MIVGPU_LOCK_DIR", "/tmp/vgpulock"))


def board_path(bdf: str, root: Path | None = None) -> Path | None:
    """``0000:75:00.1`` -> ``<lock dir>/mivgpu-board-0000-75-00-1``."""
    try:
        dbd, fn = bdf.rsplit(".", 1)
        domain, bus, dev = dbd.split(":")
        name = f"mivgpu-board-{int(domain, 16):04x}-{int(bus, 16):02x}-{int(dev, 16):02x}-{int(fn, 16):x}"
    except ValueError:
        return None
    return (root or lock_dir()) / name


def read_slots(path: Path) -> list[tuple[int, int]]:
    try:
        raw = path.read_bytes()
    except OSError:
        return []
    n = min(SLOTS, len(raw) // 16)
    return [struct.unpack_from("<QQ", raw, 16 * i) for i in range(n)]


def active_tenants(path: Path, window_s: float = 1.0, at_ns: int | None = None) -> int:
    """Tenants that launched on this GPU within ``window_s`` (of ``at_ns``, default now)."""
    now = now_ns() if at_ns is None else at_ns
    win = int(window_s * 1e9)
    return sum(1 for tok, last in read_slots(path) if tok and (last > now or now - last < win))
