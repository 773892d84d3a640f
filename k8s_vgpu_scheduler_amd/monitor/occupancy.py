"""Host-side wave-occupancy sampler (monitor side of the governor's share signal).

KFD publishes, for every process that opened a GPU, the wavefronts its queues
have resident on that GPU: ``<kfd>/proc/<host pid>/stats_<gpu_id>/cu_occupancy``
(SPI_CSQ_WF_ACTIVE_COUNT in CU units; ~7 us per read on MI355X,
profiles/governor_occupancy/).  The shim integrates its own share of it to
charge the governor; the monitor, which runs with hostPID, samples every
process on every GPU to

  * count the tenants actually running on a GPU (``mivgpu_host_gpu_active_tenants``),
  * report a container's utilisation when its shim has not (occupancy off, no
    KFD view inside the container): the share of resident waves its processes
    held over the sampling window -- the analogue of the per-process SM
    utilisation the reference reads from NVML (cmd/vGPUmonitor/metrics.go:468-497).

GPUs are matched by PCI location (KFD topology ``location_id``/``domain``
against the backend's BDF), so partitions (one KFD node per PCI function) are
told apart.
"""

from __future__ import annotations

import os
import threading
import time
from collections import deque
from pathlib import Path

KFD_ROOT = Path(os.environ.get("MIVGPU_KFD_SYSFS", "/sys/class/kfd/kfd"))


def _props(path: Path) -> dict:
    out = {}
    try:
        for line in path.read_text().splitlines():
            k, _, v = line.partition(" ")
            try:
                out[k] = int(v)
            except ValueError:
                pass
    except OSError:
        pass
    return out


def kfd_gpu_nodes(root: Path = KFD_ROOT) -> list[dict]:
    """Every GPU node of the KFD topology: ``{"node", "gpu_id", "bdf",
    "uuid"}`` (``uuid`` is ``GPU-<unique_id as 16 hex digits>``, the form the
    backends register, smi/__init__.py ``_rocr_id_from_kfd``; "" without one)."""
    out = []
    nodes = Path(root) / "topology" / "nodes"
    try:
        entries = sorted(nodes.iterdir(), key=lambda p: int(p.name) if p.name.isdigit() else -1)
    except OSError:
        return out
    for n in entries:
        try:
            gid = int((n / "gpu_id").read_text().strip() or 0)
        except (OSError, ValueError):
            continue
        if not gid:
            continue
        p = _props(n / "properties")
        loc, dom = p.get("location_id"), p.get("domain", 0)
        bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}" if loc is not None else ""
        uid = p.get("unique_id")
        out.append({"node": int(n.name) if n.name.isdigit() else -1, "gpu_id": gid, "bdf": bdf,
                    "uuid": f"GPU-{uid:016x}" if uid else ""})
    return out


def norm_bdf(bdf: str) -> str:
    """``0000:A4:00.0`` / ``a4:00.0`` -> ``0000:a4:00.0`` (amd-smi and sysfs
    spell the same function differently on some stacks)."""
    s = str(bdf or "").strip().lower()
    if not s:
        return ""
    if s.count(":") == 1:
        s = "0000:" + s
    dom, _, rest = s.partition(":")
    try:
        return f"{int(dom, 16):04x}:{rest}"
    except ValueError:
        return s


def gpu_ids_by_bdf(root: Path = KFD_ROOT) -> dict[str, int]:
    """``{"0000:75:00.0": gpu_id}`` for every GPU node of the KFD topology."""
    return {n["bdf"]: n["gpu_id"] for n in kfd_gpu_nodes(root) if n["bdf"]}


def read_occupancy(root: Path = KFD_ROOT) -> dict[int, dict[int, int]]:
    """One sample: ``{gpu_id: {host pid: cu_occupancy}}`` (zeros included)."""
    out: dict[int, dict[int, int]] = {}
    proc = root / "proc"
    try:
        pids = [d for d in os.listdir(proc) if d.isdigit()]
    except OSError:
        return out
    for pid in pids:
        base = proc / pid
        try:
            stats = [s for s in os.listdir(base) if s.startswith("stats_")]
        except OSError:
            continue
        for s in stats:
            try:
                gid = int(s[6:])
                v = int((base / s / "cu_occupancy").read_text().strip() or 0)
            except (OSError, ValueError):
                continue
            out.setdefault(gid, {})[int(pid)] = v
    return out


class OccupancySampler:
    """Samples every ``period_s`` on a daemon thread; keeps ``window_s`` of history."""

    def __init__(self, root: Path = KFD_ROOT, period_s: float = 0.05, window_s: float = 2.0):
        self.root, self.period, self.window = Path(root), period_s, window_s
        self._hist: deque[tuple[float, dict[int, dict[int, int]]]] = deque()
        self._mu = threading.Lock()
        self._stop = threading.Event()
        self._th: threading.Thread | None = None

    def available(self) -> bool:
        return (self.root / "proc").is_dir()

    def sample_once(self, now: float | None = None):
        snap = read_occupancy(self.root)
        t = time.monotonic() if now is None else now
        with self._mu:
            self._hist.append((t, snap))
            while self._hist and t - self._hist[0][0] > self.window:
                self._hist.popleft()

    def start(self):
        if self._th is None and self.available():
            self._th = threading.Thread(target=self._run, name="occupancy", daemon=True)
            self._th.start()
        return self

    def stop(self):
        self._stop.set()

    def _run(self):
        while not self._stop.wait(self.period):
            self.sample_once()

    def _samples(self, gpu_id: int) -> list[dict[int, int]]:
        with self._mu:
            return [s.get(gpu_id, {}) for _, s in self._hist]

    def active_tenants(self, gpu_id: int) -> int | None:
        """Processes with waves resident on the GPU in any sample of the window."""
        samples = self._samples(gpu_id)
        if not samples:
            return None
        return len({pid for s in samples for pid, v in s.items() if v > 0})

    def share_pct(self, gpu_id: int, pids) -> float | None:
        """Mean share (percent) of the GPU's resident waves held by ``pids``."""
        samples = self._samples(gpu_id)
        if not samples:
            return None
        pids = set(pids)
        acc = 0.0
        for s in samples:
            tot = sum(v for v in s.values() if v > 0)
            if tot:
                acc += sum(v for p, v in s.items() if p in pids and v > 0) / tot
        return 100.0 * acc / len(samples)
