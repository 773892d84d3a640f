"""Device discovery / health / telemetry layer (the AMD replacement for NVML).

``GPUInfo`` is what the device plugin registers and the monitor exports.
Backends:
  * :class:`AmdSmiBackend`  -- ROCm amd-smi Python bindings (``amdsmi``):
    memory, CU count, NUMA node, BDF, DRM render/card minor, KFD unique id
    (the ROCr-compatible ``GPU-<hex>`` id: docs/develop/amd-vgpu.md:174-180),
    xGMI link type/hops/bandwidth, RAS/ECC, activity, per-process VRAM;
  * :class:`SysfsBackend`   -- /sys/class/kfd topology, no library needed;
  * :class:`FakeBackend`    -- synthetic MI355X nodes for tests.
``detect()`` picks the first that works.
"""

from __future__ import annotations

import logging
import os
import re
from dataclasses import dataclass, field
from pathlib import Path

log = logging.getLogger(__name__)


@dataclass
class GPUInfo:
    index: int
    uuid: str                 # stable id registered with the scheduler
    rocr_id: str              # value for ROCR_VISIBLE_DEVICES ("GPU-<16 hex>" or index)
    name: str = "AMD Instinct MI355X"
    memory_mib: int = 294912
    cus: int = 256
    xcds: int = 8
    numa: int = 0
    bdf: str = ""
    render_minor: int = -1    # /dev/dri/renderD<minor>
    card_minor: int = -1      # /dev/dri/card<minor>
    healthy: bool = True
    compute_partition: str = "SPX"
    memory_partition: str = "NPS1"
    physical_index: int = -1     # physical GPU this (partition) device belongs to; -1 = index
    partition_index: int = 0
    extra: dict = field(default_factory=dict)

    @property
    def physical(self) -> int:
        return self.index if self.physical_index < 0 else self.physical_index


# MI355X compute-partition modes: logical GPUs per physical GPU (XCDs split evenly).
PARTITION_MODES = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}
MEMORY_MODES = ("NPS1", "NPS2")


class PartitionError(RuntimeError):
    pass


@dataclass
class LinkInfo:
    type: str        # "XGMI" | "PCIE" | "NONE"
    hops: int = 1
    links: int = 1
    max_bw_gbps: float | None = None


class Backend:
    name = "base"
    skip_checks: set = set()     # health checks disabled via DP_DISABLE_HEALTHCHECKS

    def gpus(self) -> list[GPUInfo]:
        raise NotImplementedError

    def link(self, a: GPUInfo, b: GPUInfo) -> LinkInfo:
        return LinkInfo("NONE", 0, 0)

    def health(self, g: GPUInfo) -> tuple[bool, str]:
        return True, ""

    def memory_used_mib(self, g: GPUInfo) -> int:
        return 0

    def utilization(self, g: GPUInfo) -> dict:
        return {"gfx": 0.0, "umc": 0.0}

    def processes(self, g: GPUInfo) -> list[dict]:
        return []

    def set_compute_partition(self, physical_index: int, mode: str) -> None:
        """Reconfigure one physical GPU (must be idle; needs privileges)."""
        raise PartitionError(f"{self.name}: compute partitioning not supported")

    def shutdown(self):
        pass


def pair_scores(backend: Backend, gpus: list[GPUInfo]) -> dict[str, dict[str, int]]:
    from k8s_vgpu_scheduler_amd.device.amd.topology import pair_score
    out: dict[str, dict[str, int]] = {}
    for a in gpus:
        row = {}
        for b in gpus:
            if a.uuid == b.uuid:
                continue
            li = backend.link(a, b)
            row[b.uuid] = pair_score(li.type, li.hops, li.links, li.max_bw_gbps, a.numa == b.numa)
        out[a.uuid] = row
    return out


# ------------------------------------------------------------------- amd-smi
class AmdSmiBackend(Backend):
    name = "amdsmi"

    def __init__(self):
        import amdsmi  # noqa: F401  (raises ImportError where absent)
        self.m = amdsmi
        amdsmi.amdsmi_init()
        self.handles = amdsmi.amdsmi_get_processor_handles()
        if not self.handles:
            raise RuntimeError("amd-smi found no GPUs")
        self._by_uuid = {}

    def gpus(self) -> list[GPUInfo]:
        m, out = self.m, []
        for i, h in enumerate(self.handles):
            def q(fn, *a, default=None):
                try:
                    return getattr(m, fn)(h, *a)
                except Exception:  # noqa: BLE001
                    return default
            uuid = q("amdsmi_get_gpu_device_uuid", default=f"gpu-{i}")
            asic = q("amdsmi_get_gpu_asic_info", default={}) or {}
            total = q("amdsmi_get_gpu_memory_total", m.AmdSmiMemoryType.VRAM, default=0) or 0
            numa = q("amdsmi_topo_get_numa_node_number", default=0) or 0
            bdf = q("amdsmi_get_gpu_device_bdf", default="") or ""
            enum = q("amdsmi_get_gpu_enumeration_info", default={}) or {}
            kfd = q("amdsmi_get_gpu_kfd_info", default={}) or {}
            part = q("amdsmi_get_gpu_compute_partition", default="SPX") or "SPX"
            cus = int(asic.get("num_of_compute_units") or asic.get("num_compute_units") or 256)
            rocr = _rocr_id_from_kfd(kfd.get("node_id")) or str(i)
            g = GPUInfo(index=i, uuid=str(uuid), rocr_id=rocr,
                        name=str(asic.get("market_name") or "AMD Instinct MI355X"),
                        memory_mib=int(total) // (1 << 20), cus=cus, numa=max(0, int(numa)), bdf=str(bdf),
                        render_minor=int(enum.get("drm_render", -1) if isinstance(enum.get("drm_render"), int) else -1),
                        card_minor=int(enum.get("drm_card", -1) if isinstance(enum.get("drm_card"), int) else -1),
                        compute_partition=str(part))
            self._by_uuid[g.uuid] = h
            out.append(g)
        # partitions of one physical GPU share domain:bus:device, differ in function
        phys: dict[str, int] = {}
        for g in out:
            key = g.bdf.rsplit(".", 1)[0] if g.bdf else f"idx{g.index}"
            g.partition_index = sum(1 for o in out[: g.index] if (o.bdf.rsplit(".", 1)[0] if o.bdf else "") == key)
            g.physical_index = phys.setdefault(key, len(phys))
        return out

    def set_compute_partition(self, physical_index: int, mode: str) -> None:
        mode = mode.upper()
        if mode not in PARTITION_MODES:
            raise PartitionError(f"unknown compute partition {mode}")
        gs = [g for g in self.gpus() if g.physical == physical_index]
        if not gs:
            raise PartitionError(f"no physical GPU {physical_index}")
        enum = getattr(self.m, "AmdSmiComputePartitionType", None)
        try:
            self.m.amdsmi_set_gpu_compute_partition(self._h(gs[0]), getattr(enum, mode) if enum else mode)
        except Exception as e:  # noqa: BLE001
            raise PartitionError(f"amd-smi set compute partition {mode} on GPU {physical_index}: {e}") from e
        self.handles = self.m.amdsmi_get_processor_handles()
        self._by_uuid = {}

    def processes(self, g):
        try:
            return [dict(p) if isinstance(p, dict) else {"pid": p}
                    for p in self.m.amdsmi_get_gpu_process_list(self._h(g))]
        except Exception:  # noqa: BLE001
            return []

    def _h(self, g):
        return self._by_uuid.get(g.uuid) or self.handles[g.index]

    def link(self, a, b):
        m = self.m
        try:
            lt = m.amdsmi_topo_get_link_type(self._h(a), self._h(b))
            t = lt.get("type")
            xgmi = getattr(getattr(m, "AmdSmiLinkType", None), "XGMI", None)
            pcie = getattr(getattr(m, "AmdSmiLinkType", None), "PCIE", None)
            tname = "XGMI" if (t == xgmi or t == 2) else ("PCIE" if (t == pcie or t == 1) else "NONE")
            bw = None
            try:
                mm = m.amdsmi_get_minmax_bandwidth_between_processors(self._h(a), self._h(b))
                bw = mm.get("max_bandwidth", 0) / 1000.0 or None   # MB/s -> GB/s
            except Exception:  # noqa: BLE001
                pass
            return LinkInfo(tname, int(lt.get("hops", 1) or 1), 1, bw)
        except Exception:  # noqa: BLE001
            return LinkInfo("NONE", 0, 0)

    def health(self, g):
        if "ecc" in getattr(self, "skip_checks", set()):
            return True, ""
        try:
            ecc = self.m.amdsmi_get_gpu_total_ecc_count(self._h(g))
            if ecc.get("uncorrectable_count", 0):
                return False, f"{ecc['uncorrectable_count']} uncorrectable ECC errors"
        except Exception:  # noqa: BLE001 -- RAS not supported: treat as healthy
            pass
        return True, ""

    def memory_used_mib(self, g):
        try:
            return int(self.m.amdsmi_get_gpu_memory_usage(self._h(g), self.m.AmdSmiMemoryType.VRAM)) >> 20
        except Exception:  # noqa: BLE001
            return 0

    def utilization(self, g):
        try:
            a = self.m.amdsmi_get_gpu_activity(self._h(g))
            return {"gfx": float(a.get("gfx_activity") or 0), "umc": float(a.get("umc_activity") or 0)}
        except Exception:  # noqa: BLE001
            return {"gfx": 0.0, "umc": 0.0}

    def processes(self, g):
        try:
            return list(self.m.amdsmi_get_gpu_process_list(self._h(g)))
        except Exception:  # noqa: BLE001
            return []

    def shutdown(self):
        try:
            self.m.amdsmi_shut_down()
        except Exception:  # noqa: BLE001
            pass


KFD_TOPO = Path("/sys/class/kfd/kfd/topology/nodes")


def _kfd_props(node: Path) -> dict:
    out = {}
    try:
        for line in (node / "properties").read_text().splitlines():
            parts = line.split()
            if len(parts) == 2:
                try:
                    out[parts[0]] = int(parts[1])
                except ValueError:
                    pass
    except OSError:
        pass
    return out


def _rocr_id_from_kfd(node_id) -> str | None:
    if node_id is None:
        return None
    p = _kfd_props(KFD_TOPO / str(node_id))
    uid = p.get("unique_id")
    return f"GPU-{uid:016x}" if uid else None


# --------------------------------------------------------------------- sysfs
class SysfsBackend(Backend):
    """KFD topology only: GPUs are nodes with simd_count > 0."""
    name = "sysfs"

    def __init__(self, root: Path = KFD_TOPO):
        self.root = root
        if not root.exists():
            raise RuntimeError(f"{root} not present")

    def gpus(self):
        out = []
        nodes = sorted((p for p in self.root.iterdir() if p.name.isdigit()), key=lambda p: int(p.name))
        for n in nodes:
            p = _kfd_props(n)
            if not p.get("simd_count"):
                continue
            uid = p.get("unique_id", 0)
            cus = p.get("simd_count", 0) // max(1, p.get("simd_per_cu", 4))
            mem = 0
            for b in (n / "mem_banks").glob("*"):
                mp = _kfd_props(b)
                mem += mp.get("size_in_bytes", 0)
            idx = len(out)
            out.append(GPUInfo(index=idx, uuid=f"GPU-{uid:016x}" if uid else f"kfd-{n.name}",
                               rocr_id=f"GPU-{uid:016x}" if uid else str(idx), memory_mib=mem >> 20, cus=cus,
                               numa=max(0, p.get("cpu_core_id_base", 0) and 0), render_minor=p.get("drm_render_minor", -1)))
        return out

    def link(self, a, b):
        return LinkInfo("XGMI", 1, 1)

    def set_compute_partition(self, physical_index: int, mode: str) -> None:
        mode = mode.upper()
        if mode not in PARTITION_MODES:
            raise PartitionError(f"unknown compute partition {mode}")
        cards = sorted(Path("/sys/class/drm").glob("card*/device/current_compute_partition"))
        if physical_index >= len(cards):
            raise PartitionError(f"no compute-partition sysfs node for GPU {physical_index}")
        try:
            cards[physical_index].write_text(mode + "\n")
        except OSError as e:
            raise PartitionError(f"write {cards[physical_index]}: {e}") from e


# ---------------------------------------------------------------------- fake
class FakeBackend(Backend):
    name = "fake"

    def __init__(self, n: int = 8, prefix: str = "GPU", memory_mib: int = 294912, cus: int = 256,
                 degraded: dict | None = None, unhealthy: set | None = None, numa_per: int = 4):
        self.n, self.prefix, self.memory_mib, self.cus = n, prefix, memory_mib, cus
        self.degraded = degraded or {}
        self.unhealthy = set(unhealthy or ())
        self.numa_per = numa_per
        self.used: dict[str, int] = {}
        self.util: dict[str, dict] = {}
        self.modes: dict[int, str] = {i: "SPX" for i in range(n)}
        self.procs: dict[str, list] = {}
        self.partition_calls: list[tuple[int, str]] = []

    def gpus(self):
        out = []
        for i in range(self.n):
            mode = self.modes.get(i, "SPX")
            parts = PARTITION_MODES[mode]
            for j in range(parts):
                uid = f"{self.prefix}-{i:04x}" if parts == 1 else f"{self.prefix}-{i:04x}-{mode.lower()}{j}"
                k = len(out)
                out.append(GPUInfo(index=k, uuid=uid, rocr_id=uid, memory_mib=self.memory_mib // parts,
                                   cus=self.cus // parts, xcds=8 // parts,
                                   numa=i // self.numa_per if self.numa_per else 0,
                                   bdf=f"0000:{0x11 + i:02x}:00.{j}", render_minor=128 + k, card_minor=k,
                                   compute_partition=mode, physical_index=i, partition_index=j))
        return out

    def processes(self, g):
        return list(self.procs.get(g.uuid, []))

    def set_compute_partition(self, physical_index: int, mode: str) -> None:
        mode = mode.upper()
        if mode not in PARTITION_MODES:
            raise PartitionError(f"unknown compute partition {mode}")
        if physical_index not in self.modes:
            raise PartitionError(f"no physical GPU {physical_index}")
        if any(self.procs.get(g.uuid) for g in self.gpus() if g.physical == physical_index):
            raise PartitionError(f"GPU {physical_index} busy")
        self.partition_calls.append((physical_index, mode))
        self.modes[physical_index] = mode

    def link(self, a, b):
        if a.physical == b.physical:
            return LinkInfo("XGMI", 0, 8)          # partitions of one package: on-die
        key = tuple(sorted((a.physical, b.physical)))
        if key in self.degraded:
            return LinkInfo("XGMI", 1, 1, self.degraded[key])
        return LinkInfo("XGMI", 1, 1)

    def health(self, g):
        if g.uuid in self.unhealthy:
            return False, "injected fault"
        return True, ""

    def memory_used_mib(self, g):
        return self.used.get(g.uuid, 0)

    def utilization(self, g):
        return self.util.get(g.uuid, {"gfx": 0.0, "umc": 0.0})


def detect(prefer: str | None = None) -> Backend:
    prefer = prefer or os.environ.get("MIVGPU_SMI_BACKEND")
    if prefer == "fake":
        return FakeBackend(int(os.environ.get("MIVGPU_FAKE_GPUS", "8")))
    errors = []
    for cls in (AmdSmiBackend, SysfsBackend):
        if prefer and cls.name != prefer:
            continue
        try:
            return cls()
        except Exception as e:  # noqa: BLE001
            errors.append(f"{cls.name}: {e}")
    raise RuntimeError("no GPU discovery backend available: " + "; ".join(errors))


_SAN = re.compile(r"[^A-Za-z0-9 ._-]")


def sanitize_type(name: str) -> str:
    """Device type string safe for the comma/colon separated annotations."""
    return _SAN.sub("", name).strip() or "AMD GPU"
