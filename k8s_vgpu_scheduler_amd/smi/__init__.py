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
import threading
import time
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
    max_bw_gbps: float | None = None    # per direction; a degraded link reports less than nominal
    weight: int | None = None           # KFD io_link weight (lower = closer: xGMI 15, PCIe 20 on MI355X)


# KFD io_link types (kfd_crat.h CRAT_IOLINK_TYPE_*); measured on an 8 x MI355X
# node (scripts/probe/topology_probe.py, tests/fixtures/mi355x_8gpu_kfd_links.json):
# GPU<->GPU type 11 (xGMI), weight 15, min = max bandwidth 76000 MB/s (= the
# 608 Gb/s per link amd-smi link_metrics reports); GPU<->CPU type 2 (PCIe),
# weight 20, 64000 MB/s.
KFD_IOLINK_PCIE, KFD_IOLINK_XGMI = 2, 11


def kfd_link(root: Path, node_a: str, node_b: str) -> LinkInfo | None:
    """The io_link from KFD topology node ``node_a`` to ``node_b`` (None: none)."""
    base = root / str(node_a) / "io_links"
    try:
        entries = list(base.iterdir())
    except OSError:
        return None
    for e in entries:
        p = _kfd_props(e)
        if str(p.get("node_to")) != str(node_b):
            continue
        t = p.get("type")
        kind = "XGMI" if t == KFD_IOLINK_XGMI else ("PCIE" if t == KFD_IOLINK_PCIE else "NONE")
        bws = [v for v in (p.get("min_bandwidth"), p.get("max_bandwidth")) if v]
        return LinkInfo(kind, 1, 1, (min(bws) / 1000.0) if bws else None, p.get("weight"))   # MB/s -> GB/s
    return None


@dataclass
class HealthEvent:
    """One amd-smi event notification (the AMD analog of an NVML XID event).
    ``kind`` is the lower-case AmdSmiEvtNotificationType name; ``physical`` is
    the physical GPU index it was raised on (None: unknown device)."""
    kind: str
    physical: int | None
    message: str = ""


# kinds the device plugin subscribes to (AmdSmiEvtNotificationType names)
HEALTH_EVENT_KINDS = ("vmfault", "thermal_throttle", "gpu_pre_reset", "gpu_post_reset")


class Backend:
    name = "base"
    skip_checks: set = set()     # health checks disabled via DP_DISABLE_HEALTHCHECKS

    def wait_health_events(self, gpus: list[GPUInfo], timeout_s: float) -> list[HealthEvent] | None:
        """Block up to ``timeout_s`` for device events.  None = this backend has
        no event source (the caller sleeps and polls instead)."""
        return None

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


def _group_physical(out: list[GPUInfo]) -> list[GPUInfo]:
    """Partitions of one physical GPU share domain:bus:device and differ in
    the PCI function: number the physical GPUs and the partitions inside each."""
    phys: dict[str, int] = {}
    for g in out:
        key = g.bdf.rsplit(".", 1)[0] if g.bdf else f"idx{g.index}"
        g.partition_index = sum(1 for o in out[: g.index] if (o.bdf.rsplit(".", 1)[0] if o.bdf else "") == key)
        g.physical_index = phys.setdefault(key, len(phys))
    return out


# ------------------------------------------------------------ device identity
# One identity whatever the backend (amd-smi published
# "AMD Radeon Graphics" and its own UUID format while sysfs published the
# board name and GPU-<unique_id>, so a node falling back from one backend to
# the other changed every device id under live allocations):
#   uuid = rocr_id = "GPU-<KFD unique_id, 16 lower-case hex>", the id ROCr
#          accepts in ROCR_VISIBLE_DEVICES (docs/develop/amd-vgpu.md:174-180;
#          amd-smi reports the same value as enumeration_info.hip_uuid and,
#          on MI355X, as asic_serial);
#   name = the board's product name (amd-smi board_info.product_name = sysfs
#          product_name, "AMD Instinct MI355 OAM"), never the generic
#          "AMD Radeon Graphics" libdrm answers when its id table is missing.
GENERIC_NAMES = {"", "amd radeon graphics", "n/a", "na", "unknown"}
DEVICE_ID_NAMES = {0x75A3: "AMD Instinct MI355X", 0x75A0: "AMD Instinct MI350X", 0x74A1: "AMD Instinct MI300X",
                   0x74A5: "AMD Instinct MI325X"}


def canonical_name(*candidates, device_id: int | None = None) -> str:
    for c in candidates:
        if c and str(c).strip().lower() not in GENERIC_NAMES:
            return str(c).strip()
    return DEVICE_ID_NAMES.get(device_id or 0, "AMD Instinct MI355X")


def rocr_uuid(unique_id) -> str | None:
    """``GPU-<16 hex>`` from a KFD unique_id / asic serial (int or hex string)."""
    if unique_id in (None, "", 0, "0"):
        return None
    try:
        v = int(unique_id, 16) if isinstance(unique_id, str) else int(unique_id)
    except ValueError:
        return None
    return f"GPU-{v:016x}" if v else None


def _dedupe_partition_ids(out: list[GPUInfo]) -> list[GPUInfo]:
    """Compute partitions of one package may share the package's unique id:
    suffix ``-<mode><partition>`` (and address them by index) so every
    schedulable device keeps a distinct id."""
    seen: dict[str, int] = {}
    for g in out:
        seen[g.uuid] = seen.get(g.uuid, 0) + 1
    for g in out:
        if seen[g.uuid] > 1:
            g.uuid = f"{g.uuid}-{g.compute_partition.lower()}{g.partition_index}"
            g.rocr_id = str(g.index)
    return out


def _sysfs_product_name(bdf: str) -> str:
    try:
        return Path(f"/sys/bus/pci/devices/{bdf}/product_name").read_text().strip()
    except OSError:
        return ""


# ------------------------------------------------------------------- amd-smi
def _handle_key(h) -> int | None:
    """amd-smi processor handles come back as ctypes pointers or plain ints."""
    if h is None:
        return None
    v = getattr(h, "value", h)
    try:
        return int(v) if v is not None else None
    except (TypeError, ValueError):
        return None


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
            asic = q("amdsmi_get_gpu_asic_info", default={}) or {}
            board = q("amdsmi_get_gpu_board_info", default={}) or {}
            total = q("amdsmi_get_gpu_memory_total", m.AmdSmiMemoryType.VRAM, default=0) or 0
            numa = q("amdsmi_topo_get_numa_node_number", default=0) or 0
            bdf = q("amdsmi_get_gpu_device_bdf", default="") or ""
            enum = q("amdsmi_get_gpu_enumeration_info", default={}) or {}
            kfd = q("amdsmi_get_gpu_kfd_info", default={}) or {}
            part = q("amdsmi_get_gpu_compute_partition", default="SPX") or "SPX"
            cus = int(asic.get("num_of_compute_units") or asic.get("num_compute_units") or 256)
            rocr = (_rocr_id_from_kfd(kfd.get("node_id")) or
                    (str(enum.get("hip_uuid")).lower() if str(enum.get("hip_uuid", "")).startswith("GPU-") else None)
                    or rocr_uuid(asic.get("asic_serial")))
            uuid = rocr or str(q("amdsmi_get_gpu_device_uuid", default=f"gpu-{i}"))
            try:
                did = int(str(asic.get("device_id", "0")), 0)
            except ValueError:
                did = 0
            g = GPUInfo(index=i, uuid=uuid, rocr_id=rocr or str(i),
                        name=canonical_name(board.get("product_name"), asic.get("market_name"),
                                            _sysfs_product_name(str(bdf)), device_id=did),
                        memory_mib=int(total) // (1 << 20), cus=cus, numa=max(0, int(numa)), bdf=str(bdf),
                        render_minor=int(enum.get("drm_render", -1) if isinstance(enum.get("drm_render"), int) else -1),
                        card_minor=int(enum.get("drm_card", -1) if isinstance(enum.get("drm_card"), int) else -1),
                        compute_partition=str(part),
                        extra={"kfd_node": kfd.get("node_id"), "gpu_id": kfd.get("kfd_id")})
            out.append((g, h))
        gs = _dedupe_partition_ids(_group_physical([g for g, _ in out]))
        self._by_uuid = {g.uuid: h for g, h in zip(gs, (h for _, h in out))}
        return gs

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
        """Link type from the AmdSmiLinkType enum (PCIE = 1, XGMI = 2 in this
        amd-smi; the names are resolved, not the numbers), hops, KFD weight and
        the min/max bandwidth (MB/s, the KFD io_link unit) -- the weaker bound
        counts, so a degraded link scores lower.  Falls back to the KFD io_links
        when amd-smi cannot answer for a pair."""
        m = self.m
        enum = getattr(m, "AmdSmiLinkType", None)
        xgmi = int(getattr(enum, "AMDSMI_LINK_TYPE_XGMI", 2)) if enum is not None else 2
        pcie = int(getattr(enum, "AMDSMI_LINK_TYPE_PCIE", 1)) if enum is not None else 1
        try:
            lt = m.amdsmi_topo_get_link_type(self._h(a), self._h(b))
            t = int(lt.get("type"))
        except Exception:  # noqa: BLE001
            kl = kfd_link(KFD_TOPO, a.extra.get("kfd_node"), b.extra.get("kfd_node")) \
                if a.extra.get("kfd_node") is not None else None
            return kl or LinkInfo("NONE", 0, 0)
        tname = "XGMI" if t == xgmi else ("PCIE" if t == pcie else "NONE")
        weight = None
        try:
            weight = int(m.amdsmi_topo_get_link_weight(self._h(a), self._h(b)))
        except Exception:  # noqa: BLE001
            pass
        bw = None
        try:
            mm = m.amdsmi_get_minmax_bandwidth_between_processors(self._h(a), self._h(b))
            vals = [v for v in (mm.get("min_bandwidth"), mm.get("max_bandwidth")) if v]
            bw = min(vals) / 1000.0 if vals else None     # MB/s -> GB/s
        except Exception:  # noqa: BLE001
            pass
        return LinkInfo(tname, int(lt.get("hops", 1) or 1), 1, bw, weight)

    def wait_health_events(self, gpus, timeout_s):
        m = self.m
        if getattr(self, "_evt_handles", None) is None:
            # one registration per physical GPU (partitions share the package's events)
            self._evt_handles = {}
            mask = 0
            for k in HEALTH_EVENT_KINDS:
                mask |= 1 << (int(getattr(m.AmdSmiEvtNotificationType, k.upper())) - 1)
            for g in gpus:
                if g.physical in self._evt_handles.values():
                    continue
                h = self._h(g)
                try:
                    m.amdsmi_init_gpu_event_notification(h)
                    m.amdsmi_set_gpu_event_notification_mask(h, mask)
                    self._evt_handles[_handle_key(h)] = g.physical
                except Exception as e:  # noqa: BLE001 -- e.g. no permission on /dev/kfd events
                    log.warning("GPU %s: amd-smi event notification unavailable (%s); ECC polling only",
                                g.uuid, e)
        if not self._evt_handles:
            return None
        t0 = time.monotonic()
        try:
            res = m.amdsmi_get_gpu_event_notification(int(timeout_s * 1000))
        except Exception as e:  # noqa: BLE001
            # an idle card answers the wait with NO_DATA (measured on MI355X) or a timeout
            code = getattr(e, "get_error_code", lambda: None)()
            if "NO_DATA" in str(e) or "TIMEOUT" in str(e).upper() or code in (
                    getattr(m.amdsmi_wrapper, "AMDSMI_STATUS_NO_DATA", -1),
                    getattr(m.amdsmi_wrapper, "AMDSMI_STATUS_TIMEOUT", -1)):
                # keep the "block up to timeout_s" contract even if the answer came early
                time.sleep(max(0.0, timeout_s - (time.monotonic() - t0)))
                return []
            raise
        out = []
        names = {int(v): v.name.lower() for v in m.AmdSmiEvtNotificationType}
        for d in res.get("data", []):
            kind = names.get(int(d.get("event", 0)), "none")
            if kind == "none":
                continue
            out.append(HealthEvent(kind, self._evt_handles.get(_handle_key(d.get("processor_handle"))),
                                   str(d.get("message", ""))))
        return out

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
    """KFD topology (GPUs are nodes with simd_count > 0) joined with the DRM
    render node's PCI device for NUMA node, BDF, card minor and partition mode."""
    name = "sysfs"

    def __init__(self, root: Path = KFD_TOPO, drm: Path = Path("/sys/class/drm")):
        self.root, self.drm = root, drm
        if not root.exists():
            raise RuntimeError(f"{root} not present")

    def _pci(self, render_minor: int) -> Path | None:
        d = self.drm / f"renderD{render_minor}" / "device"
        return d if d.exists() else None

    @staticmethod
    def _read(p: Path, default: str = "") -> str:
        try:
            return p.read_text().strip()
        except OSError:
            return default

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
            minor = p.get("drm_render_minor", -1)
            numa, bdf, card, part, name = 0, "", -1, "SPX", "AMD Instinct MI355X"
            dev = self._pci(minor)
            if dev is not None:
                try:
                    numa = max(0, int(self._read(dev / "numa_node", "0") or 0))
                except ValueError:
                    numa = 0
                bdf = os.path.basename(os.path.realpath(dev))
                cards = [c.name for c in (dev / "drm").glob("card*")] if (dev / "drm").exists() else []
                card = int(cards[0][4:]) if cards and cards[0][4:].isdigit() else -1
                part = self._read(dev / "current_compute_partition", "SPX") or "SPX"
                name = canonical_name(self._read(dev / "product_name"), device_id=p.get("device_id"))
            idx = len(out)
            rid = rocr_uuid(uid)
            gid = None
            try:
                gid = int((n / "gpu_id").read_text().strip() or 0)
            except (OSError, ValueError):
                pass
            out.append(GPUInfo(index=idx, uuid=rid or f"kfd-{n.name}", rocr_id=rid or str(idx), name=name,
                               memory_mib=mem >> 20, cus=cus, numa=numa, bdf=bdf, render_minor=minor,
                               card_minor=card, compute_partition=part.upper(),
                               extra={"kfd_node": n.name, "gpu_id": gid}))
        return _dedupe_partition_ids(_group_physical(out))

    def link(self, a, b):
        """From the KFD io_links (type, weight, bandwidth); partitions of one
        package talk on-die."""
        if a.physical == b.physical and a.bdf and b.bdf:
            return LinkInfo("XGMI", 0, 8)
        kl = kfd_link(self.root, a.extra.get("kfd_node"), b.extra.get("kfd_node"))
        return kl or LinkInfo("NONE", 0, 0)

    def set_compute_partition(self, physical_index: int, mode: str) -> None:
        mode = mode.upper()
        if mode not in PARTITION_MODES:
            raise PartitionError(f"unknown compute partition {mode}")
        gs = [g for g in self.gpus() if g.physical == physical_index and g.partition_index == 0]
        dev = self._pci(gs[0].render_minor) if gs else None
        if dev is None:
            raise PartitionError(f"no compute-partition sysfs node for GPU {physical_index}")
        node = dev / "current_compute_partition"
        try:
            node.write_text(mode + "\n")
        except OSError as e:
            raise PartitionError(f"write {node}: {e}") from e


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
        self.events: list[HealthEvent] = []
        self._events_cv = threading.Condition()
        self.event_source = True

    def inject_event(self, kind: str, physical: int | None, message: str = ""):
        with self._events_cv:
            self.events.append(HealthEvent(kind, physical, message))
            self._events_cv.notify_all()

    def wait_health_events(self, gpus, timeout_s):
        if not self.event_source:
            return None
        with self._events_cv:
            if not self.events:
                self._events_cv.wait(timeout_s)
            out, self.events = self.events, []
        return out

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


class SerializedBackend:
    """Every call into the wrapped backend under one lock.  The monitor calls
    its backend from the metrics HTTP thread (every scrape) and from the
    feedback thread (host truth's uuid -> KFD gpu_id map); amd-smi's library
    does not document its calls as thread-safe, so they never overlap."""

    def __init__(self, inner):
        import threading
        self._inner = inner
        self._mu = threading.RLock()
        self.name = getattr(inner, "name", "base")

    def __getattr__(self, attr):
        v = getattr(self._inner, attr)
        if not callable(v):
            return v
        mu = self._mu

        def call(*a, **kw):
            with mu:
                return v(*a, **kw)
        return call


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
