"""vGPU monitor Prometheus collector on :9394 (cmd/vGPUmonitor/metrics.go:57-617).

Host series come from amd-smi (the NVML replacement), container series from
the shim's shared regions; names and labels match the reference so the HAMi
dashboards keep working.  MI355X extras: governor busy/throttled time, CU
mask size and partition identity per container, active tenants per GPU from
KFD wave occupancy.  ``legacy=True`` also emits the pre-2.x series names
(cmd/vGPUmonitor/metrics.go:133-212, ``--legacy-metrics``).

Container utilisation (``hami_container_device_utilization_ratio``) is the
GPU share the container's processes received -- their share of the resident
wavefronts, integrated by the shim (``util_pct``) or, when no shim process
reports one, sampled by the monitor itself from KFD (monitor/occupancy.py).
"""

from __future__ import annotations

import time

from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily

from .occupancy import gpu_ids_by_bdf, norm_bdf

CTR_LABELS = ["namespace", "pod", "container", "vdevice_index", "device_uuid"]
LEGACY_CTR_LABELS = ["podnamespace", "podname", "ctrname", "vdeviceid", "deviceuuid"]
LEGACY_HOST_LABELS = ["nodeid", "deviceidx", "deviceuuid", "devicetype"]


class MonitorCollector:
    def __init__(self, lister, backend=None, node_name: str = "", occupancy=None, legacy: bool = False,
                 truth=None, escalation=None, board=None):
        self.lister = lister
        self.board = board        # monitor.board.BoardSampler (the node share-board sampler) or None
        self.truth = truth        # monitor.hosttruth.HostTruth (host-truth HBM usage) or None
        self.escalation = escalation   # monitor.escalate.OverGrantPolicy or None
        self.backend = backend
        self.node = node_name
        self.occ = occupancy      # monitor.occupancy.OccupancySampler (hostPID view) or None
        self.legacy = legacy
        self._gpu_ids: dict[str, int] | None = None

    def _gpu_id(self, g) -> int | None:
        """The KFD gpu_id of backend GPU ``g``: host truth's uuid map when the
        monitor runs one (KFD unique_id first, hosttruth.GpuIdMap), else the
        normalised PCI location."""
        if self.occ is None or g is None:
            return None
        m = getattr(self.truth, "gpu_ids", None) if self.truth is not None else None
        if m is not None and hasattr(m, "ensure"):
            gid = m.ensure([g.uuid]).get(g.uuid)
            if gid is not None:
                return gid
        bdf = norm_bdf(getattr(g, "bdf", ""))
        if not bdf:
            return None
        if self._gpu_ids is None or bdf not in self._gpu_ids:
            self._gpu_ids = gpu_ids_by_bdf(self.occ.root)
        return self._gpu_ids.get(bdf)

    def collect(self):
        host_mem = GaugeMetricFamily("hami_host_gpu_memory_used_bytes", "GPU device memory usage in bytes",
                                     labels=["node", "device_index", "device_uuid", "device_type"])
        host_util = GaugeMetricFamily("hami_host_gpu_utilization_ratio", "GPU core utilization ratio (0-100)",
                                      labels=["node", "device_index", "device_uuid", "device_type"])
        host_mc = GaugeMetricFamily("hami_host_gpu_memory_controller_utilization_ratio",
                                    "GPU memory controller utilization ratio (0-100)",
                                    labels=["device_index", "device_uuid", "device_type"])
        tenants = GaugeMetricFamily("mivgpu_host_gpu_active_tenants",
                                    "Processes with wavefronts resident on the GPU in the sampling window "
                                    "(KFD cu_occupancy)", labels=["node", "device_index", "device_uuid"])
        l_mem = GaugeMetricFamily("HostGPUMemoryUsage", "GPU device memory usage", labels=LEGACY_HOST_LABELS)
        l_util = GaugeMetricFamily("HostCoreUtilization", "GPU core utilization", labels=LEGACY_HOST_LABELS)
        gpus = {}
        if self.backend is not None:
            for g in self.backend.gpus():
                gpus[g.uuid] = g
                gid = self._gpu_id(g)
                n = self.occ.active_tenants(gid) if gid is not None else None
                if n is not None:
                    tenants.add_metric([self.node, str(g.index), g.uuid], float(n))
                u = self.backend.utilization(g)
                mem_b = float(self.backend.memory_used_mib(g)) * 1024 * 1024
                host_mem.add_metric([self.node, str(g.index), g.uuid, g.name], mem_b)
                host_util.add_metric([self.node, str(g.index), g.uuid, g.name], float(u.get("gfx", 0)))
                host_mc.add_metric([str(g.index), g.uuid, g.name], float(u.get("umc", 0)))
                if self.legacy:
                    l_mem.add_metric([self.node, str(g.index), g.uuid, g.name], mem_b)
                    l_util.add_metric([self.node, str(g.index), g.uuid, g.name], float(u.get("gfx", 0)))
        yield from (host_mem, host_util, host_mc, tenants)
        if self.legacy:
            yield from (l_mem, l_util)

        used = GaugeMetricFamily("hami_vgpu_memory_used_bytes", "vGPU device memory usage in bytes", labels=CTR_LABELS)
        limit = GaugeMetricFamily("hami_vgpu_memory_limit_bytes", "vGPU device memory limit in bytes",
                                  labels=CTR_LABELS)
        dmem = GaugeMetricFamily("hami_container_device_memory_bytes", "Container device memory usage in bytes",
                                 labels=CTR_LABELS)
        dutil = GaugeMetricFamily("hami_container_device_utilization_ratio",
                                  "Container device compute utilization ratio", labels=CTR_LABELS)
        lastk = GaugeMetricFamily("hami_container_last_kernel_elapsed_seconds",
                                  "Seconds since last kernel execution in container", labels=CTR_LABELS)
        ctx = GaugeMetricFamily("hami_vgpu_memory_context_bytes", "Container device memory context size in bytes",
                                labels=CTR_LABELS)
        mod = GaugeMetricFamily("hami_vgpu_memory_module_bytes", "Container device memory module size in bytes",
                                labels=CTR_LABELS)
        buf = GaugeMetricFamily("hami_vgpu_memory_buffer_bytes", "Container device memory buffer size in bytes",
                                labels=CTR_LABELS)
        busy = CounterMetricFamily("mivgpu_container_gpu_busy_seconds", "GPU busy time measured by the governor",
                                   labels=CTR_LABELS)
        held = CounterMetricFamily("mivgpu_container_throttled_seconds",
                                   "Time the governor held the container's streams", labels=CTR_LABELS)
        cumask = GaugeMetricFamily("mivgpu_container_cu_mask_cus", "CUs granted through HSA_CU_MASK",
                                   labels=CTR_LABELS)
        share = GaugeMetricFamily("mivgpu_container_gpu_share_ratio",
                                  "Governor's measured GPU share of the container while contending (percent of "
                                  "the resident wavefronts, KFD occupancy), summed over its processes",
                                  labels=CTR_LABELS)
        occw = GaugeMetricFamily("mivgpu_container_wave_occupancy",
                                 "Last KFD cu_occupancy sample of the container's processes (CU units)",
                                 labels=CTR_LABELS)
        part = GaugeMetricFamily("mivgpu_container_partition_info",
                                 "Compute-partition identity of a container allocation (the MI355X analogue "
                                 "of hami_mig_device_info)",
                                 labels=CTR_LABELS + ["compute_partition", "memory_partition", "partition_index",
                                                      "physical_index", "cus"])
        # the reference's series name and labels for the same identity, so HAMi
        # dashboards built on hami_mig_device_info keep working
        # (cmd/vGPUmonitor/metrics.go:102-106): mig_uuid = the partition
        # device, profile = <mode>.<CUs>cu, gpu instance = partition index
        mig = GaugeMetricFamily("hami_mig_device_info", "MIG runtime identity for a container allocation "
                                "(MI355X: compute-partition identity)",
                                labels=CTR_LABELS + ["mig_uuid", "profile", "gpu_instance_id", "compute_instance_id"])
        host_b = GaugeMetricFamily("mivgpu_container_memory_host_bytes",
                                   "Container device memory from host truth (KFD per-process VRAM of the pod's "
                                   "processes), independent of the tenant-writable shared region",
                                   labels=CTR_LABELS)
        over_g = GaugeMetricFamily("mivgpu_container_memory_over_grant",
                                   "1 while the container's host-truth HBM exceeds its grant (launches blocked)",
                                   labels=CTR_LABELS)
        shim = GaugeMetricFamily("mivgpu_container_shim_loaded",
                                 "0 while a granted container holds HBM on its GPU with no process under "
                                 "libmivgpu.so (host truth; enforced from KFD alone), else 1", labels=CTR_LABELS)
        st = self.truth.state() if self.truth is not None else {"truth": {}, "over": set(), "no_shim": set(),
                                                                  "grants": {}}
        truth, over, no_shim = st["truth"], st["over"], st["no_shim"]
        l_used = GaugeMetricFamily("vGPU_device_memory_usage_in_bytes", "vGPU device usage", labels=LEGACY_CTR_LABELS)
        l_limit = GaugeMetricFamily("vGPU_device_memory_limit_in_bytes", "vGPU device limit",
                                    labels=LEGACY_CTR_LABELS)
        l_desc = GaugeMetricFamily("Device_memory_desc_of_container", "Container device memory description",
                                   labels=LEGACY_CTR_LABELS + ["context", "module", "data", "offset"])
        l_cutil = GaugeMetricFamily("Device_utilization_desc_of_container",
                                    "Container device utilization description", labels=LEGACY_CTR_LABELS)
        l_lastk = GaugeMetricFamily("Device_last_kernel_of_container", "Container device last kernel description",
                                    labels=LEGACY_CTR_LABELS)
        now = time.time()
        seen = set()
        for c in self.lister.list_containers():
            seen.add((c.pod_uid, c.container))
            r = c.region
            r.refresh()
            for i in range(r.device_num()):
                if not r.is_valid_uuid(i):
                    continue
                lab = [c.namespace, c.pod_name, c.container, str(i), r.uuid(i)]
                total = r.memory_total(i)
                used.add_metric(lab, float(total))
                dmem.add_metric(lab, float(total))
                limit.add_metric(lab, float(r.memory_limit(i)))
                ctx.add_metric(lab, float(r.memory_field(i, "context")))
                mod.add_metric(lab, float(r.memory_field(i, "module")))
                buf.add_metric(lab, float(r.memory_field(i, "buffer") + r.memory_field(i, "vmm")))
                util = float(self._container_util(r, i, gpus.get(r.uuid(i))))
                dutil.add_metric(lab, util)
                lkt = r.last_kernel_time()
                if lkt > 0:
                    lastk.add_metric(lab, max(0.0, now - lkt))
                g = gpus.get(r.uuid(i))
                if g is not None:
                    part.add_metric(lab + [g.compute_partition, g.memory_partition, str(g.partition_index),
                                           str(g.physical), str(g.cus)], 1.0)
                    if str(g.compute_partition).upper() != "SPX":
                        mig.add_metric(lab + [r.uuid(i), f"{str(g.compute_partition).lower()}.{g.cus}cu",
                                              str(g.partition_index), "0"], 1.0)
                if self.legacy:
                    ctx_b, mod_b = r.memory_field(i, "context"), r.memory_field(i, "module")
                    data_b = r.memory_field(i, "buffer") + r.memory_field(i, "vmm")
                    l_used.add_metric(lab, float(total))
                    l_limit.add_metric(lab, float(r.memory_limit(i)))
                    l_desc.add_metric(lab + [str(ctx_b), str(mod_b), str(data_b),
                                             str(max(0, total - ctx_b - mod_b - data_b))], float(total))
                    l_cutil.add_metric(lab, util)
                    if lkt > 0:
                        l_lastk.add_metric(lab, max(0.0, now - lkt))
                busy.add_metric(lab, r.busy_ns(i) / 1e9)
                held.add_metric(lab, sum(p.util[i].throttled_ns for p in r.active_procs()) / 1e9)
                cumask.add_metric(lab, float(r.r.cu_mask_count[i]))
                procs = r.active_procs()
                if any(p.util[i].share_ppm for p in procs):
                    share.add_metric(lab, min(100.0, sum(p.util[i].share_ppm for p in procs) / 1e4))
                occw.add_metric(lab, float(sum(p.util[i].occupancy for p in procs)))
                tb = truth.get((c.pod_uid, c.container, i))
                if tb is not None:
                    host_b.add_metric(lab, float(tb))
                    over_g.add_metric(lab, 1.0 if (c.pod_uid, c.container) in over else 0.0)
                    shim.add_metric(lab, 0.0 if (c.pod_uid, c.container) in no_shim else 1.0)
        # granted containers without a shared region (no shim ever started in
        # them, or the region was removed): the host-truth rows alone
        for g in st["grants"].values():
            if (g.pod_uid, g.container) in seen:
                continue
            md = (self.lister.pod(g.pod_uid) or {}).get("metadata") or {}
            for i, u in enumerate(g.uuids):
                tb = truth.get((g.pod_uid, g.container, i))
                if tb is None:
                    continue
                lab = [md.get("namespace", ""), md.get("name", ""), g.container, str(i), u]
                host_b.add_metric(lab, float(tb))
                limit.add_metric(lab, float(g.mem[i] if i < len(g.mem) else 0))
                over_g.add_metric(lab, 1.0 if (g.pod_uid, g.container) in over else 0.0)
                shim.add_metric(lab, 0.0 if (g.pod_uid, g.container) in no_shim else 1.0)
        yield from (used, limit, dmem, dutil, lastk, ctx, mod, buf, busy, held, cumask, part, mig, share, occw)
        if self.truth is not None:
            yield from (host_b, over_g, shim)
        if self.escalation is not None:
            acts = CounterMetricFamily("mivgpu_over_grant_actions", "Over-grant escalations taken (evict / kill)",
                                       labels=["node", "action"])
            for a, n in self.escalation.actions.items():
                if a != "block":
                    acts.add_metric([self.node, a], float(n))
            yield acts
        if self.board is not None:
            up = GaugeMetricFamily("mivgpu_board_sampler_up",
                                   "1 while the node share-board sampler (mivgpu-boardd) runs", labels=["node"])
            up.add_metric([self.node], 1.0 if self.board.alive() else 0.0)
            rs = CounterMetricFamily("mivgpu_board_sampler_restarts", "Times the monitor restarted mivgpu-boardd",
                                     labels=["node"])
            rs.add_metric([self.node], float(getattr(self.board, "restarts", 0)))
            yield from (up, rs)
        if self.legacy:
            yield from (l_used, l_limit, l_desc, l_cutil, l_lastk)

    def _container_util(self, r, i: int, g) -> float:
        """Percent of the GPU the container's processes received: the shims'
        own occupancy integral when any reports one, else the monitor's KFD
        sample of the processes' host pids."""
        procs = r.active_procs()
        if any(p.util[i].share_ns for p in procs):
            return float(min(100, sum(p.util[i].util_pct for p in procs)))
        gid = self._gpu_id(g)
        pids = [p.hostpid for p in procs if p.hostpid > 0]
        if gid is None or not pids:
            return 0.0
        v = self.occ.share_pct(gid, pids)
        return round(v, 1) if v is not None else 0.0
