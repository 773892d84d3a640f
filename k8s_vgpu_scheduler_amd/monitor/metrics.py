"""vGPU monitor Prometheus collector on :9394 (cmd/vGPUmonitor/metrics.go:57-617).

Host series come from amd-smi (the NVML replacement), container series from
the shim's shared regions; names and labels match the reference so the HAMi
dashboards keep working.  MI355X extras: governor busy/throttled time and CU
mask size per container.
"""

from __future__ import annotations

import time

from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily

from .board import active_tenants, board_path

CTR_LABELS = ["namespace", "pod", "container", "vdevice_index", "device_uuid"]


class MonitorCollector:
    def __init__(self, lister, backend=None, node_name: str = ""):
        self.lister = lister
        self.backend = backend
        self.node = node_name

    def collect(self):
        host_mem = GaugeMetricFamily("hami_host_gpu_memory_used_bytes", "GPU device memory usage in bytes",
                                     labels=["node", "device_index", "device_uuid", "device_type"])
        host_util = GaugeMetricFamily("hami_host_gpu_utilization_ratio", "GPU core utilization ratio (0-100)",
                                      labels=["node", "device_index", "device_uuid", "device_type"])
        host_mc = GaugeMetricFamily("hami_host_gpu_memory_controller_utilization_ratio",
                                    "GPU memory controller utilization ratio (0-100)",
                                    labels=["device_index", "device_uuid", "device_type"])
        tenants = GaugeMetricFamily("mivgpu_host_gpu_active_tenants",
                                    "Shimmed processes that launched work on the GPU in the last second "
                                    "(the governor's share board)", labels=["node", "device_index", "device_uuid"])
        if self.backend is not None:
            for g in self.backend.gpus():
                bp = board_path(g.bdf) if g.bdf else None
                if bp is not None and bp.exists():
                    tenants.add_metric([self.node, str(g.index), g.uuid], float(active_tenants(bp)))
                u = self.backend.utilization(g)
                host_mem.add_metric([self.node, str(g.index), g.uuid, g.name],
                                    float(self.backend.memory_used_mib(g)) * 1024 * 1024)
                host_util.add_metric([self.node, str(g.index), g.uuid, g.name], float(u.get("gfx", 0)))
                host_mc.add_metric([str(g.index), g.uuid, g.name], float(u.get("umc", 0)))
        yield from (host_mem, host_util, host_mc, tenants)

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
        now = time.time()
        for c in self.lister.list_containers():
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
                util = sum(p.util[i].util_pct for p in r.active_procs())
                dutil.add_metric(lab, float(util))
                lkt = r.last_kernel_time()
                if lkt > 0:
                    lastk.add_metric(lab, max(0.0, now - lkt))
                busy.add_metric(lab, r.busy_ns(i) / 1e9)
                held.add_metric(lab, sum(p.util[i].throttled_ns for p in r.active_procs()) / 1e9)
                cumask.add_metric(lab, float(r.r.cu_mask_count[i]))
        yield from (used, limit, dmem, dutil, lastk, ctx, mod, buf, busy, held, cumask)
