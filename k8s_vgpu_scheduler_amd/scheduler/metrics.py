"""Scheduler Prometheus collector on :9395 (cmd/scheduler/metrics.go:58-429).

Same series names and label sets as the reference so the HAMi Grafana
dashboard works unchanged; every series carries ``zone="vGPU"``.  AMD core
values are normalised from CU counts to the 0..100 ratio unit
(``normalizeAMDCoreMetrics``, metrics.go:58-65).  ``--legacy-metrics`` adds the
pre-rename series.
"""

from __future__ import annotations

import math
import platform

from prometheus_client.core import GaugeMetricFamily

from k8s_vgpu_scheduler_amd import __version__

NORMALIZED_CORE_LIMIT = 100.0
ZONE = "vGPU"


def mib_to_bytes(m) -> float:
    return float(m) * 1024 * 1024


def normalize_amd_core(device_type: str, total: int, allocated: int) -> tuple[float, float]:
    if not device_type.upper().startswith("AMD") or total <= 0:
        return float(total), float(allocated)
    return NORMALIZED_CORE_LIMIT, math.ceil(allocated / total * NORMALIZED_CORE_LIMIT)


def _g(name, doc, labels):
    return GaugeMetricFamily(name, doc, labels=list(labels) + ["zone"])


class SchedulerCollector:
    def __init__(self, scheduler, legacy: bool = False):
        self.s = scheduler
        self.legacy = legacy

    def collect(self):
        nu = self.s.inspect_all_nodes_usage()
        dl = ["node", "device_uuid", "device_index", "device_type"]
        mem_limit = _g("hami_gpu_memory_limit_bytes", "Device memory limit for a certain GPU", dl)
        core_limit = _g("hami_gpu_core_limit_ratio", "Device core limit for a certain GPU", dl)
        mem_alloc = _g("hami_gpu_memory_allocated_bytes", "Device memory allocated for a certain GPU",
                       ["node", "device_uuid", "device_index", "device_cores", "device_type"])
        shared = _g("hami_gpu_shared_count", "Number of containers sharing this GPU", dl)
        core_alloc = _g("hami_gpu_core_allocated_ratio", "Device core allocated for a certain GPU", dl)
        overview = _g("hami_node_gpu_overview", "GPU overview on a certain node",
                      ["node", "device_uuid", "device_index", "device_cores", "device_memory_limit", "device_type"])
        mem_pct = _g("hami_node_gpu_memory_allocated_ratio", "GPU memory allocated ratio on a certain node", dl)
        # MI355X counterpart of hami_node_gpu_mig_instance_info: one series per
        # compute-partition device (mode dpx/qpx/cpx), value = its CU count
        part = _g("hami_node_gpu_partition_info", "Compute-partition devices (SPX/DPX/QPX/CPX) on a node",
                  ["node", "device_uuid", "device_index", "mode", "device_type"])
        # the reference's name and labels for the same rows (cmd/scheduler/metrics.go:142-146), so
        # HAMi dashboards keep working: mig_uuid = the partition device, profile = its mode,
        # placement = its CU count
        mig = _g("hami_node_gpu_mig_instance_info", "Realized MIG instance identity and scheduler placement "
                 "(MI355X: compute-partition devices)",
                 ["node", "device_uuid", "device_index", "mig_uuid", "profile", "gpu_instance_id",
                  "compute_instance_id", "placement_start", "placement_size"])
        legacy = []
        if self.legacy:
            ll = ["nodeid", "deviceuuid", "deviceidx", "devicetype"]
            l_mem = _g("GPUDeviceMemoryLimit", "legacy", ll)
            l_core = _g("GPUDeviceCoreLimit", "legacy", ll)
            l_shared = _g("GPUDeviceSharedNum", "legacy", ll)
            legacy = [l_mem, l_core, l_shared]
        for node_id, usage in nu.items():
            for d in (x.device for x in usage.devices.device_lists):
                idx = str(d.index)
                climit, calloc = normalize_amd_core(d.type, d.totalcore, d.usedcores)
                mem_limit.add_metric([node_id, d.id, idx, d.type, ZONE], mib_to_bytes(d.totalmem))
                core_limit.add_metric([node_id, d.id, idx, d.type, ZONE], climit)
                mem_alloc.add_metric([node_id, d.id, idx, str(d.totalcore), d.type, ZONE], mib_to_bytes(d.usedmem))
                shared.add_metric([node_id, d.id, idx, d.type, ZONE], float(d.used))
                core_alloc.add_metric([node_id, d.id, idx, d.type, ZONE], calloc)
                overview.add_metric([node_id, d.id, idx, str(d.totalcore), str(d.totalmem), d.type, ZONE],
                                    mib_to_bytes(d.usedmem))
                if d.totalmem > 0:
                    mem_pct.add_metric([node_id, d.id, idx, d.type, ZONE], d.usedmem / d.totalmem)
                if d.mode and d.mode != "hami-core":
                    part.add_metric([node_id, d.id, idx, d.mode, d.type, ZONE], float(d.totalcore))
                    mig.add_metric([node_id, d.id, idx, d.id, d.mode, idx, "0", "0", str(d.totalcore), ZONE], 1.0)
                if self.legacy:
                    legacy[0].add_metric([node_id, d.id, idx, d.type, ZONE], mib_to_bytes(d.totalmem))
                    legacy[1].add_metric([node_id, d.id, idx, d.type, ZONE], float(d.totalcore))
                    legacy[2].add_metric([node_id, d.id, idx, d.type, ZONE], float(d.used))
        yield from (mem_limit, core_limit, mem_alloc, shared, core_alloc, overview, mem_pct, part, mig, *legacy)

        q_used = _g("hami_resource_quota_used", "resource quota used", ["namespace", "quota_name", "limit"])
        q_limit = _g("hami_resource_quota_limit", "resource quota limit", ["namespace", "quota_name"])
        for ns, dq in self.s.quota_manager.get_resource_quota().items():
            for name, q in dq.items():
                if not q.limit_set:
                    continue
                q_used.add_metric([ns, name, str(q.limit), ZONE], float(q.used))
                q_limit.add_metric([ns, name, ZONE], float(q.limit))
        yield q_used
        yield q_limit

        c_mem = _g("hami_vgpu_memory_allocated_bytes", "vGPU memory allocated from a container",
                   ["namespace", "node", "pod", "container_index", "device_uuid"])
        c_core = _g("hami_vgpu_core_allocated_ratio", "vGPU core allocated from a container",
                    ["namespace", "node", "pod", "container_index", "device_uuid"])
        dev_index = {}
        for usage in nu.values():
            for x in usage.devices.device_lists:
                dev_index[x.device.id] = x.device
        for pi in self.s.pod_manager.get_scheduled_pods().values():
            for single in pi.devices.values():
                for cidx, ctr in enumerate(single):
                    for cd in ctr:
                        if not cd.uuid:
                            continue
                        labels = [pi.namespace, pi.node_id, pi.name, str(cidx), cd.uuid, ZONE]
                        c_mem.add_metric(labels, mib_to_bytes(cd.usedmem))
                        d = dev_index.get(cd.uuid)
                        _, ca = normalize_amd_core(d.type if d else "", d.totalcore if d else 0, cd.usedcores)
                        c_core.add_metric(labels, ca)
        yield c_mem
        yield c_core

        bi = GaugeMetricFamily("hami_build_info", "build metadata exposed as labels with a constant value of 1",
                               labels=["version", "revision", "build_date", "python_version", "compiler",
                                       "platform", "zone"])
        bi.add_metric([__version__, "", "", platform.python_version(), "cpython",
                       f"{platform.system().lower()}/{platform.machine()}", ZONE], 1.0)
        yield bi
