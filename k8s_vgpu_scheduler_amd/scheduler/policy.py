"""GPU- and node-level scheduling policies.

GPU level (pkg/scheduler/policy/gpu_policy.go:77-222): devices of a node are
sorted ascending by ``less`` and backends' Fit walks the list from the END,
so "last" == most preferred.  Policies: binpack, spread, mutex, numa and
comma chains of sort keys ("binpack,numa"); topology-aware and mutex are Fit
filters, not sort keys.  Device score =
``10 * (w_slot*used/count + w_core*cores/totalcore + w_mem*mem/totalmem)``
including the pending request.

Node level (node_policy.go:48-130): node score =
``10 * (used/total + cores/totalcores + mem/totalmem)``; binpack picks the
highest, spread the lowest.  Backends flagged ``policy_neutral_score`` add
``+-10000 * ScoreNode`` (sign by policy) so device-level topology dominates.
"""

from __future__ import annotations

import functools
from dataclasses import dataclass, field

from k8s_vgpu_scheduler_amd.device import devices as D
from k8s_vgpu_scheduler_amd.device.types import DeviceUsage
from k8s_vgpu_scheduler_amd.utils import types as T
from k8s_vgpu_scheduler_amd.utils.weights import DeviceScoringWeights

_SORT_KEYS = (T.GPU_POLICY_BINPACK, T.GPU_POLICY_SPREAD, T.GPU_POLICY_NUMA)


def sort_key_chain(policy: str) -> list[str]:
    seen, chain = set(), []
    for p in (policy or "").split(","):
        p = p.strip()
        if p in _SORT_KEYS and p not in seen:
            chain.append(p)
            seen.add(p)
    return chain


@dataclass
class DeviceListsScore:
    device: DeviceUsage
    score: float = 0.0

    def compute_score(self, requests: dict, weights: DeviceScoringWeights):
        d = self.device
        if d is None or d.count == 0 or d.totalcore == 0 or d.totalmem == 0:
            self.score = 0.0
            return
        req = core = mem = 0
        for r in requests.values():
            # Only requests of this device family count (reference compares Type).
            if r.type.lower() not in d.type.lower() and r.type != d.type:
                continue
            req += 1
            core += _core_units(d, r.coresreq)
            if r.mem_percentage_req not in (0, 101):
                mem += d.totalmem * r.mem_percentage_req // 100
                continue
            mem += r.memreq
        used = (req + d.used) / d.count
        cores = (core + d.usedcores) / d.totalcore
        mems = (mem + d.usedmem) / d.totalmem
        self.score = float(T.WEIGHT) * (weights.slot * used + weights.core * cores + weights.memory * mems)


def _core_units(d: DeviceUsage, pct: int) -> int:
    """Requests are in % while AMD usage is in CUs: convert for a like-for-like score."""
    if d.totalcore > 100 and pct > 0:
        return d.totalcore * pct // 100
    return pct


@dataclass
class DeviceUsageList:
    device_lists: list = field(default_factory=list)
    policy: str = T.GPU_POLICY_SPREAD
    numa_bind: bool = False

    def less(self, a: DeviceListsScore, b: DeviceListsScore) -> bool:
        if "," in self.policy or self.policy == T.GPU_POLICY_NUMA:
            return self._less_chain(a, b)
        si, sj = a.score, b.score
        ni, nj = a.device.numa, b.device.numa
        binpack = self.policy == T.GPU_POLICY_BINPACK
        if self.policy == T.GPU_POLICY_MUTEX:
            if a.device.used != b.device.used:
                return a.device.used > b.device.used
            return ni < nj
        if self.numa_bind:
            if binpack:
                return si < sj if ni == nj else ni > nj
            return si > sj if ni == nj else ni < nj
        if binpack:
            return si < sj if si != sj else ni < nj
        return si > sj if si != sj else ni < nj

    def _less_chain(self, a, b) -> bool:
        chain = sort_key_chain(self.policy) or [T.GPU_POLICY_SPREAD]
        if self.numa_bind and chain[0] != T.GPU_POLICY_NUMA:
            chain = [T.GPU_POLICY_NUMA] + [k for k in chain if k != T.GPU_POLICY_NUMA]
        for key in chain:
            if key == T.GPU_POLICY_BINPACK and a.score != b.score:
                return a.score < b.score
            if key == T.GPU_POLICY_SPREAD and a.score != b.score:
                return a.score > b.score
            if key == T.GPU_POLICY_NUMA and a.device.numa != b.device.numa:
                return a.device.numa < b.device.numa
        return a.device.index < b.device.index

    def sort(self):
        def cmp(x, y):
            if self.less(x, y):
                return -1
            if self.less(y, x):
                return 1
            return 0
        self.device_lists.sort(key=functools.cmp_to_key(cmp))

    def deepcopy(self) -> "DeviceUsageList":
        return DeviceUsageList([DeviceListsScore(d.device.deepcopy(), d.score) for d in self.device_lists],
                               self.policy, self.numa_bind)


@dataclass
class NodeScore:
    node_id: str
    node: dict | None
    devices: dict = field(default_factory=dict)   # PodDevices
    score: float = 0.0

    def compute_default_score(self, devices: DeviceUsageList):
        used = sum(d.device.used for d in devices.device_lists)
        ucore = sum(d.device.usedcores for d in devices.device_lists)
        umem = sum(d.device.usedmem for d in devices.device_lists)
        total = sum(d.device.count for d in devices.device_lists)
        tcore = sum(d.device.totalcore for d in devices.device_lists)
        tmem = sum(d.device.totalmem for d in devices.device_lists)
        if total == 0 or tcore == 0 or tmem == 0:
            self.score = 0.0
            return
        self.score = float(T.WEIGHT) * (used / total + ucore / tcore + umem / tmem)

    @staticmethod
    def snapshot_device(devices: DeviceUsageList) -> list[DeviceUsage]:
        return [d.device.deepcopy() for d in devices.device_lists]

    def override_score(self, previous: list, policy: str):
        dev_score = 0.0
        for t, single in self.devices.items():
            dev = D.get_devices().get(t)
            if dev is None:
                continue
            s = dev.score_node(self.node, single, previous, policy)
            if getattr(dev, "policy_neutral_score", False):
                w = -10000.0 if policy == T.NODE_POLICY_SPREAD else 10000.0
                s *= w
            dev_score += s
        self.score += dev_score


@dataclass
class NodeScoreList:
    node_list: list = field(default_factory=list)
    policy: str = T.NODE_POLICY_BINPACK

    def sort(self):
        spread = self.policy == T.NODE_POLICY_SPREAD
        # ascending by Less; the best node is the LAST element
        self.node_list.sort(key=lambda n: -n.score if spread else n.score)
