"""Device data model shared by scheduler, webhook and device plugin.

Field-for-field capability match of pkg/device/devices.go:106-252
(``DeviceInfo``, ``DeviceUsage``, ``ContainerDevice``, ``ContainerDeviceRequest``,
``PodDevices`` ...), with the JSON tags of the node-registration wire format
kept identical so a registration annotation written by either implementation
decodes in the other.  MIG-only fields are dropped (no MIG on MI355X; its
analogue, CPX/NPS compute partitions, is reported via ``mode``).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any

from k8s_vgpu_scheduler_amd.utils.jcopy import jcopy

# Mode string of a device shared by libmivgpu time/CU slicing (the AMD analogue
# of the reference's "hami-core" mode, nvidia/device.go:62).
MODE_SHARED = "hami-core"


@dataclass
class DeviceInfo:
    """One physical GPU as registered by the device plugin (node annotation)."""
    id: str = ""
    index: int = 0
    count: int = 0          # schedulable slots (device-split-count)
    devmem: int = 0         # MiB
    devcore: int = 0        # total cores; for AMD = CU count (MI355X: 256)
    type: str = ""
    numa: int = 0
    mode: str = ""
    health: bool = False
    devicevendor: str = ""
    custominfo: dict = field(default_factory=dict)
    # xGMI pair scores: peer uuid -> score (own annotation, never in the payload)
    pair_scores: dict = field(default_factory=dict)

    def to_json(self) -> dict:
        """Same keys and omitempty behaviour as Go's `json:"...,omitempty"`."""
        d: dict[str, Any] = {}
        for k in ("id", "index", "count", "devmem", "devcore", "type", "numa", "mode", "health"):
            v = getattr(self, k)
            if v not in (0, "", False, None):
                d[k] = v
        return d

    @classmethod
    def from_json(cls, d: dict) -> "DeviceInfo":
        return cls(id=d.get("id", ""), index=int(d.get("index", 0) or 0), count=int(d.get("count", 0) or 0),
                   devmem=int(d.get("devmem", 0) or 0), devcore=int(d.get("devcore", 0) or 0),
                   type=d.get("type", ""), numa=int(d.get("numa", 0) or 0), mode=d.get("mode", ""),
                   health=bool(d.get("health", False)), devicevendor=d.get("devicevendor", ""),
                   custominfo=dict(d.get("custominfo") or {}))

    def deepcopy(self) -> "DeviceInfo":
        return DeviceInfo(self.id, self.index, self.count, self.devmem, self.devcore, self.type, self.numa,
                          self.mode, self.health, self.devicevendor, jcopy(self.custominfo),
                          jcopy(self.pair_scores))


@dataclass
class PodInfoRef:
    namespace: str
    name: str
    uid: str


@dataclass
class DeviceUsage:
    """Scheduling view of one GPU: capacity plus what cached pods consume."""
    id: str = ""
    index: int = 0
    used: int = 0
    count: int = 0
    usedmem: int = 0
    totalmem: int = 0
    totalcore: int = 0
    usedcores: int = 0
    mode: str = ""
    numa: int = 0
    type: str = ""
    health: bool = True
    pod_infos: list = field(default_factory=list)
    custominfo: dict = field(default_factory=dict)

    def deepcopy(self) -> "DeviceUsage":
        return DeviceUsage(id=self.id, index=self.index, used=self.used, count=self.count,
                           usedmem=self.usedmem, totalmem=self.totalmem, totalcore=self.totalcore,
                           usedcores=self.usedcores, mode=self.mode, numa=self.numa, type=self.type,
                           health=self.health, pod_infos=list(self.pod_infos),
                           # values are replaced, never mutated in place (pair
                           # scores, the cu_used bitmap): a shallow copy suffices
                           custominfo=dict(self.custominfo))


@dataclass
class ContainerDevice:
    idx: int = 0
    uuid: str = ""
    type: str = ""
    usedmem: int = 0
    usedcores: int = 0
    slots: int = 0          # collapsed entries: concurrent tasks represented (0 == 1)
    custominfo: dict = field(default_factory=dict)

    def deepcopy(self) -> "ContainerDevice":
        return ContainerDevice(self.idx, self.uuid, self.type, self.usedmem, self.usedcores,
                               self.slots, jcopy(self.custominfo))


@dataclass
class ContainerDeviceRequest:
    nums: int = 0
    type: str = ""
    memreq: int = 0
    mem_percentage_req: int = 101   # 101 == "unset" sentinel (nvidia/device.go:548)
    coresreq: int = 0


# Type aliases mirroring the reference's nested containers:
#   ContainerDevices = list[ContainerDevice]             (one container)
#   PodSingleDevice  = list[ContainerDevices]            (all containers, init first)
#   PodDevices       = dict[device_type, PodSingleDevice]
#   ContainerDeviceRequests = dict[device_type, ContainerDeviceRequest]
#   PodDeviceRequests = list[ContainerDeviceRequests]     (init first)


def copy_pod_devices(pd: dict | None) -> dict | None:
    if pd is None:
        return None
    return {t: [[c.deepcopy() for c in ctr] for ctr in single] for t, single in pd.items()}


@dataclass
class NodeInfo:
    id: str
    node: dict
    devices: dict = field(default_factory=dict)   # vendor -> list[DeviceInfo]

    def deepcopy(self) -> "NodeInfo":
        # The node object is replaced wholesale on every informer update and is
        # never mutated in place, so snapshots share it; only the device
        # records (whose usage fields the scorer updates) are copied.
        return NodeInfo(self.id, self.node, {k: [d.deepcopy() for d in v] for k, v in self.devices.items()})


@dataclass
class ResourceNames:
    count: str = ""
    memory: str = ""
    core: str = ""
    memory_factor: int = 0
