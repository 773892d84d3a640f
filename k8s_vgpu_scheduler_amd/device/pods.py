"""PodManager: UID -> scheduled pod + effective device usage (pkg/device/pods.go:29-290).

Every read returns deep copies (the stored entries are rewritten in place by
informer callbacks).  ``init_released`` marks pods whose usage already shrank
to app-containers-only so an informer resync cannot re-inflate it.

Beyond the reference: a node -> pods index and a per-node generation that
moves whenever the device usage on that node changes, so the scheduler keeps
one usage view per node and rebuilds only the nodes that changed instead of
re-deriving every node from every pod on each Filter (scheduler.go:744-863
walks all pods per call).
"""

from __future__ import annotations

import itertools
import logging
import threading
from dataclasses import dataclass, field

from k8s_vgpu_scheduler_amd.utils.jcopy import jcopy

from .types import copy_pod_devices

log = logging.getLogger(__name__)


@dataclass
class PodInfo:
    pod: dict
    node_id: str
    devices: dict = field(default_factory=dict)
    init_released: bool = False

    @property
    def name(self):
        return self.pod["metadata"]["name"]

    @property
    def namespace(self):
        return self.pod["metadata"].get("namespace", "default")

    @property
    def uid(self):
        return self.pod["metadata"].get("uid", "")

    @property
    def annotations(self):
        return self.pod["metadata"].get("annotations") or {}

    def deepcopy(self) -> "PodInfo":
        # `pod` is a private copy taken in add_pod/update_pod and only ever
        # replaced, never mutated, so snapshots share it.
        return PodInfo(self.pod, self.node_id, copy_pod_devices(self.devices), self.init_released)


def _uid(pod: dict) -> str:
    md = pod.get("metadata") or {}
    return md.get("uid") or f"{md.get('namespace', 'default')}/{md.get('name')}"


_GEN = itertools.count(1)


class PodManager:
    def __init__(self):
        self._pods: dict[str, PodInfo] = {}
        self._by_node: dict[str, set[str]] = {}
        self._node_gen: dict[str, int] = {}
        self._mu = threading.RLock()

    # caller holds _mu
    def _touch(self, node_id: str):
        self._node_gen[node_id] = next(_GEN)

    def _index(self, k: str, node_id: str):
        self._by_node.setdefault(node_id, set()).add(k)
        self._touch(node_id)

    def _unindex(self, k: str, node_id: str):
        s = self._by_node.get(node_id)
        if s is not None:
            s.discard(k)
            if not s:
                del self._by_node[node_id]
        self._touch(node_id)

    def _pop(self, k: str) -> PodInfo | None:
        pi = self._pods.pop(k, None)
        if pi is not None:
            self._unindex(k, pi.node_id)
        return pi

    def add_pod(self, pod: dict, node_id: str, devices: dict) -> bool:
        """Store collapsed usage; returns True if newly added."""
        with self._mu:
            k = _uid(pod)
            pi = self._pods.get(k)
            if pi is None:
                self._pods[k] = PodInfo(jcopy(pod), node_id, copy_pod_devices(devices))
                self._index(k, node_id)
                log.info("pod added %s/%s node=%s", pod["metadata"].get("namespace"), pod["metadata"]["name"], node_id)
                return True
            pi.pod = jcopy(pod)
            if pi.node_id != node_id:
                self._unindex(k, pi.node_id)
                pi.node_id = node_id
                self._index(k, node_id)
            if not pi.init_released:
                pi.devices = copy_pod_devices(devices)
                self._touch(node_id)
            return False

    def update_pod(self, pod: dict):
        with self._mu:
            pi = self._pods.get(_uid(pod))
            if pi:
                pi.pod = jcopy(pod)

    def del_pod(self, pod: dict):
        with self._mu:
            self._pop(_uid(pod))

    def get_pod(self, pod: dict) -> PodInfo | None:
        with self._mu:
            pi = self._pods.get(_uid(pod))
            return pi.deepcopy() if pi else None

    def take_and_delete_pod(self, pod: dict) -> PodInfo | None:
        with self._mu:
            return self._pop(_uid(pod))

    def update_pod_device(self, pod: dict, new_devices: dict):
        with self._mu:
            pi = self._pods.get(_uid(pod))
            if pi is None:
                return None, False
            old = pi.devices
            pi.devices = copy_pod_devices(new_devices)
            pi.init_released = True
            self._touch(pi.node_id)
            return old, True

    def node_generation(self, node_id: str) -> int:
        with self._mu:
            return self._node_gen.get(node_id, 0)

    def pods_on_node(self, node_id: str) -> tuple[int, list[PodInfo]]:
        """(generation, live entries) of the pods placed on ``node_id``.  The
        entries are read-only for the caller: their ``devices`` are replaced,
        never mutated, by the writers above."""
        with self._mu:
            ks = self._by_node.get(node_id, ())
            return self._node_gen.get(node_id, 0), [self._pods[k] for k in ks]

    def list_pods_info(self) -> list[PodInfo]:
        with self._mu:
            return [p.deepcopy() for p in self._pods.values()]

    def get_scheduled_pods(self) -> dict[str, PodInfo]:
        with self._mu:
            return {k: p.deepcopy() for k, p in self._pods.items()}

    def __len__(self):
        with self._mu:
            return len(self._pods)
