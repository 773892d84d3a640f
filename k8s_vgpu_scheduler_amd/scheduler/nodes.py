"""Thread-safe node -> NodeInfo cache with deep-copy discipline (pkg/scheduler/nodes.go:30-170).

Stored entries are copy-on-write: every change replaces the node's NodeInfo
object and bumps its generation, so ``get_node_ref`` can hand out the live
object without a deep copy (callers must treat it as read-only) and the
scheduler's per-node usage cache can tell when a registration changed.
"""

from __future__ import annotations

import itertools
import threading

from k8s_vgpu_scheduler_amd.device.types import NodeInfo

_GEN = itertools.count(1)


class NodeManager:
    def __init__(self):
        self._nodes: dict[str, NodeInfo] = {}
        self._gen: dict[str, int] = {}
        self._mu = threading.RLock()

    def add_node(self, node_id: str, info: NodeInfo):
        """Merge per-vendor device lists (a vendor's entry is replaced whole)."""
        if info is None or not info.devices:
            return
        with self._mu:
            cur = self._nodes.get(node_id)
            if cur is None:
                new = info.deepcopy()
            else:
                merged = dict(cur.devices)
                for vendor, devs in info.devices.items():
                    merged[vendor] = [d.deepcopy() for d in devs]
                new = NodeInfo(id=cur.id, node=info.deepcopy().node, devices=merged)
            self._nodes[node_id] = new
            self._gen[node_id] = next(_GEN)

    def rm_node_devices(self, node_id: str, vendor: str):
        with self._mu:
            cur = self._nodes.get(node_id)
            if cur is None:
                return
            devs = {k: v for k, v in cur.devices.items() if k != vendor}
            if not devs:
                self._nodes.pop(node_id, None)
                self._gen.pop(node_id, None)
                return
            self._nodes[node_id] = NodeInfo(id=cur.id, node=cur.node, devices=devs)
            self._gen[node_id] = next(_GEN)

    def rm_node(self, node_id: str):
        with self._mu:
            self._nodes.pop(node_id, None)
            self._gen.pop(node_id, None)

    def get_node(self, node_id: str) -> NodeInfo:
        with self._mu:
            n = self._nodes.get(node_id)
            if n is None:
                raise LookupError(f"node {node_id} not found")
            return n.deepcopy()

    def get_node_ref(self, node_id: str) -> tuple[int, NodeInfo] | None:
        """(generation, live NodeInfo) without copying; None if unregistered.
        The object is never mutated after publication."""
        with self._mu:
            n = self._nodes.get(node_id)
            return None if n is None else (self._gen[node_id], n)

    def generation(self, node_id: str) -> int:
        with self._mu:
            return self._gen.get(node_id, 0)

    def node_ids(self) -> list[str]:
        with self._mu:
            return list(self._nodes)

    def list_nodes(self) -> dict[str, NodeInfo]:
        with self._mu:
            return {k: v.deepcopy() for k, v in self._nodes.items()}
