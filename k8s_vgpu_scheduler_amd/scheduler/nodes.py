"""Thread-safe node -> NodeInfo cache with deep-copy discipline (pkg/scheduler/nodes.go:30-170)."""

from __future__ import annotations

import threading

from k8s_vgpu_scheduler_amd.device.types import NodeInfo


class NodeManager:
    def __init__(self):
        self._nodes: dict[str, NodeInfo] = {}
        self._mu = threading.RLock()

    def add_node(self, node_id: str, info: NodeInfo):
        """Merge per-vendor device lists (a vendor's entry is replaced whole)."""
        if info is None or not info.devices:
            return
        with self._mu:
            cur = self._nodes.get(node_id)
            if cur is None:
                self._nodes[node_id] = info.deepcopy()
                return
            cur.node = info.deepcopy().node
            for vendor, devs in info.devices.items():
                cur.devices[vendor] = [d.deepcopy() for d in devs]

    def rm_node_devices(self, node_id: str, vendor: str):
        with self._mu:
            cur = self._nodes.get(node_id)
            if cur is None:
                return
            cur.devices.pop(vendor, None)
            if not cur.devices:
                self._nodes.pop(node_id, None)

    def rm_node(self, node_id: str):
        with self._mu:
            self._nodes.pop(node_id, None)

    def get_node(self, node_id: str) -> NodeInfo:
        with self._mu:
            n = self._nodes.get(node_id)
            if n is None:
                raise LookupError(f"node {node_id} not found")
            return n.deepcopy()

    def node_ids(self) -> list[str]:
        with self._mu:
            return list(self._nodes)

    def list_nodes(self) -> dict[str, NodeInfo]:
        with self._mu:
            return {k: v.deepcopy() for k, v in self._nodes.items()}
