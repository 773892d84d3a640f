"""Filter/score engine: fit every container of a pod onto every candidate node.

Reference: pkg/scheduler/score.go:81-419.  Per node: init containers are fitted
one at a time on throw-away copies and only their PEAK usage is kept
(they run sequentially), app containers are fitted cumulatively on one copy,
the node's default score is taken before the app fit, and the backend's
policy-neutral ``ScoreNode`` is added after.  Failures carry "n/N Reason"
strings that are aggregated into FilteringFailed events.
"""

from __future__ import annotations

import logging
from dataclasses import dataclass, field

from k8s_vgpu_scheduler_amd.device import common as R
from k8s_vgpu_scheduler_amd.device import devices as D
from k8s_vgpu_scheduler_amd.device.types import NodeInfo
from k8s_vgpu_scheduler_amd.k8s.client import init_containers
from k8s_vgpu_scheduler_amd.utils import types as T
from k8s_vgpu_scheduler_amd.utils.weights import DeviceScoringWeights, weights_for_pod

from .policy import DeviceUsageList, NodeScore, NodeScoreList

log = logging.getLogger(__name__)


@dataclass
class NodeUsage:
    node: dict
    node_info: NodeInfo | None
    devices: DeviceUsageList = field(default_factory=DeviceUsageList)

    def deepcopy(self) -> "NodeUsage":
        return NodeUsage(self.node, self.node_info, self.devices.deepcopy())


def get_node_resources(node: NodeUsage, t: str) -> list:
    tt = t.lower()
    return [d.device for d in node.devices.device_lists if tt in d.device.type.lower()]


def fit_in_devices(node: NodeUsage, requests: dict, pod: dict, node_info: NodeInfo | None,
                   devinput: dict, weights: DeviceScoringWeights) -> tuple[bool, str]:
    for dl in node.devices.device_lists:
        dl.compute_score(requests, weights)
    for k in requests.values():
        node.devices.sort()
        backend = D.get_devices().get(k.type)
        if backend is None:
            return False, "Device type not found"
        type_devices = get_node_resources(node, k.type)
        if k.nums > len(type_devices):
            return False, R.NODE_INSUFFICIENT_DEVICE
        ok, tmp, reason = backend.fit(type_devices, k, pod, node_info, devinput)
        if not ok:
            return False, reason
        by_id = {dl.device.id: dl.device for dl in node.devices.device_lists}
        for cd in tmp.get(k.type, []):
            d = by_id.get(cd.uuid)
            if d is None:
                return False, f"Device with UUID {cd.uuid!r} not found on node after Fit"
            backend.add_resource_usage(pod, d, cd)
        devinput.setdefault(k.type, []).append(tmp.get(k.type, []))
    return True, ""


def _snapshot_peak(devices: DeviceUsageList) -> dict:
    return {dl.device.id: (dl.device.used, dl.device.usedcores, dl.device.usedmem,
                           dl.device.custominfo.get("cu_used", 0), dl.device.custominfo.get("cu_shared") or {})
            for dl in devices.device_lists}


def _update_peak(peak: dict, copy: NodeUsage):
    from k8s_vgpu_scheduler_amd.device.amd.cu_alloc import merge_shared
    for dl in copy.devices.device_lists:
        d = dl.device
        p = peak.get(d.id)
        if p is None:
            peak[d.id] = (d.used, d.usedcores, d.usedmem, d.custominfo.get("cu_used", 0),
                          d.custominfo.get("cu_shared") or {})
        else:
            peak[d.id] = (max(p[0], d.used), max(p[1], d.usedcores), max(p[2], d.usedmem),
                          p[3] | d.custominfo.get("cu_used", 0), merge_shared(p[4], d.custominfo.get("cu_shared")))


def _apply_peak(node: NodeUsage, app_copy: NodeUsage, peak: dict):
    from k8s_vgpu_scheduler_amd.device.amd.cu_alloc import merge_shared
    app = {dl.device.id: dl.device for dl in app_copy.devices.device_lists}
    for dl in node.devices.device_lists:
        d = dl.device
        a = app.get(d.id)
        u, c, m, cu, sh = ((a.used, a.usedcores, a.usedmem, a.custominfo.get("cu_used", 0),
                            a.custominfo.get("cu_shared") or {}) if a else (0, 0, 0, 0, {}))
        p = peak.get(d.id)
        if p:
            u, c, m, cu, sh = max(u, p[0]), max(c, p[1]), max(m, p[2]), cu | p[3], merge_shared(sh, p[4])
        d.used, d.usedcores, d.usedmem = u, c, m
        if cu:
            d.custominfo["cu_used"] = cu
        if sh:
            d.custominfo["cu_shared"] = sh


def _base_types(devices: DeviceUsageList) -> set:
    out = set()
    for dl in devices.device_lists:
        for t in D.get_devices():
            if t.lower() in dl.device.type.lower():
                out.add(t)
    return out


def allocate_init_containers(node: NodeUsage, reqs: list, pod: dict, node_info, base_types, n_init,
                             peak, weights):
    init_allocs: dict = {}
    for i, req in enumerate(reqs[:n_init]):
        if not req:
            for t in base_types:
                init_allocs.setdefault(t, []).append([])
            continue
        copy = node.deepcopy()
        ok, reason = fit_in_devices(copy, req, pod, node_info, init_allocs, weights)
        if not ok:
            return None, False, reason
        _update_peak(peak, copy)
        for t in base_types:
            lst = init_allocs.setdefault(t, [])
            if len(lst) == i:
                lst.append([])
    return init_allocs, True, ""


def allocate_app_containers(score: NodeScore, app_copy: NodeUsage, reqs: list, pod: dict, node_info,
                            base_types, n_init, weights) -> tuple[str, bool]:
    app_index = 0
    for cid, req in enumerate(reqs):
        if cid < n_init:
            continue
        if sum(k.nums for k in req.values()) == 0:
            for t in base_types:
                score.devices.setdefault(t, []).append([])
            app_index += 1
            continue
        ok, reason = fit_in_devices(app_copy, req, pod, node_info, score.devices, weights)
        if not ok:
            return reason, False
        for t in base_types:
            lst = score.devices.setdefault(t, [])
            if len(lst) == app_index:
                lst.append([])
        app_index += 1
    return "", True


def score_node(node_id: str, node: NodeUsage, reqs: list, pod: dict, node_policy: str,
               weights: DeviceScoringWeights):
    """-> (NodeScore | None, reason)"""
    node_info = node.node_info
    base_types = _base_types(node.devices)
    peak = _snapshot_peak(node.devices)
    n_init = len(init_containers(pod))
    init_allocs = None
    if n_init:
        init_allocs, ok, reason = allocate_init_containers(node, reqs, pod, node_info, base_types, n_init,
                                                           peak, weights)
        if not ok:
            return None, reason
    app_copy = node.deepcopy()
    score = NodeScore(node_id=node_id, node=node.node, devices={}, score=0.0)
    score.compute_default_score(app_copy.devices)
    snapshot = NodeScore.snapshot_device(app_copy.devices)
    reason, ok = allocate_app_containers(score, app_copy, reqs, pod, node_info, base_types, n_init, weights)
    if not ok:
        return None, reason
    if n_init and init_allocs is not None:
        for t, lst in init_allocs.items():
            score.devices[t] = lst + score.devices.get(t, [])
    _apply_peak(node, app_copy, peak)
    score.override_score(snapshot, node_policy)
    return score, ""


def resolve_node_policy(pod: dict, default: str) -> str:
    annos = (pod.get("metadata") or {}).get("annotations") or {}
    return annos.get(T.NODE_POLICY_ANNOTATION, default)


def record_result(res: "NodeScoreList", failure: dict, failed: dict, node_id: str, s, reason: str):
    """Fold one node's (score | None, reason) into the Filter aggregates."""
    if s is None:
        failed[node_id] = reason
        for r in R.parse_reason(reason) or {reason: 1}:
            failure.setdefault(r, []).append(node_id)
    else:
        res.node_list.append(s)


def score_node_safe(node_id: str, usage: NodeUsage, reqs: list, pod: dict, policy: str,
                    weights: DeviceScoringWeights):
    """score_node that turns an exception into a per-node failure (one bad
    node must not fail the pod)."""
    try:
        return score_node(node_id, usage, reqs, pod, policy, weights)
    except Exception as e:  # noqa: BLE001
        log.exception("scoring node %s failed", node_id)
        return None, f"scoring error: {e}"


def calc_score(nodes: dict, reqs: list, pod: dict, failed: dict, default_node_policy: str):
    """-> (NodeScoreList, failure_reasons {reason: [nodes]})."""
    weights = weights_for_pod(pod)
    policy = resolve_node_policy(pod, default_node_policy)
    res = NodeScoreList(node_list=[], policy=policy)
    failure: dict[str, list] = {}
    for node_id, usage in nodes.items():
        s, reason = score_node_safe(node_id, usage, reqs, pod, policy, weights)
        record_result(res, failure, failed, node_id, s, reason)
    return res, failure
