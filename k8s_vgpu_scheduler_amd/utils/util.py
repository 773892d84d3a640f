"""Cluster helpers shared by the control plane (pkg/util/util.go:76-403).

Pending-pod discovery for Allocate, merge-patch helpers for pods and nodes,
policy parsing, pod state predicates, deduplicated node warning events and
PodGroup detection.  All helpers go through the global client
(:func:`k8s_vgpu_scheduler_amd.k8s.client.get_client`).
"""

from __future__ import annotations

import datetime as _dt
import logging

from k8s_vgpu_scheduler_amd.k8s.client import NotFound, get_client
from k8s_vgpu_scheduler_amd.utils import types as T

log = logging.getLogger(__name__)

# vendor -> handshake annotation key (util.go:31-37)
HANDSHAKE_ANNOS: dict[str, str] = {}


def get_node(name: str) -> dict:
    if not name:
        raise ValueError("nodename is empty")
    return get_client().get_node(name)


def get_allocate_pod_by_node(node_name: str) -> dict | None:
    """Pod named by the node lock (the lock holder is the pod being allocated)."""
    from k8s_vgpu_scheduler_amd.utils.nodelock import parse_node_lock

    node = get_client().get_node(node_name)
    value = ((node.get("metadata") or {}).get("annotations") or {}).get(T.NODE_LOCK_KEY)
    if value is None:
        return None
    _, ns, name = parse_node_lock(value)
    if not ns or not name:
        return None
    return get_client().get_pod(ns, name)


def get_pending_pod(node_name: str) -> dict:
    """util.go:76-118: lock holder first, else a Pending pod bound to this node
    in bind-phase allocating|success whose vgpu-node annotation matches."""
    pod = get_allocate_pod_by_node(node_name)
    if pod is not None:
        return pod
    for p in get_client().list_pods(field_selector={"spec.nodeName": node_name}):
        if (p.get("status") or {}).get("phase") != "Pending":
            continue
        annos = (p.get("metadata") or {}).get("annotations") or {}
        if T.BIND_TIME_ANNOTATION not in annos:
            continue
        if annos.get(T.DEVICE_BIND_PHASE) not in (T.DEVICE_BIND_ALLOCATING, T.DEVICE_BIND_SUCCESS):
            continue
        if annos.get(T.ASSIGNED_NODE_ANNOTATION) == node_name:
            return p
    raise LookupError(f"no binding pod found on node {node_name}")


def patch_node_annotations(node: dict | str, annotations: dict) -> dict:
    name = node if isinstance(node, str) else node["metadata"]["name"]
    return get_client().patch_node(name, {"metadata": {"annotations": dict(annotations)}})


def patch_pod_annotations(pod: dict, annotations: dict) -> dict:
    """Also mirrors hami.io/vgpu-node into a label (util.go:174-205)."""
    patch = {"metadata": {"annotations": dict(annotations)}}
    node = annotations.get(T.ASSIGNED_NODE_ANNOTATION)
    if node:
        patch["metadata"]["labels"] = {T.ASSIGNED_NODE_ANNOTATION: node}
    md = pod["metadata"]
    return get_client().patch_pod(md.get("namespace", "default"), md["name"], patch)


def patch_pod_labels(namespace: str, name: str, labels: dict) -> dict:
    return get_client().patch_pod(namespace, name, {"metadata": {"labels": dict(labels)}})


def remove_node_annotation(node_name: str, *keys: str) -> dict:
    return get_client().patch_node(node_name, {"metadata": {"annotations": {k: None for k in keys}}})


def mark_annotations_to_delete(key: str, node_name: str) -> dict:
    get_node(node_name)
    return remove_node_annotation(node_name, key)


def get_gpu_scheduler_policy_by_pod(default_policy: str, pod: dict | None) -> str:
    if pod:
        annos = (pod.get("metadata") or {}).get("annotations") or {}
        if T.GPU_POLICY_ANNOTATION in annos:
            return annos[T.GPU_POLICY_ANNOTATION]
    return default_policy


def policy_contains(policy: str, name: str) -> bool:
    return any(p.strip() == name for p in (policy or "").split(","))


def is_pod_terminated(pod: dict | None) -> bool:
    return bool(pod) and (pod.get("status") or {}).get("phase") in ("Failed", "Succeeded")


def is_pod_terminating(pod: dict | None) -> bool:
    return bool(pod) and bool((pod.get("metadata") or {}).get("deletionTimestamp"))


def all_containers_created(pod: dict | None) -> bool:
    if not pod:
        return False
    return len((pod.get("status") or {}).get("containerStatuses") or []) >= len(
        (pod.get("spec") or {}).get("containers") or [])


def all_init_containers_succeeded(pod: dict) -> bool:
    sts = (pod.get("status") or {}).get("initContainerStatuses") or []
    if not sts:
        return False
    for s in sts:
        term = (s.get("state") or {}).get("terminated")
        if not term or term.get("exitCode", 1) != 0:
            return False
    return True


def is_pod_group_member(pod: dict | None) -> bool:
    if not pod:
        return False
    if ((pod.get("metadata") or {}).get("labels") or {}).get(T.POD_GROUP_LABEL):
        return True
    sg = (pod.get("spec") or {}).get("schedulingGroup") or {}
    return bool(sg.get("podGroupName"))


def _now_rfc3339() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def emit_node_warning_event(node: dict, reason: str, message: str, dedup_window_s: float = 600.0,
                            component: str = "hami-device-plugin"):
    """Warning Event on a Node, deduplicated within a window (util.go:322-390)."""
    try:
        c = get_client()
    except RuntimeError:
        log.warning("cannot emit node event for %s: client not initialized", node["metadata"]["name"])
        return
    md = node["metadata"]
    now = _dt.datetime.now(_dt.timezone.utc)
    try:
        existing = c.list("events", "default", field_selector={
            "involvedObject.kind": "Node", "involvedObject.name": md["name"], "reason": reason})
    except Exception as e:  # noqa: BLE001
        log.warning("failed to list events for node %s: %s", md["name"], e)
        existing = []
    latest = None
    for ev in existing:
        if (ev.get("involvedObject") or {}).get("uid", "") != md.get("uid", "") or ev.get("reason") != reason:
            continue
        if latest is None or ev.get("lastTimestamp", "") > latest.get("lastTimestamp", ""):
            latest = ev
    if latest is not None:
        try:
            last = _dt.datetime.strptime(latest["lastTimestamp"], "%Y-%m-%dT%H:%M:%SZ").replace(
                tzinfo=_dt.timezone.utc)
            if (now - last).total_seconds() <= dedup_window_s:
                latest["count"] = int(latest.get("count", 1)) + 1
                latest["lastTimestamp"] = _now_rfc3339()
                latest["message"] = message
                c.update("events", latest, "default")
                return
        except (ValueError, KeyError, NotFound):
            pass
    ts = _now_rfc3339()
    c.create("events", {
        "metadata": {"generateName": md["name"] + "-", "namespace": "default"},
        "involvedObject": {"apiVersion": "v1", "kind": "Node", "name": md["name"], "uid": md.get("uid", "")},
        "reason": reason, "message": message, "type": "Warning", "count": 1,
        "firstTimestamp": ts, "lastTimestamp": ts, "source": {"component": component},
    }, "default")
