"""Kubernetes client abstraction shared by scheduler, device plugin and monitor.

Objects are plain JSON dicts (the wire format), so the same code talks to the
real API server (:mod:`.rest`) and to the in-process fake (:mod:`.fake`, the
analogue of client-go's ``fake.NewClientset()`` used by the reference's 16
fake-clientset test files).  The global-client pattern mirrors
pkg/util/client/client.go:58-107 (``InitGlobalClient`` / ``GetClient``).
"""

from __future__ import annotations

import threading
from typing import Callable, Iterable, Optional

from k8s_vgpu_scheduler_amd.utils.jcopy import jcopy

KINDS = ("nodes", "pods", "resourcequotas", "events", "leases")
NAMESPACED = {"pods", "resourcequotas", "events", "leases"}


class ApiError(Exception):
    def __init__(self, code: int, reason: str, message: str = ""):
        super().__init__(f"{code} {reason}: {message}")
        self.code = code
        self.reason = reason
        self.message = message


class NotFound(ApiError):
    def __init__(self, message=""):
        super().__init__(404, "NotFound", message)


class Conflict(ApiError):
    def __init__(self, message=""):
        super().__init__(409, "Conflict", message)


class AlreadyExists(ApiError):
    def __init__(self, message=""):
        super().__init__(409, "AlreadyExists", message)


class Unauthorized(ApiError):
    def __init__(self, message=""):
        super().__init__(401, "Unauthorized", message)


def is_not_found(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.code == 404


def is_conflict(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.code == 409


class KubeClient:
    """Interface.  Every method returns deep copies (callers may mutate)."""

    def get(self, kind: str, name: str, namespace: str | None = None) -> dict:
        raise NotImplementedError

    def list(self, kind: str, namespace: str | None = None, label_selector: dict | None = None,
             field_selector: dict | None = None) -> list[dict]:
        raise NotImplementedError

    def create(self, kind: str, obj: dict, namespace: str | None = None) -> dict:
        raise NotImplementedError

    def update(self, kind: str, obj: dict, namespace: str | None = None) -> dict:
        raise NotImplementedError

    def patch(self, kind: str, name: str, patch: dict, namespace: str | None = None) -> dict:
        """JSON merge patch (RFC 7386); a metadata.resourceVersion in the patch
        is an optimistic-concurrency precondition (409 on mismatch)."""
        raise NotImplementedError

    def delete(self, kind: str, name: str, namespace: str | None = None) -> None:
        raise NotImplementedError

    def bind(self, namespace: str, pod_name: str, node: str, uid: str | None = None) -> None:
        raise NotImplementedError

    def evict(self, namespace: str, pod_name: str) -> None:
        """Eviction API (POST pods/<name>/eviction, policy/v1): the API server
        deletes the pod unless a PodDisruptionBudget refuses (429)."""
        raise NotImplementedError

    def watch(self, kind: str, handler: Callable[[str, dict, Optional[dict]], None],
              namespace: str | None = None, field_selector: dict | None = None) -> Callable[[], None]:
        """Subscribe to ADDED/MODIFIED/DELETED events; returns an unsubscribe fn.
        handler(event_type, obj, old_obj).  With ``field_selector`` only objects
        matching it are delivered (an object leaving the selection arrives as
        DELETED, one entering it as ADDED)."""
        raise NotImplementedError

    # -- typed conveniences -------------------------------------------------
    def get_node(self, name: str) -> dict:
        return self.get("nodes", name)

    def list_nodes(self, label_selector: dict | None = None) -> list[dict]:
        return self.list("nodes", label_selector=label_selector)

    def get_pod(self, namespace: str, name: str) -> dict:
        return self.get("pods", name, namespace)

    def list_pods(self, namespace: str | None = None, label_selector=None, field_selector=None):
        return self.list("pods", namespace, label_selector, field_selector)

    def patch_node(self, name: str, patch: dict) -> dict:
        return self.patch("nodes", name, patch)

    def patch_pod(self, namespace: str, name: str, patch: dict) -> dict:
        return self.patch("pods", name, patch, namespace)


# ---------------------------------------------------------------- merge patch
def merge_patch(target, patch):
    """RFC 7386 JSON merge patch (None deletes a key)."""
    if not isinstance(patch, dict):
        return jcopy(patch)
    out = jcopy(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        elif isinstance(v, dict):
            out[k] = merge_patch(out.get(k), v)
        else:
            out[k] = jcopy(v)
    return out


def match_labels(obj: dict, selector: dict | None) -> bool:
    if not selector:
        return True
    labels = (obj.get("metadata") or {}).get("labels") or {}
    return all(labels.get(k) == v for k, v in selector.items())


def _field(obj: dict, path: str):
    cur = obj
    for part in path.split("."):
        if not isinstance(cur, dict):
            return None
        cur = cur.get(part)
    return cur


def match_fields(obj: dict, selector: dict | None) -> bool:
    if not selector:
        return True
    for k, v in selector.items():
        got = _field(obj, k)
        if (got or "") != v:
            return False
    return True


# ------------------------------------------------------------- global client
_client: KubeClient | None = None
_client_lock = threading.Lock()


def init_global_client(client: KubeClient) -> KubeClient:
    global _client
    with _client_lock:
        _client = client
    return client


def get_client() -> KubeClient:
    if _client is None:
        raise RuntimeError("kubernetes client is not initialized")
    return _client


def has_client() -> bool:
    return _client is not None


# ------------------------------------------------------------ object helpers
def meta(obj: dict) -> dict:
    return obj.setdefault("metadata", {})


def name_of(obj: dict) -> str:
    return (obj.get("metadata") or {}).get("name", "")


def ns_of(obj: dict) -> str:
    return (obj.get("metadata") or {}).get("namespace", "")


def uid_of(obj: dict) -> str:
    return (obj.get("metadata") or {}).get("uid", "")


def annotations(obj: dict) -> dict:
    return (obj.get("metadata") or {}).get("annotations") or {}


def labels(obj: dict) -> dict:
    return (obj.get("metadata") or {}).get("labels") or {}


def containers(pod: dict) -> list:
    return (pod.get("spec") or {}).get("containers") or []


def init_containers(pod: dict) -> list:
    return (pod.get("spec") or {}).get("initContainers") or []


def all_containers(pods: Iterable[dict]):
    for p in pods:
        yield from init_containers(p)
        yield from containers(p)
