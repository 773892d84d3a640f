"""In-process fake Kubernetes API server (the analogue of client-go's fake clientset).

Faithful where the control plane depends on it:
  * monotonically increasing ``resourceVersion`` and 409 Conflict when a merge
    patch / update carries a stale one (nodelock's optimistic concurrency,
    pkg/util/nodelock/nodelock.go:159-160, 222);
  * JSON merge-patch with ``null`` deletion;
  * label / field selectors (``spec.nodeName=...``, pkg/util/util.go:76-118);
  * watches (ADDED/MODIFIED/DELETED) delivered synchronously after the write;
  * ``pods/binding`` sets ``spec.nodeName``;
  * reactors to inject failures, e.g. a conflict storm or a PATCH whose
    response is lost after it was applied (nodelock_test.go:81 in the reference).
"""

from __future__ import annotations

import itertools
import threading
import time
import uuid
from typing import Callable, Optional

from k8s_vgpu_scheduler_amd.utils.jcopy import jcopy

from .client import (NAMESPACED, AlreadyExists, ApiError, Conflict, KubeClient, NotFound,
                     match_fields, match_labels, merge_patch)


class Reactor:
    """fn(verb, kind, name, namespace, payload) -> None to continue, or raise,
    or return ("after", exc) to apply the write and then raise exc."""

    def __init__(self, verb: str, kind: str, fn: Callable):
        self.verb, self.kind, self.fn = verb, kind, fn


class FakeCluster(KubeClient):
    def __init__(self):
        self._lock = threading.RLock()
        self._objs: dict[str, dict] = {}  # kind -> {(ns,name): obj}
        self._rv = itertools.count(1)
        self._watchers: dict[str, list] = {}
        self.reactors: list[Reactor] = []
        self.actions: list[tuple] = []  # (verb, kind, ns, name)
        self.evictions: list[tuple] = []  # (ns, name) of Eviction API calls

    # ------------------------------------------------------------ internals
    def _store(self, kind):
        return self._objs.setdefault(kind, {})

    @staticmethod
    def _key(kind, name, namespace):
        return ((namespace or "default") if kind in NAMESPACED else "", name)

    def _react(self, verb, kind, name, namespace, payload):
        after = None
        for r in list(self.reactors):
            if (r.verb in ("*", verb)) and (r.kind in ("*", kind)):
                res = r.fn(verb, kind, name, namespace, payload)
                if isinstance(res, tuple) and res and res[0] == "after":
                    after = res[1]
        return after

    def _notify(self, kind, etype, obj, old):
        for ns, h, fs in list(self._watchers.get(kind, [])):
            if ns and (obj.get("metadata") or {}).get("namespace") != ns:
                continue
            et = etype
            if fs:
                # a field-selected watch sees an object enter (ADDED) and leave
                # (DELETED) the selection, as the API server's filtered watch does
                now_in = match_fields(obj, fs)
                was_in = old is not None and match_fields(old, fs)
                if et == "MODIFIED" and now_in != was_in:
                    et = "ADDED" if now_in else "DELETED"
                elif not now_in and not (et == "DELETED" and was_in):
                    continue
            try:
                h(et, jcopy(obj), jcopy(old) if old else None)
            except Exception:  # a broken handler must not break the API server
                import logging
                logging.getLogger(__name__).exception("watch handler failed")

    def _bump(self, obj):
        md = obj.setdefault("metadata", {})
        md["resourceVersion"] = str(next(self._rv))

    # ------------------------------------------------------------------ API
    def get(self, kind, name, namespace=None):
        with self._lock:
            self.actions.append(("get", kind, namespace, name))
            self._react("get", kind, name, namespace, None)
            o = self._store(kind).get(self._key(kind, name, namespace))
            if o is None:
                raise NotFound(f"{kind} {namespace or ''}/{name} not found")
            return jcopy(o)

    def list(self, kind, namespace=None, label_selector=None, field_selector=None):
        with self._lock:
            self.actions.append(("list", kind, namespace, None))
            self._react("list", kind, None, namespace, None)
            out = []
            for (ns, _), o in self._store(kind).items():
                if namespace and kind in NAMESPACED and ns != namespace:
                    continue
                if match_labels(o, label_selector) and match_fields(o, field_selector):
                    out.append(jcopy(o))
            return out

    def create(self, kind, obj, namespace=None):
        events = []
        with self._lock:
            obj = jcopy(obj)
            md = obj.setdefault("metadata", {})
            if kind in NAMESPACED:
                md["namespace"] = namespace or md.get("namespace") or "default"
            if not md.get("name") and md.get("generateName"):
                md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
            md.setdefault("uid", str(uuid.uuid4()))
            md.setdefault("creationTimestamp", time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
            self.actions.append(("create", kind, md.get("namespace"), md["name"]))
            after = self._react("create", kind, md["name"], md.get("namespace"), obj)
            key = self._key(kind, md["name"], md.get("namespace"))
            if key in self._store(kind):
                raise AlreadyExists(f"{kind} {md['name']} exists")
            self._bump(obj)
            self._store(kind)[key] = obj
            events.append((kind, "ADDED", jcopy(obj), None))
        for e in events:
            self._notify(*e)
        if after:
            raise after
        return jcopy(obj)

    def update(self, kind, obj, namespace=None):
        with self._lock:
            md = obj.get("metadata") or {}
            ns = namespace or md.get("namespace")
            key = self._key(kind, md.get("name"), ns)
            self.actions.append(("update", kind, ns, md.get("name")))
            after = self._react("update", kind, md.get("name"), ns, obj)
            cur = self._store(kind).get(key)
            if cur is None:
                raise NotFound(f"{kind} {md.get('name')} not found")
            rv = md.get("resourceVersion")
            if rv and rv != cur["metadata"]["resourceVersion"]:
                raise Conflict(f"{kind} {md.get('name')}: resourceVersion {rv} is stale")
            new = jcopy(obj)
            new.setdefault("metadata", {})["uid"] = cur["metadata"].get("uid")
            self._bump(new)
            self._store(kind)[key] = new
            old = cur
        self._notify(kind, "MODIFIED", new, old)
        if after:
            raise after
        return jcopy(new)

    def patch(self, kind, name, patch, namespace=None):
        with self._lock:
            key = self._key(kind, name, namespace)
            self.actions.append(("patch", kind, namespace, name))
            after = self._react("patch", kind, name, namespace, patch)
            cur = self._store(kind).get(key)
            if cur is None:
                raise NotFound(f"{kind} {namespace or ''}/{name} not found")
            rv = ((patch or {}).get("metadata") or {}).get("resourceVersion")
            if rv is not None and rv != cur["metadata"]["resourceVersion"]:
                raise Conflict(f"{kind} {name}: resourceVersion {rv} is stale")
            new = merge_patch(cur, patch)
            new["metadata"]["name"] = cur["metadata"]["name"]
            new["metadata"]["uid"] = cur["metadata"].get("uid")
            self._bump(new)
            self._store(kind)[key] = new
            old = cur
        self._notify(kind, "MODIFIED", new, old)
        if after:
            raise after
        return jcopy(new)

    def delete(self, kind, name, namespace=None):
        with self._lock:
            key = self._key(kind, name, namespace)
            self.actions.append(("delete", kind, namespace, name))
            self._react("delete", kind, name, namespace, None)
            cur = self._store(kind).pop(key, None)
            if cur is None:
                raise NotFound(f"{kind} {name} not found")
        self._notify(kind, "DELETED", cur, None)

    def bind(self, namespace, pod_name, node, uid=None):
        with self._lock:
            self._react("create", "bindings", pod_name, namespace, {"node": node})
            cur = self._store("pods").get(self._key("pods", pod_name, namespace))
            if cur is None:
                raise NotFound(f"pod {namespace}/{pod_name} not found")
            if uid and cur["metadata"].get("uid") != uid:
                raise Conflict("pod uid mismatch")
            if (cur.get("spec") or {}).get("nodeName"):
                raise Conflict(f"pod {pod_name} is already assigned to a node")
        self.patch("pods", pod_name, {"spec": {"nodeName": node}}, namespace)

    def evict(self, namespace, pod_name):
        with self._lock:
            self.actions.append(("evict", "pods", namespace, pod_name))
            self._react("evict", "pods", pod_name, namespace, None)
            self.evictions.append((namespace or "default", pod_name))
        self.delete("pods", pod_name, namespace)

    def watch(self, kind, handler, namespace=None, field_selector=None):
        with self._lock:
            entry = (namespace, handler, field_selector)
            self._watchers.setdefault(kind, []).append(entry)

        def stop():
            with self._lock:
                try:
                    self._watchers[kind].remove(entry)
                except ValueError:
                    pass
        return stop

    # ----------------------------------------------------------- test sugar
    def add_reactor(self, verb: str, kind: str, fn: Callable) -> Reactor:
        r = Reactor(verb, kind, fn)
        self.reactors.insert(0, r)
        return r

    def remove_reactor(self, r: Reactor):
        if r in self.reactors:
            self.reactors.remove(r)

    def count(self, verb: str, kind: str) -> int:
        return sum(1 for a in self.actions if a[0] == verb and a[1] == kind)


def make_node(name: str, annotations: dict | None = None, labels: dict | None = None,
              capacity: dict | None = None, allocatable: dict | None = None) -> dict:
    return {"apiVersion": "v1", "kind": "Node",
            "metadata": {"name": name, "annotations": dict(annotations or {}),
                         "labels": dict(labels or {})},
            "status": {"capacity": dict(capacity or {}),
                       "allocatable": dict(allocatable if allocatable is not None else (capacity or {}))}}


def make_pod(name: str, namespace: str = "default", containers: list | None = None,
             init_containers: list | None = None, annotations: dict | None = None,
             labels: dict | None = None, node_name: str = "", phase: str = "Pending",
             uid: str | None = None, scheduler_name: str = "") -> dict:
    spec = {"containers": containers or [{"name": "main", "resources": {}}]}
    if init_containers:
        spec["initContainers"] = init_containers
    if node_name:
        spec["nodeName"] = node_name
    if scheduler_name:
        spec["schedulerName"] = scheduler_name
    md = {"name": name, "namespace": namespace, "annotations": dict(annotations or {}),
          "labels": dict(labels or {})}
    if uid:
        md["uid"] = uid
    return {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": spec,
            "status": {"phase": phase}}


def container(name: str, limits: dict | None = None, requests: dict | None = None,
              env: list | None = None, privileged: bool = False) -> dict:
    c = {"name": name, "resources": {}}
    if limits:
        c["resources"]["limits"] = {k: str(v) for k, v in limits.items()}
    if requests:
        c["resources"]["requests"] = {k: str(v) for k, v in requests.items()}
    if env:
        c["env"] = env
    if privileged:
        c["securityContext"] = {"privileged": True}
    return c
