"""Minimal REST client for a real API server (in-cluster or kubeconfig).

Reference: pkg/util/client/client.go:58-107 and options.go:26-69 (QPS / Burst /
Timeout).  Only the verbs the control plane uses are implemented; watches are
streamed ``?watch=1`` responses re-established on expiry (410 Gone -> relist).
"""

from __future__ import annotations

import base64
import json
import logging
import os
import tempfile
import threading
import time
from pathlib import Path

import requests
import yaml

from .client import AlreadyExists, ApiError, Conflict, KubeClient, NotFound, Unauthorized

log = logging.getLogger(__name__)

_PATHS = {
    "nodes": ("/api/v1", "nodes"),
    "pods": ("/api/v1", "pods"),
    "resourcequotas": ("/api/v1", "resourcequotas"),
    "events": ("/api/v1", "events"),
    "leases": ("/apis/coordination.k8s.io/v1", "leases"),
}
_NAMESPACED = {"pods", "resourcequotas", "events", "leases"}


class _Throttle:
    def __init__(self, qps: float, burst: int):
        self.qps, self.burst = qps, max(1, burst)
        self.tokens = float(self.burst)
        self.t = time.monotonic()
        self.mu = threading.Lock()

    def wait(self):
        if self.qps <= 0:
            return
        with self.mu:
            now = time.monotonic()
            self.tokens = min(self.burst, self.tokens + (now - self.t) * self.qps)
            self.t = now
            if self.tokens < 1:
                time.sleep((1 - self.tokens) / self.qps)
                self.tokens = 0
            else:
                self.tokens -= 1


class RestClient(KubeClient):
    def __init__(self, server: str, token: str | None = None, ca: str | bool = True,
                 cert: tuple | None = None, qps: float = 50.0, burst: int = 100,
                 timeout: float = 30.0):
        self.server = server.rstrip("/")
        self.s = requests.Session()
        if token:
            self.s.headers["Authorization"] = f"Bearer {token}"
        self.s.verify = ca
        if cert:
            self.s.cert = cert
        self.timeout = timeout
        self.throttle = _Throttle(qps, burst)

    # ------------------------------------------------------------- factory
    @classmethod
    def from_env(cls, kubeconfig: str | None = None, **kw) -> "RestClient":
        kubeconfig = kubeconfig or os.environ.get("KUBECONFIG")
        host = os.environ.get("KUBERNETES_SERVICE_HOST")
        if not kubeconfig and host:
            sa = Path("/var/run/secrets/kubernetes.io/serviceaccount")
            port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
            return cls(f"https://{host}:{port}", token=(sa / "token").read_text().strip(),
                       ca=str(sa / "ca.crt"), **kw)
        path = Path(kubeconfig or Path.home() / ".kube" / "config")
        cfg = yaml.safe_load(path.read_text())
        ctx_name = cfg.get("current-context")
        ctx = next(c["context"] for c in cfg["contexts"] if c["name"] == ctx_name)
        cluster = next(c["cluster"] for c in cfg["clusters"] if c["name"] == ctx["cluster"])
        user = next((u["user"] for u in cfg.get("users", []) if u["name"] == ctx.get("user")), {})

        def materialise(data_b64, suffix):
            f = tempfile.NamedTemporaryFile(delete=False, suffix=suffix)
            f.write(base64.b64decode(data_b64))
            f.close()
            return f.name

        ca: str | bool = True
        if cluster.get("insecure-skip-tls-verify"):
            ca = False
        elif cluster.get("certificate-authority-data"):
            ca = materialise(cluster["certificate-authority-data"], ".crt")
        elif cluster.get("certificate-authority"):
            ca = cluster["certificate-authority"]
        cert = None
        if user.get("client-certificate-data") and user.get("client-key-data"):
            cert = (materialise(user["client-certificate-data"], ".crt"),
                    materialise(user["client-key-data"], ".key"))
        elif user.get("client-certificate") and user.get("client-key"):
            cert = (user["client-certificate"], user["client-key"])
        return cls(cluster["server"], token=user.get("token"), ca=ca, cert=cert, **kw)

    # ------------------------------------------------------------ plumbing
    def _url(self, kind, name=None, namespace=None, sub=None):
        prefix, res = _PATHS[kind]
        u = self.server + prefix
        if kind in _NAMESPACED and namespace:
            u += f"/namespaces/{namespace}"
        u += f"/{res}"
        if name:
            u += f"/{name}"
        if sub:
            u += f"/{sub}"
        return u

    def _req(self, method, url, **kw):
        self.throttle.wait()
        r = self.s.request(method, url, timeout=kw.pop("timeout", self.timeout), **kw)
        if r.status_code >= 400:
            try:
                body = r.json()
                msg, reason = body.get("message", ""), body.get("reason", "")
            except ValueError:
                msg, reason = r.text, ""
            if r.status_code == 404:
                raise NotFound(msg)
            if r.status_code == 409:
                raise AlreadyExists(msg) if reason == "AlreadyExists" else Conflict(msg)
            if r.status_code == 401:
                raise Unauthorized(msg)
            raise ApiError(r.status_code, reason or r.reason, msg)
        return r.json() if r.content else {}

    @staticmethod
    def _selector(sel: dict | None) -> str | None:
        return ",".join(f"{k}={v}" for k, v in sel.items()) if sel else None

    # ----------------------------------------------------------------- API
    def get(self, kind, name, namespace=None):
        return self._req("GET", self._url(kind, name, namespace))

    def list(self, kind, namespace=None, label_selector=None, field_selector=None):
        params = {}
        if label_selector:
            params["labelSelector"] = self._selector(label_selector)
        if field_selector:
            params["fieldSelector"] = self._selector(field_selector)
        body = self._req("GET", self._url(kind, namespace=namespace), params=params)
        items = body.get("items", [])
        for it in items:
            it.setdefault("kind", body.get("kind", "").removesuffix("List"))
        return items

    def create(self, kind, obj, namespace=None):
        ns = namespace or (obj.get("metadata") or {}).get("namespace")
        return self._req("POST", self._url(kind, namespace=ns), json=obj)

    def update(self, kind, obj, namespace=None):
        md = obj.get("metadata") or {}
        return self._req("PUT", self._url(kind, md.get("name"), namespace or md.get("namespace")),
                         json=obj)

    def patch(self, kind, name, patch, namespace=None):
        return self._req("PATCH", self._url(kind, name, namespace), data=json.dumps(patch),
                         headers={"Content-Type": "application/merge-patch+json"})

    def delete(self, kind, name, namespace=None):
        self._req("DELETE", self._url(kind, name, namespace))

    def bind(self, namespace, pod_name, node, uid=None):
        body = {"apiVersion": "v1", "kind": "Binding",
                "metadata": {"name": pod_name, "namespace": namespace},
                "target": {"apiVersion": "v1", "kind": "Node", "name": node}}
        if uid:
            body["metadata"]["uid"] = uid
        self._req("POST", self._url("pods", pod_name, namespace, "binding"), json=body)

    def evict(self, namespace, pod_name):
        body = {"apiVersion": "policy/v1", "kind": "Eviction",
                "metadata": {"name": pod_name, "namespace": namespace}}
        self._req("POST", self._url("pods", pod_name, namespace, "eviction"), json=body)

    def watch(self, kind, handler, namespace=None, field_selector=None):
        stop = threading.Event()
        sel = {"fieldSelector": self._selector(field_selector)} if field_selector else {}

        def loop():
            rv = None
            known: dict = {}
            while not stop.is_set():
                try:
                    if rv is None:
                        body = self._req("GET", self._url(kind, namespace=namespace), params=dict(sel))
                        rv = body["metadata"].get("resourceVersion")
                        fresh = {}
                        for it in body.get("items", []):
                            key = (it["metadata"].get("namespace"), it["metadata"]["name"])
                            fresh[key] = it
                            handler("ADDED" if key not in known else "MODIFIED", it, known.get(key))
                        for key, old in known.items():
                            if key not in fresh:
                                handler("DELETED", old, None)
                        known = fresh
                    params = {"watch": "1", "resourceVersion": rv, "timeoutSeconds": "300",
                              "allowWatchBookmarks": "true", **sel}
                    self.throttle.wait()
                    with self.s.get(self._url(kind, namespace=namespace), params=params, stream=True,
                                    timeout=(self.timeout, 330)) as r:
                        if r.status_code == 410:
                            rv = None
                            continue
                        for line in r.iter_lines():
                            if stop.is_set():
                                return
                            if not line:
                                continue
                            ev = json.loads(line)
                            et, obj = ev.get("type"), ev.get("object", {})
                            if et == "ERROR":
                                if obj.get("code") == 410:
                                    rv = None
                                break
                            rv = obj.get("metadata", {}).get("resourceVersion", rv)
                            if et == "BOOKMARK":
                                continue
                            key = (obj["metadata"].get("namespace"), obj["metadata"]["name"])
                            old = known.get(key)
                            if et == "DELETED":
                                known.pop(key, None)
                            else:
                                known[key] = obj
                            handler(et, obj, old)
                except Exception as e:  # network hiccup: back off and resume
                    log.warning("watch %s failed: %s", kind, e)
                    time.sleep(2)

        th = threading.Thread(target=loop, name=f"watch-{kind}", daemon=True)
        th.start()
        return stop.set
