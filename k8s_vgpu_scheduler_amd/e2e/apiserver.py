"""A Kubernetes API server over real HTTP, backed by :class:`FakeCluster`.

The reference's e2e suite (test/e2e, hack/e2e-test.sh) runs against a real
cluster; this container has none, so the e2e tier runs the real binaries
(scheduler, device plugin, monitor) against this server instead.  They talk to
it through :class:`~k8s_vgpu_scheduler_amd.k8s.rest.RestClient`, the client a
real deployment uses, over the same REST paths:

  /api/v1/{nodes,pods,events,resourcequotas}[/name]
  /api/v1/namespaces/{ns}/{pods,events,resourcequotas}[/name[/binding|/status]]
  /apis/coordination.k8s.io/v1[/namespaces/{ns}]/leases[/name]

Semantics the clients depend on:
  * LIST returns ``metadata.resourceVersion``; ``labelSelector`` / ``fieldSelector``;
  * ``?watch=1&resourceVersion=N`` replays every event after N, then streams
    (one JSON object per line); a compacted N answers 410 Gone; idle streams
    get BOOKMARK events; ``timeoutSeconds`` ends the stream;
  * POST 201 / 409 AlreadyExists; PUT and merge PATCH with 409 on a stale
    resourceVersion; ``pods/{name}/binding``; errors are ``Status`` objects.
"""

from __future__ import annotations

import argparse
import json
import logging
import queue
import re
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

from k8s_vgpu_scheduler_amd.k8s.client import ApiError, match_fields, match_labels
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster

log = logging.getLogger(__name__)

KINDS = {"nodes": ("v1", "Node"), "pods": ("v1", "Pod"), "events": ("v1", "Event"),
         "resourcequotas": ("v1", "ResourceQuota"), "leases": ("coordination.k8s.io/v1", "Lease")}
_ROUTE = re.compile(r"^/(?:api/v1|apis/coordination\.k8s\.io/v1)"
                    r"(?:/namespaces/(?P<ns>[^/]+))?/(?P<kind>[a-z]+)(?:/(?P<name>[^/]+))?(?:/(?P<sub>[a-z]+))?/?$")
LOG_CAP = 20000          # events kept per kind for watch replay (older -> 410 Gone)


def _selector(s: str | None) -> dict | None:
    if not s:
        return None
    out = {}
    for part in s.split(","):
        k, _, v = part.partition("=")
        out[k.strip()] = v.strip().lstrip("=")
    return out


class FakeApiServer:
    def __init__(self, cluster: FakeCluster | None = None, host: str = "127.0.0.1", port: int = 0,
                 bookmark_s: float = 5.0, max_watch_s: float = 1800.0):
        self.cluster = cluster or FakeCluster()
        self.bookmark_s = bookmark_s
        self.max_watch_s = max_watch_s       # like --min-request-timeout: streams end, clients re-watch
        self._mu = threading.Lock()
        self._log: dict[str, list] = {k: [] for k in KINDS}       # kind -> [(rv, type, obj)]
        self._oldest: dict[str, int] = {k: 0 for k in KINDS}      # rv below which replay is gone
        self._subs: dict[str, set] = {k: set() for k in KINDS}
        self.latest_rv = 0
        for kind in KINDS:
            self.cluster.watch(kind, self._recorder(kind))
        self.requests: list[tuple[str, str]] = []                  # (method, path) for assertions
        handler = type("Handler", (_Handler,), {"api": self})
        self.httpd = ThreadingHTTPServer((host, port), handler)
        self.httpd.daemon_threads = True
        self.url = f"http://{host}:{self.httpd.server_address[1]}"
        self._thread: threading.Thread | None = None

    # ------------------------------------------------------------ events
    def _recorder(self, kind):
        def on_event(etype, obj, old):
            md = obj.setdefault("metadata", {})
            if etype == "DELETED":
                # a delete is a new revision of the store
                md["resourceVersion"] = str(next(self.cluster._rv))
            rv = int(md.get("resourceVersion") or 0)
            with self._mu:
                self.latest_rv = max(self.latest_rv, rv)
                lg = self._log[kind]
                lg.append((rv, etype, obj))
                if len(lg) > LOG_CAP:
                    drop = len(lg) - LOG_CAP
                    self._oldest[kind] = max(r for r, _, _ in lg[:drop])
                    del lg[:drop]
                for q in self._subs[kind]:
                    q.put((rv, etype, obj))
        return on_event

    def subscribe(self, kind: str, since: int):
        """-> (queue, replay events after `since`) or None when `since` is compacted."""
        q: queue.Queue = queue.Queue()
        with self._mu:
            if since < self._oldest[kind]:
                return None
            replay = [e for e in self._log[kind] if e[0] > since]
            self._subs[kind].add(q)
        return q, replay

    def unsubscribe(self, kind: str, q):
        with self._mu:
            self._subs[kind].discard(q)

    def compact(self, kind: str):
        """Drop the replay log (tests: forces 410 Gone on the next stale watch)."""
        with self._mu:
            if self._log[kind]:
                self._oldest[kind] = max(r for r, _, _ in self._log[kind])
            self._log[kind].clear()

    # ------------------------------------------------------------ lifecycle
    def start(self) -> "FakeApiServer":
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="apiserver", daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()

    def kubeconfig(self) -> str:
        return json.dumps({
            "apiVersion": "v1", "kind": "Config", "current-context": "e2e",
            "clusters": [{"name": "e2e", "cluster": {"server": self.url}}],
            "contexts": [{"name": "e2e", "context": {"cluster": "e2e", "user": "e2e"}}],
            "users": [{"name": "e2e", "user": {"token": "e2e"}}],
        })

    def write_kubeconfig(self, path: str) -> str:
        with open(path, "w") as f:
            f.write(self.kubeconfig())
        return path


class _Handler(BaseHTTPRequestHandler):
    api: FakeApiServer
    protocol_version = "HTTP/1.0"       # bodies end at close: streams need no chunking

    def log_message(self, fmt, *args):  # quiet; failures are reported as Status bodies
        log.debug("apiserver: " + fmt, *args)

    # ----------------------------------------------------------- plumbing
    def _send(self, code: int, body: dict):
        data = json.dumps(body).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def _status(self, code: int, reason: str, message: str):
        self._send(code, {"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": message,
                          "reason": reason, "code": code})

    def _body(self) -> dict:
        n = int(self.headers.get("Content-Length") or 0)
        return json.loads(self.rfile.read(n) or b"{}") if n else {}

    def _route(self):
        u = urlparse(self.path)
        self.api.requests.append((self.command, u.path))
        m = _ROUTE.match(u.path)
        if not m or m.group("kind") not in KINDS:
            return None, u
        return m, u

    def _dispatch(self, fn):
        m, u = self._route()
        if u.path in ("/healthz", "/readyz", "/livez"):
            data = b"ok"
            self.send_response(200)
            self.send_header("Content-Length", "2")
            self.end_headers()
            self.wfile.write(data)
            return
        if u.path == "/version":
            return self._send(200, {"major": "1", "minor": "31", "gitVersion": "v1.31.0-mivgpu-e2e"})
        if m is None:
            return self._status(404, "NotFound", f"no route for {u.path}")
        try:
            fn(m.group("kind"), m.group("ns"), m.group("name"), m.group("sub"), parse_qs(u.query))
        except ApiError as e:
            self._status(e.code, e.reason, e.message)
        except (BrokenPipeError, ConnectionResetError):
            pass
        except Exception as e:  # noqa: BLE001
            log.exception("apiserver handler failed")
            self._status(500, "InternalError", str(e))

    # -------------------------------------------------------------- verbs
    def do_GET(self):  # noqa: N802
        self._dispatch(self._get)

    def do_POST(self):  # noqa: N802
        self._dispatch(self._post)

    def do_PUT(self):  # noqa: N802
        self._dispatch(self._put)

    def do_PATCH(self):  # noqa: N802
        self._dispatch(self._patch)

    def do_DELETE(self):  # noqa: N802
        self._dispatch(self._delete)

    def _get(self, kind, ns, name, sub, q):
        c = self.api.cluster
        if name:
            return self._send(200, c.get(kind, name, ns))
        labels = _selector((q.get("labelSelector") or [None])[0])
        fields = _selector((q.get("fieldSelector") or [None])[0])
        if (q.get("watch") or ["0"])[0] in ("1", "true"):
            return self._watch(kind, ns, labels, fields, q)
        with self.api._mu:
            rv = self.api.latest_rv
        items = c.list(kind, ns, label_selector=labels, field_selector=fields)
        rv = max([rv] + [int(i["metadata"].get("resourceVersion") or 0) for i in items])
        api_version, k = KINDS[kind]
        self._send(200, {"kind": f"{k}List", "apiVersion": api_version,
                         "metadata": {"resourceVersion": str(rv)}, "items": items})

    def _watch(self, kind, ns, labels, fields, q):
        since = int((q.get("resourceVersion") or ["0"])[0] or 0)
        timeout = min(float((q.get("timeoutSeconds") or ["300"])[0]), self.api.max_watch_s)
        sub = self.api.subscribe(kind, since)
        if sub is None:
            return self._status(410, "Expired", f"too old resource version: {since}")
        qu, replay = sub
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.end_headers()
        api_version, k = KINDS[kind]

        def emit(etype, obj):
            self.wfile.write(json.dumps({"type": etype, "object": obj}).encode() + b"\n")
            self.wfile.flush()

        def wanted(obj):
            md = obj.get("metadata") or {}
            if ns and md.get("namespace") != ns:
                return False
            return match_labels(obj, labels) and match_fields(obj, fields)

        deadline = time.monotonic() + timeout
        try:
            for _, etype, obj in replay:
                if wanted(obj):
                    emit(etype, obj)
            while time.monotonic() < deadline:
                try:
                    _, etype, obj = qu.get(timeout=min(self.api.bookmark_s, max(0.05, deadline - time.monotonic())))
                except queue.Empty:
                    with self.api._mu:
                        rv = self.api.latest_rv
                    emit("BOOKMARK", {"kind": k, "apiVersion": api_version,
                                      "metadata": {"resourceVersion": str(rv)}})
                    continue
                if wanted(obj):
                    emit(etype, obj)
        except (BrokenPipeError, ConnectionResetError, OSError):
            pass
        finally:
            self.api.unsubscribe(kind, qu)

    def _post(self, kind, ns, name, sub, q):
        c = self.api.cluster
        body = self._body()
        if kind == "pods" and name and sub == "binding":
            target = (body.get("target") or {}).get("name")
            c.bind(ns or "default", name, target, (body.get("metadata") or {}).get("uid"))
            return self._send(201, {"kind": "Status", "apiVersion": "v1", "status": "Success", "code": 201})
        if kind == "pods" and name and sub == "eviction":
            if body.get("kind") != "Eviction":
                return self._status(400, "BadRequest", "eviction body must be an Eviction")
            c.evict(ns or "default", name)
            return self._send(201, {"kind": "Status", "apiVersion": "v1", "status": "Success", "code": 201})
        if name:
            return self._status(405, "MethodNotAllowed", "POST to a named resource")
        self._send(201, c.create(kind, body, ns))

    def _put(self, kind, ns, name, sub, q):
        body = self._body()
        md = body.setdefault("metadata", {})
        if name and md.get("name") not in (None, name):
            return self._status(400, "BadRequest", "name in body does not match the URL")
        md["name"] = name
        self._send(200, self.api.cluster.update(kind, body, ns))

    def _patch(self, kind, ns, name, sub, q):
        ctype = (self.headers.get("Content-Type") or "").split(";")[0].strip()
        if ctype not in ("application/merge-patch+json", "application/strategic-merge-patch+json",
                         "application/json"):
            return self._status(415, "UnsupportedMediaType", f"patch type {ctype}")
        self._send(200, self.api.cluster.patch(kind, name, self._body(), ns))

    def _delete(self, kind, ns, name, sub, q):
        self.api.cluster.delete(kind, name, ns)
        self._send(200, {"kind": "Status", "apiVersion": "v1", "status": "Success", "code": 200})


def main(argv=None):
    ap = argparse.ArgumentParser("mivgpu-e2e-apiserver")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--kubeconfig-out", required=True)
    a = ap.parse_args(argv)
    srv = FakeApiServer(port=a.port).start()
    srv.write_kubeconfig(a.kubeconfig_out)
    print(srv.url, flush=True)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        srv.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
