"""HTTP(S) front end of the extender (pkg/scheduler/routes/route.go:51-186, cmd/scheduler/main.go:145-156).

Routes: POST /filter, POST /bind, POST /webhook, GET /healthz, GET /readyz and,
behind --profiling, GET /debug/pprof/ (Python stack dump + tracemalloc top).
Bodies are capped at 1 MiB; /filter waits for the scheduler's cache sync.
A ThreadingHTTPServer serves concurrent kube-scheduler calls; TLS via the
stdlib ssl module with cert/key reloaded on change (the reference's cert
watcher).
"""

from __future__ import annotations

import json
import logging
import os
import ssl
import sys
import threading
import traceback
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

log = logging.getLogger(__name__)
MAX_BODY = 1024 * 1024
DRAIN_LIMIT = 16 * MAX_BODY   # oversized bodies up to this are drained before the 413


def make_handler(scheduler, webhook, profiling: bool = False):
    class Handler(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, fmt, *args):  # route access logs to logging
            log.debug("%s - %s", self.address_string(), fmt % args)

        def _json(self, code: int, obj):
            body = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def _text(self, code: int, text: str):
            body = text.encode()
            self.send_response(code)
            self.send_header("Content-Type", "text/plain")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def _body(self):
            """Request body, None when absent; b"" marks one over the 1 MiB cap
            (route.go's MaxBytesReader).  A moderately oversized body is read
            and discarded so the client, still sending, gets the 413 instead
            of a broken pipe; either way the connection closes after the reply."""
            try:
                n = int(self.headers.get("Content-Length") or 0)
            except ValueError:
                n = 0
            if n <= 0:
                return None
            if n > MAX_BODY:
                self.close_connection = True
                if n <= DRAIN_LIMIT:
                    left = n
                    while left > 0:
                        chunk = self.rfile.read(min(left, 1 << 16))
                        if not chunk:
                            break
                        left -= len(chunk)
                return b""
            return self.rfile.read(n)

        def do_GET(self):  # noqa: N802
            if self.path == "/healthz":
                return self._text(200, "")
            if self.path == "/readyz":
                return self._text(200, "leader" if scheduler.leader.is_leader() else "follower")
            if profiling and self.path.startswith("/debug/pprof"):
                out = []
                for tid, frame in sys._current_frames().items():
                    out.append(f"--- thread {tid}\n" + "".join(traceback.format_stack(frame)))
                return self._text(200, "\n".join(out))
            return self._text(404, "not found")

        def do_POST(self):  # noqa: N802
            raw = self._body()
            if raw is None:
                return self._text(400, "Please send a request body")
            if raw == b"":
                return self._text(413, "request body too large")
            try:
                args = json.loads(raw)
            except ValueError as e:
                if self.path == "/bind":
                    return self._json(200, {"Error": str(e)})
                return self._json(200, {"Error": str(e)})
            if self.path == "/filter":
                if not (args.get("Pod") or args.get("pod")):
                    return self._json(200, {"Error": "extender args missing pod"})
                if not scheduler.wait_for_cache_sync(timeout=30):
                    return self._json(200, {"Error": "context cancelled"})
                try:
                    return self._json(200, scheduler.filter(args))
                except Exception as e:  # noqa: BLE001
                    log.exception("filter failed")
                    return self._json(200, {"Error": str(e)})
            if self.path == "/bind":
                try:
                    return self._json(200, scheduler.bind(args))
                except Exception as e:  # noqa: BLE001
                    log.exception("bind failed")
                    return self._json(200, {"Error": str(e)})
            if self.path == "/webhook":
                return self._json(200, webhook.handle_review(args))
            return self._text(404, "not found")

    return Handler


class ExtenderServer:
    def __init__(self, scheduler, webhook, bind: str = "127.0.0.1:8080", cert: str = "", key: str = "",
                 profiling: bool = False):
        host, _, port = bind.rpartition(":")
        self.httpd = ThreadingHTTPServer((host or "0.0.0.0", int(port)), make_handler(scheduler, webhook, profiling))
        self.cert, self.key = cert, key
        self._mtime = None
        if cert and key:
            self._ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            self._load()
            self.httpd.socket = self._ctx.wrap_socket(self.httpd.socket, server_side=True)
        self.thread = None

    def _load(self):
        self._ctx.load_cert_chain(self.cert, self.key)
        self._mtime = (os.path.getmtime(self.cert), os.path.getmtime(self.key))

    def maybe_reload_cert(self):
        """Cert watcher: reload when the mounted secret rotates."""
        if not (self.cert and self.key):
            return False
        m = (os.path.getmtime(self.cert), os.path.getmtime(self.key))
        if m != self._mtime:
            self._load()
            return True
        return False

    @property
    def port(self) -> int:
        return self.httpd.server_address[1]

    def start(self):
        self.thread = threading.Thread(target=self.httpd.serve_forever, name="extender-http", daemon=True)
        self.thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()
