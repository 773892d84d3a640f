"""OpenAI-compatible HTTP server over serve.engine (the vllm-openai server of
the reference's benchmark pod, benchmarks/ai-benchmark/Dockerfile).

  GET  /health                 200 once the model is loaded
  GET  /v1/models              the served model
  POST /v1/chat/completions    {"messages": [...], "stream": bool, "max_tokens": n}
  POST /v1/completions         {"prompt": "...", "stream": bool, "max_tokens": n}

Streaming responses are server-sent events, one ``data: {chunk}`` line per
generated token, a final chunk carrying ``finish_reason`` and ``usage``, then
``data: [DONE]``; the connection closes after each response.  Requests are
served one at a time, in arrival order, by the engine thread that owns the
GPU; further clients wait.

    python -m k8s_vgpu_scheduler_amd.serve.server --model qwen3-8b --port 8000
"""

from __future__ import annotations

import argparse
import json
import sys
import time
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from k8s_vgpu_scheduler_amd.serve.engine import MODELS, Engine

MAX_BODY = 1 << 20


class Handler(BaseHTTPRequestHandler):
    engine: Engine = None            # set by make_server
    default_max_tokens = 128
    protocol_version = "HTTP/1.0"    # one response per connection; SSE ends at close

    def log_message(self, fmt, *args):   # quiet: the benchmark measures latency
        pass

    def _json(self, code: int, obj):
        body = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def do_GET(self):
        if self.path == "/health":
            return self._json(200, {"status": "ok", "model": self.engine.model_name,
                                    "load_s": round(self.engine.load_s, 2), "max_model_len": self.engine.max_ctx,
                                    "device_mem_total_mib": self.engine.mem_total_mib})
        if self.path == "/v1/models":
            return self._json(200, {"object": "list", "data": [{"id": self.engine.model_name, "object": "model",
                                                                 "max_model_len": self.engine.max_ctx}]})
        self._json(404, {"error": {"message": f"no route {self.path}"}})

    def do_POST(self):
        n = int(self.headers.get("Content-Length") or 0)
        if n > MAX_BODY:
            return self._json(413, {"error": {"message": "request body too large"}})
        try:
            req = json.loads(self.rfile.read(n) or b"{}")
        except ValueError:
            return self._json(400, {"error": {"message": "body is not JSON"}})
        tok = self.engine.tok
        if self.path == "/v1/chat/completions":
            msgs = req.get("messages")
            if not isinstance(msgs, list) or not msgs:
                return self._json(400, {"error": {"message": "messages must be a non-empty list"}})
            ids, kind = tok.chat(msgs), "chat.completion"
        elif self.path == "/v1/completions":
            ids, kind = tok.encode(str(req.get("prompt", ""))), "text_completion"
        else:
            return self._json(404, {"error": {"message": f"no route {self.path}"}})
        if not ids or len(ids) >= self.engine.max_ctx:
            return self._json(400, {"error": {"message": f"prompt of {len(ids)} tokens does not fit "
                                                         f"max_model_len {self.engine.max_ctx}"}})
        max_tokens = int(req.get("max_tokens") or req.get("max_completion_tokens") or self.default_max_tokens)
        rid = f"{'chatcmpl' if kind.startswith('chat') else 'cmpl'}-{uuid.uuid4().hex[:24]}"
        created = int(time.time())
        model = req.get("model") or self.engine.model_name

        def choice(text, finish=None):
            if kind == "chat.completion":
                return {"index": 0, "delta": {"content": text} if text else {}, "finish_reason": finish}
            return {"index": 0, "text": text, "finish_reason": finish}

        if not req.get("stream"):
            gen = self.engine.generate(ids, max_tokens)
            text = "".join(tok.decode_one(t) for t in gen.tokens)
            ch = ({"index": 0, "message": {"role": "assistant", "content": text}, "finish_reason": "length"}
                  if kind == "chat.completion" else {"index": 0, "text": text, "finish_reason": "length"})
            return self._json(200, {"id": rid, "object": kind, "created": created, "model": model, "choices": [ch],
                                    "usage": {"prompt_tokens": len(ids), "completion_tokens": len(gen.tokens),
                                              "total_tokens": len(ids) + len(gen.tokens)}})
        self.send_response(200)
        self.send_header("Content-Type", "text/event-stream")
        self.send_header("Cache-Control", "no-cache")
        self.end_headers()
        obj = kind + ".chunk" if kind == "chat.completion" else kind
        done = 0
        try:
            for t in self.engine.stream(ids, max_tokens):
                done += 1
                self.wfile.write(b"data: " + json.dumps({"id": rid, "object": obj, "created": created, "model": model,
                                                          "choices": [choice(tok.decode_one(t))]}).encode() + b"\n\n")
                self.wfile.flush()
            final = {"id": rid, "object": obj, "created": created, "model": model, "choices": [choice("", "length")],
                     "usage": {"prompt_tokens": len(ids), "completion_tokens": done,
                               "total_tokens": len(ids) + done}}
            self.wfile.write(b"data: " + json.dumps(final).encode() + b"\n\ndata: [DONE]\n\n")
            self.wfile.flush()
        except (BrokenPipeError, ConnectionResetError):
            pass       # client went away: the generator's close releases the engine


def make_server(engine: Engine, host: str = "127.0.0.1", port: int = 8000, default_max_tokens: int = 128):
    handler = type("BoundHandler", (Handler,), {"engine": engine, "default_max_tokens": default_max_tokens})
    srv = ThreadingHTTPServer((host, port), handler)
    srv.daemon_threads = True
    return srv


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--model", default="qwen3-8b", choices=sorted(MODELS))
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--max-model-len", type=int, default=8192,
                    help="context length (the reference benchmark's vLLM --max-model-len 8192)")
    ap.add_argument("--max-tokens", type=int, default=128, help="default completion length")
    ap.add_argument("--no-graph", action="store_true", help="eager decode steps instead of hipGraph replays")
    ap.add_argument("--device", default=None)
    ap.add_argument("--gpu-memory-utilization", type=float, default=None,
                    help="size max_model_len to this fraction of the device memory the process sees "
                         "(the slice's grant under libmivgpu.so), capped by --max-model-len")
    a = ap.parse_args(argv)
    eng = Engine(a.model, max_ctx=a.max_model_len, device=a.device, graph=not a.no_graph,
                 gpu_memory_utilization=a.gpu_memory_utilization)
    srv = make_server(eng, a.host, a.port, a.max_tokens)
    print(json.dumps({"serving": eng.model_name, "url": f"http://{a.host}:{srv.server_address[1]}",
                      "load_s": round(eng.load_s, 2), "graph": eng.graph, "max_model_len": eng.max_ctx,
                      "device_mem_total_mib": eng.mem_total_mib}), flush=True)
    try:
        srv.serve_forever(poll_interval=0.2)
    except KeyboardInterrupt:
        pass
    finally:
        srv.server_close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
