"""Streaming latency client: TTFT and per-token timestamps per request
(the measurement of the reference's benchmarks/ai-benchmark/benchmark.py:11-105,
same JSONL row schema -- t0, t_first, t_tokens, t_end, usage -- so results
from either harness feed serve/report.py).

    python -m k8s_vgpu_scheduler_amd.serve.client --url http://127.0.0.1:8000 \\
        --warmup 30 --runs 200 --output native.jsonl
"""

from __future__ import annotations

import argparse
import http.client
import json
import sys
import time
from urllib.parse import urlparse

DEFAULT_PROMPT = "Explain the difference between supervised and unsupervised learning."


def stream_request(url: str, prompt: str, model: str | None = None, max_tokens: int | None = None,
                   timeout: float = 60.0) -> dict:
    """One streaming chat completion; timestamps each SSE data chunk on arrival."""
    u = urlparse(url)
    path = u.path if u.path and u.path != "/" else "/v1/chat/completions"
    body = {"messages": [{"role": "user", "content": prompt}], "stream": True}
    if model:
        body["model"] = model
    if max_tokens:
        body["max_tokens"] = max_tokens
    conn = http.client.HTTPConnection(u.hostname, u.port or 80, timeout=timeout)
    t0 = time.time()
    conn.request("POST", path, json.dumps(body), {"Content-Type": "application/json"})
    resp = conn.getresponse()
    if resp.status != 200:
        raise RuntimeError(f"HTTP {resp.status}: {resp.read()[:500]!r}")
    t_first, stamps, usage = None, [], None
    while True:
        line = resp.readline()
        if not line:
            break
        line = line.strip()
        if not line.startswith(b"data:"):
            continue
        payload = line[5:].strip()
        if payload == b"[DONE]":
            break
        now = time.time()
        try:
            chunk = json.loads(payload)
        except ValueError:
            continue
        if chunk.get("usage"):
            usage = chunk["usage"]
        if not any((c.get("delta") or {}).get("content") or c.get("text") for c in chunk.get("choices", [])):
            continue          # the closing chunk carries no token
        if t_first is None:
            t_first = now
        stamps.append(now)
    t_end = time.time()
    conn.close()
    return {"t0": t0, "t_first": t_first, "t_tokens": stamps, "t_end": t_end, "usage": usage}


def wait_ready(url: str, timeout: float = 600.0, proc=None) -> dict:
    u = urlparse(url)
    deadline = time.time() + timeout
    last = None
    while time.time() < deadline:
        if proc is not None and proc.poll() is not None:
            raise RuntimeError(f"server exited with {proc.returncode} before it was ready")
        try:
            c = http.client.HTTPConnection(u.hostname, u.port or 80, timeout=5)
            c.request("GET", "/health")
            r = c.getresponse()
            if r.status == 200:
                return json.loads(r.read())
        except OSError as e:
            last = e
        time.sleep(0.5)
    raise TimeoutError(f"server at {url} not ready after {timeout}s ({last})")


def run(url: str, runs: int, warmup: int, prompt: str = DEFAULT_PROMPT, max_tokens: int | None = None,
        output: str | None = None, timeout: float = 60.0, log=print) -> list[dict]:
    for i in range(warmup):
        stream_request(url, prompt, max_tokens=max_tokens, timeout=timeout)
        if log and (i + 1) % 10 == 0:
            log(f"  warmup {i + 1}/{warmup}")
    rows = []
    f = open(output, "w") if output else None
    try:
        for i in range(runs):
            r = stream_request(url, prompt, max_tokens=max_tokens, timeout=timeout)
            rows.append(r)
            if f:
                f.write(json.dumps(r) + "\n")
                f.flush()
            if log and (i + 1) % 10 == 0:
                log(f"  run {i + 1}/{runs}")
    finally:
        if f:
            f.close()
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser(description="streaming TTFT / per-token latency client")
    ap.add_argument("--url", default="http://127.0.0.1:8000/v1/chat/completions")
    ap.add_argument("--prompt", default=DEFAULT_PROMPT)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--runs", type=int, default=200)
    ap.add_argument("--max-tokens", type=int, default=None)
    ap.add_argument("--timeout", type=float, default=60.0, help="seconds to wait for the next chunk")
    ap.add_argument("--output", default="bench.jsonl")
    a = ap.parse_args(argv)
    wait_ready(a.url)
    run(a.url, a.runs, a.warmup, a.prompt, a.max_tokens, a.output, a.timeout)
    print("saved:", a.output)
    return 0


if __name__ == "__main__":
    sys.exit(main())
