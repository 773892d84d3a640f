"""Serving path (serve/): prefill numerics against teacher-forced decode, the
OpenAI-compatible server + streaming client + report on a tiny model on the
CPU, and the native-vs-slice orchestrator (bench/serving.py) end to end.
The reference's benchmark is the client/report pair of
benchmarks/ai-benchmark (benchmark.py:11-105, gen_report.py:25-201)."""

from __future__ import annotations

import http.client
import json
import threading

import numpy as np
import pytest
import torch

from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_TINY, Qwen3Decoder
from k8s_vgpu_scheduler_amd.serve import client, report
from k8s_vgpu_scheduler_amd.serve.engine import ByteTokenizer, Engine
from k8s_vgpu_scheduler_amd.serve.server import make_server


def test_prefill_matches_teacher_forced_decode():
    """Prefill of L prompt tokens == L decode steps fed the same tokens: same
    last logits, same KV cache rows, same next position."""
    torch.manual_seed(0)
    prompt = torch.randint(0, QWEN3_TINY.vocab, (37,)).tolist()
    a = Qwen3Decoder(QWEN3_TINY, batch=1, max_ctx=96, device="cpu")
    la = a.prefill(prompt).float()
    b = Qwen3Decoder(QWEN3_TINY, batch=1, max_ctx=96, device="cpu")
    for t in prompt:
        b.tokens[0] = t
        lb = b.step()[0].float()
    torch.testing.assert_close(la, lb, atol=2e-2, rtol=2e-2)
    assert int(a.tokens[0]) == int(torch.argmax(lb))
    assert int(a.pos[0]) == int(b.pos[0]) == len(prompt) and int(a.seqlens[0]) == int(b.seqlens[0])
    for li in range(QWEN3_TINY.layers):
        # bf16 cache entries: a couple of ulps apart (GEMM row blocking differs)
        torch.testing.assert_close(a.k_cache[li][0, :, :37].float(), b.k_cache[li][0, :, :37].float(),
                                   atol=5e-2, rtol=2e-2)
        torch.testing.assert_close(a.v_cache[li][0, :, :37].float(), b.v_cache[li][0, :, :37].float(),
                                   atol=5e-2, rtol=2e-2)
    # decoding continues identically from either state
    a.step()
    b.step()
    assert int(a.tokens[0]) == int(b.tokens[0])


def test_prefill_rejects_oversized_prompt():
    d = Qwen3Decoder(QWEN3_TINY, batch=1, max_ctx=64, device="cpu")
    with pytest.raises(ValueError):
        d.prefill(list(range(64)))


def test_byte_tokenizer_chat_template():
    t = ByteTokenizer(QWEN3_TINY.vocab)
    ids = t.chat([{"role": "user", "content": "hi"}])
    assert ids[0] == t.SPECIALS["<|im_start|>"] and ids.count(t.SPECIALS["<|im_end|>"]) == 1
    assert t.encode("hi") == [ord("h") + 3, ord("i") + 3]
    assert all(0x20 <= ord(t.decode_one(x)) < 0x7f for x in range(0, 5000, 7))


@pytest.fixture(scope="module")
def server():
    eng = Engine("qwen3-tiny", max_ctx=256, device="cpu")
    srv = make_server(eng, port=0, default_max_tokens=8)
    th = threading.Thread(target=srv.serve_forever, kwargs={"poll_interval": 0.05}, daemon=True)
    th.start()
    yield f"http://127.0.0.1:{srv.server_address[1]}", eng
    srv.shutdown()
    srv.server_close()


def _req(base, method, path, body=None):
    host, port = base.split("//")[1].split(":")
    c = http.client.HTTPConnection(host, int(port), timeout=30)
    c.request(method, path, json.dumps(body) if body is not None else None,
              {"Content-Type": "application/json"} if body is not None else {})
    r = c.getresponse()
    return r.status, r.read()


def test_server_routes(server):
    base, eng = server
    st, body = _req(base, "GET", "/health")
    assert st == 200 and json.loads(body)["model"] == "Qwen3-tiny"
    st, body = _req(base, "GET", "/v1/models")
    assert st == 200 and json.loads(body)["data"][0]["max_model_len"] == eng.max_ctx
    st, body = _req(base, "POST", "/v1/chat/completions",
                    {"messages": [{"role": "user", "content": "hello"}], "max_tokens": 5})
    r = json.loads(body)
    assert st == 200 and r["usage"]["completion_tokens"] == 5 and len(r["choices"][0]["message"]["content"]) == 5
    st, body = _req(base, "POST", "/v1/completions", {"prompt": "abc", "max_tokens": 3})
    assert st == 200 and len(json.loads(body)["choices"][0]["text"]) == 3
    assert _req(base, "POST", "/v1/chat/completions", {"messages": []})[0] == 400
    assert _req(base, "POST", "/v1/chat/completions", {"messages": [{"content": "x" * 300}]})[0] == 400
    assert _req(base, "POST", "/v1/nope", {})[0] == 404
    assert _req(base, "GET", "/nope")[0] == 404


def test_streaming_client_and_report(server, tmp_path):
    base, eng = server
    url = base + "/v1/chat/completions"
    assert client.wait_ready(url, timeout=10)["status"] == "ok"
    rows = client.run(url, runs=4, warmup=1, max_tokens=6, output=str(tmp_path / "a.jsonl"), log=None)
    assert len(rows) == 4
    for r in rows:
        assert len(r["t_tokens"]) == 6 and r["usage"]["completion_tokens"] == 6
        assert r["t0"] <= r["t_first"] <= r["t_tokens"][-1] <= r["t_end"]
    # the same requests deterministic: greedy decoding of the same prompt
    g1 = eng.generate(eng.tok.chat([{"role": "user", "content": client.DEFAULT_PROMPT}]), 6).tokens
    g2 = eng.generate(eng.tok.chat([{"role": "user", "content": client.DEFAULT_PROMPT}]), 6).tokens
    assert g1 == g2
    rows_b = client.run(url, runs=3, warmup=0, max_tokens=6, output=str(tmp_path / "b.jsonl"), log=None)
    summary = report.write_report({"native": report.load(tmp_path / "a.jsonl"),
                                   "vgpu": report.load(tmp_path / "b.jsonl")}, tmp_path / "rep")
    assert summary["native"]["requests"] == 4 and summary["vgpu"]["requests"] == len(rows_b)
    assert summary["native"]["ttft_clean_mean_overhead_pct"] == 0.0
    assert "ttft_clean_mean_overhead_pct" in summary["vgpu"]
    assert summary["native"]["tokens_per_request"] == 6.0
    text = (tmp_path / "rep" / "report.md").read_text()
    assert "| native | 4 |" in text and "| vgpu | 3 |" in text


def test_report_statistics():
    """Percentiles on the raw data; trim + MAD filter before the clean means."""
    rows = [{"t0": 0.0, "t_first": 0.010 + 0.001 * i, "t_tokens": [0.010 + 0.001 * i + 0.002 * k for k in range(5)],
             "t_end": 1.0} for i in range(40)]
    rows.append({"t0": 0.0, "t_first": 5.0, "t_tokens": [5.0, 5.002], "t_end": 6.0})     # outlier
    rows.append({"t0": 0.0, "t_first": None, "t_tokens": [], "t_end": 1.0})             # failed request
    ttft, gaps = report.latencies(rows)
    assert ttft.size == 41 and np.allclose(gaps, 0.002)
    s = report.summarize(rows)
    assert s["ttft_p99_s"] > 1.0 > s["ttft_p50_s"]
    assert s["ttft_clean_mean_s"] < 0.06            # the 5 s outlier is gone
    assert abs(s["per_token_clean_mean_s"] - 0.002) < 1e-9


def test_serving_orchestrator_cpu(tmp_path):
    """bench/serving.py: a server process per configuration, client, report."""
    from k8s_vgpu_scheduler_amd.bench import serving
    rc = serving.main(["--configs", "native", "--model", "qwen3-tiny", "--device", "cpu", "--warmup", "1",
                       "--runs", "3", "--max-tokens", "4", "--max-model-len", "256", "--out-dir", str(tmp_path)])
    assert rc == 0
    out = json.loads((tmp_path / "serving.json").read_text())
    assert out["configs"]["native"]["requests"] == 3 and out["configs"]["native"]["tokens_per_request"] == 4.0
    assert (tmp_path / "report.md").exists() and (tmp_path / "native.jsonl").exists()


def test_serving_long_prompt_ttft_cpu(tmp_path):
    """--long-prompt-tokens: TTFT of a long prompt per configuration."""
    from k8s_vgpu_scheduler_amd.bench import serving
    rc = serving.main(["--configs", "native", "--model", "qwen3-tiny", "--device", "cpu", "--warmup", "0",
                       "--runs", "1", "--max-tokens", "2", "--max-model-len", "512", "--long-prompt-tokens", "300",
                       "--long-runs", "2", "--out-dir", str(tmp_path)])
    assert rc == 0
    lp = json.loads((tmp_path / "serving.json").read_text())["configs"]["native"]["long_prompt"]
    assert lp["runs"] == 2 and lp["ttft_ms_p50"] > 0 and 200 < lp["prompt_chars"] <= 300


def test_serving_orchestrator_with_neighbours_cpu(tmp_path):
    """``native+1``: one busy neighbour (the bench/slices child in --loop
    mode) runs while the server is measured, then stops and reports."""
    from k8s_vgpu_scheduler_amd.bench import serving
    rc = serving.main(["--configs", "native+1", "--model", "qwen3-tiny", "--device", "cpu", "--warmup", "1",
                       "--runs", "2", "--max-tokens", "3", "--max-model-len", "256", "--neighbour-model",
                       "qwen3-tiny", "--out-dir", str(tmp_path)])
    assert rc == 0
    out = json.loads((tmp_path / "serving.json").read_text())["configs"]["native+1"]
    assert out["requests"] == 2
    nb = out["neighbours"]
    assert len(nb) == 1 and nb[0].get("loop") is True and nb[0]["tokens"] > 0, nb


def test_neighbour_layouts():
    from k8s_vgpu_scheduler_amd.bench import serving
    sl = serving.neighbour_specs(serving.CONFIGS["slice25"], 3)
    assert [s.cu_ranges for s in sl] == [[(64, 127)], [(128, 191)], [(192, 255)]]
    assert all(s.shim and s.gpumem_mib == 36864 for s in sl)
    nat = serving.neighbour_specs(serving.CONFIGS["native"], 2)
    assert all(s.cu_ranges is None and not s.shim for s in nat)
    tmp = serving.neighbour_specs(serving.CONFIGS["temporal25"], 3)
    assert all(s.shim and s.cu_ranges is None and s.core_pct == 25 and s.policy == "force" for s in tmp)


def test_engine_reports_a_failed_request_and_keeps_serving():
    """A job that raises on the engine thread (here: a prompt id outside the
    vocabulary) reaches its request as an exception; the next request works."""
    eng = Engine("qwen3-tiny", max_ctx=128, device="cpu")
    try:
        with pytest.raises(Exception):
            list(eng.stream([10 ** 9], 3))
        assert len(eng.generate(eng.tok.encode("ok"), 3).tokens) == 3
    finally:
        eng.close()
    with pytest.raises(RuntimeError, match="engine thread"):
        list(eng.stream([5, 6], 2))
