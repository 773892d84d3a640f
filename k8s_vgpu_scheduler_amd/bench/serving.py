"""Serving benchmark: TTFT and per-token latency of the OpenAI-compatible
server natively vs inside vGPU slices (the reference's
benchmarks/deployments/job-on-hami.yml vs job-on-nvidia-device-plugin.yml,
run as processes on one MI355X instead of pods).

Each configuration starts ``serve.server`` in its own process with exactly the
environment a pod would get (libmivgpu.so preloaded, the grant in a limits
file, HSA_CU_MASK / queue count for CU slices), waits for /health, drives it
with ``serve.client`` (sequential streaming requests, warmup then timed runs),
stops it, and ``serve.report`` compares every configuration with the first.

    python -m k8s_vgpu_scheduler_amd.bench.serving --configs native,vgpu50,slice25 \\
        --warmup 30 --runs 200 --out-dir gpurun_out/serving

Configurations:
  native    no shim, whole GPU
  vgpu50    shim, gpumem 50 % of the card (the reference's job-on-hami.yml), all CUs
  slice25   shim, gpucores 25: 64-CU balanced mask + 2 HW queues, gpumem 36 GiB
  slice50   shim, gpucores 50: 128-CU mask, gpumem 72 GiB
  temporal25 shim, gpucores 25 time-sliced by the governor (no mask, policy force, 2 HW queues)
A ``+K`` suffix (``slice25+3``, ``native+3``) runs K busy Qwen3-8B decode
tenants (batch 32) next to the server for that configuration: in the other CU
partitions of a 4-way split for slice configs (shim, 36 GiB grants, as pods),
governed at the same limit for the temporal config, unpartitioned without the
vGPU layer otherwise (a plain time-shared GPU).
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time
from pathlib import Path

from k8s_vgpu_scheduler_amd.bench.slices import SliceProc, SliceSpec, plan_slices, slice_env
from k8s_vgpu_scheduler_amd.serve import client, report

CARD_MIB = 288 * 1024     # MI355X HBM3E

CONFIGS = {
    "native": SliceSpec(index=0, gpumem_mib=None, cu_ranges=None, shim=False),
    "vgpu50": SliceSpec(index=1, gpumem_mib=CARD_MIB // 2, cu_ranges=None),
    "slice25": SliceSpec(index=2, gpumem_mib=36864, cu_ranges=[(0, 63)], core_pct=25, hw_queues=2),
    "slice50": SliceSpec(index=3, gpumem_mib=73728, cu_ranges=[(0, 127)], core_pct=50, hw_queues=2),
    # 2 HW queues: what the device plugin grants a shared pod (--hw-queues)
    "temporal25": SliceSpec(index=4, gpumem_mib=36864, cu_ranges=None, core_pct=25, policy="force", hw_queues=2),
}


def _nb_ok(name: str) -> bool:
    _, _, nb = name.partition("+")
    return not nb or (nb.isdigit() and int(nb) <= 3)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _log(msg):
    print(msg, flush=True)


infos: dict = {}     # config -> the server's /health (visible device memory, context length)


def neighbour_specs(spec: SliceSpec, k: int) -> list[SliceSpec]:
    """k busy tenants next to the server: in the other CU partitions of a
    4-way split when the server has one (each with the shim and a 36 GiB
    grant, as pods), else unpartitioned processes without the shim (plain
    time-shared GPU, no vGPU layer)."""
    if spec.cu_ranges:
        own = spec.cu_ranges[0][0]
        others = [s for s in plan_slices(4, shim=True, gpumem_mib=36864) if s.cu_ranges[0][0] != own]
        out = others[:k]
    elif spec.shim and spec.core_pct < 100:
        # a time-sliced server: the neighbours are governed the same way
        out = [SliceSpec(index=0, gpumem_mib=36864, cu_ranges=None, core_pct=spec.core_pct, policy=spec.policy,
                         hw_queues=spec.hw_queues) for _ in range(k)]
    else:
        out = [SliceSpec(index=0, gpumem_mib=None, cu_ranges=None, shim=False) for _ in range(k)]
    for i, s in enumerate(out):
        s.index = 20 + i
    return out


def start_neighbours(name, spec, a, workdir: Path, log=_log) -> list:
    procs = []
    args = ["--model", a.neighbour_model, "--batch", "32", "--ctx", "1024", "--steps", "64", "--loop"]
    if a.device == "cpu":
        args += ["--device", "cpu"]
    for s in neighbour_specs(spec, a.neighbours):
        procs.append(SliceProc(s, slice_env(s, None, workdir), args, workdir / f"{name}.neighbour{s.index}.log"))
    for p in procs:
        p.send("LOAD")
    for p in procs:
        p.expect("READY", a.load_timeout)
    for p in procs:
        p.send("GO")
    kind = ("CU partitions" if spec.cu_ranges else
            f"governed at {spec.core_pct} %" if spec.shim and spec.core_pct < 100 else "unpartitioned, no shim")
    log(f"[serving] {name}: {len(procs)} busy neighbours ({kind})")
    return procs


def stop_neighbours(procs) -> list[dict]:
    done = []
    for p in procs:
        try:
            p.send("STOP")
            done.append(p.expect("DONE", 120))
        except (OSError, RuntimeError, TimeoutError) as e:
            done.append({"error": str(e)})
        p.close(timeout=60)
    return done


def run_config(name: str, spec: SliceSpec, a, workdir: Path, log=_log) -> list[dict]:
    if getattr(a, "neighbours", 0):
        nb = start_neighbours(name, spec, a, workdir, log)
        try:
            return _run_server(name, spec, a, workdir, log)
        finally:
            neighbours_done[name] = stop_neighbours(nb)
    return _run_server(name, spec, a, workdir, log)


neighbours_done: dict = {}
long_ttft: dict = {}      # config -> TTFT of the long prompt (--long-prompt-tokens)


def _run_server(name: str, spec: SliceSpec, a, workdir: Path, log=_log) -> list[dict]:
    env = dict(os.environ)
    env.update(slice_env(spec, None, workdir))
    env["PYTHONPATH"] = os.pathsep.join(p for p in (str(Path(__file__).resolve().parents[2]),
                                                    env.get("PYTHONPATH")) if p)
    port = free_port()
    cmd = [sys.executable, "-u", "-m", "k8s_vgpu_scheduler_amd.serve.server", "--model", a.model,
           "--port", str(port), "--max-model-len", str(a.max_model_len), "--max-tokens", str(a.max_tokens)]
    if a.device:
        cmd += ["--device", a.device]
    if a.no_graph:
        cmd.append("--no-graph")
    if a.gpu_memory_utilization:
        cmd += ["--gpu-memory-utilization", str(a.gpu_memory_utilization)]
    logf = open(workdir / f"{name}.server.log", "w")
    proc = subprocess.Popen(cmd, env=env, stdout=logf, stderr=subprocess.STDOUT, start_new_session=True)
    url = f"http://127.0.0.1:{port}/v1/chat/completions"
    try:
        info = client.wait_ready(url, timeout=a.load_timeout, proc=proc)
        log(f"[serving] {name}: ready in {info.get('load_s')} s (device memory {info.get('device_mem_total_mib')} MiB, "
            f"max_model_len {info.get('max_model_len')}), {a.warmup} warmup + {a.runs} runs")
        infos[name] = info
        rows = client.run(url, a.runs, a.warmup, a.prompt, a.max_tokens, str(workdir / f"{name}.jsonl"),
                          timeout=a.request_timeout, log=lambda m: log(f"[serving] {name}:{m}"))
        n_long = getattr(a, "long_prompt_tokens", 0)
        if n_long:
            # a long prompt through the flash prefill: TTFT at the reference's
            # context length (the chat template adds ~20 tokens)
            words = ("lorem ipsum dolor sit amet " * (n_long // 27 + 2))[:max(1, n_long - 32)]
            long_rows = client.run(url, a.long_runs, 1, words, 4, str(workdir / f"{name}.long.jsonl"),
                                   timeout=max(a.request_timeout, 120.0), log=None)
            ttfts = sorted((r["t_first"] - r["t0"]) * 1e3 for r in long_rows if r.get("t_first"))
            long_ttft[name] = {"prompt_chars": len(words), "runs": len(ttfts),
                               "ttft_ms_p50": round(ttfts[len(ttfts) // 2], 2) if ttfts else None,
                               "ttft_ms_min": round(ttfts[0], 2) if ttfts else None,
                               "ttft_ms_max": round(ttfts[-1], 2) if ttfts else None}
            log(f"[serving] {name}: long prompt TTFT {long_ttft[name]}")
    finally:
        if proc.poll() is None:
            os.killpg(proc.pid, signal.SIGTERM)
            try:
                proc.wait(timeout=60)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
                proc.wait()
        logf.close()
    if not rows or any(r.get("t_first") is None for r in rows):
        tail = (workdir / f"{name}.server.log").read_text()[-3000:]
        raise RuntimeError(f"{name}: {sum(r.get('t_first') is None for r in rows)} of {len(rows)} requests "
                           f"streamed no token; server log tail:\n{tail}")
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--configs", default="native,vgpu50,slice25")
    ap.add_argument("--model", default="qwen3-8b")
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--runs", type=int, default=200)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--max-model-len", type=int, default=8192,
                    help="the reference's vLLM --max-model-len (benchmarks/ai-benchmark/Dockerfile:7-9)")
    ap.add_argument("--long-prompt-tokens", type=int, default=0,
                    help="after the timed runs, TTFT of a prompt of about this many tokens (e.g. 8000; the "
                         "byte tokenizer: one token per prompt character), --long-runs times")
    ap.add_argument("--long-runs", type=int, default=5)
    ap.add_argument("--prompt", default=client.DEFAULT_PROMPT)
    ap.add_argument("--device", default=None)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--gpu-memory-utilization", type=float, default=None)
    ap.add_argument("--neighbours", type=int, default=0,
                    help="busy Qwen3 decode tenants next to the server during each configuration: in the other "
                         "CU partitions for slice configs, unpartitioned (no vGPU layer) otherwise")
    ap.add_argument("--neighbour-model", default="qwen3-8b")
    ap.add_argument("--load-timeout", type=float, default=600.0)
    ap.add_argument("--request-timeout", type=float, default=60.0)
    ap.add_argument("--out-dir", default=None)
    a = ap.parse_args(argv)
    names = [n.strip() for n in a.configs.split(",") if n.strip()]
    unknown = [n for n in names if n.split("+")[0] not in CONFIGS or not _nb_ok(n)]
    if unknown:
        ap.error(f"unknown configs {unknown}; choose from {sorted(CONFIGS)}")
    default_nb = a.neighbours
    workdir = Path(a.out_dir or tempfile.mkdtemp(prefix="mivgpu-serving-"))
    workdir.mkdir(parents=True, exist_ok=True)
    results = {}
    t0 = time.time()
    for n in names:
        base, _, nb = n.partition("+")
        a.neighbours = int(nb) if nb else default_nb
        results[n] = run_config(n, CONFIGS[base], a, workdir)
        s = report.summarize(results[n])
        print(json.dumps({"config": n, "ttft_p50_ms": round(s["ttft_p50_s"] * 1e3, 3),
                          "per_token_clean_mean_ms": round(s["per_token_clean_mean_s"] * 1e3, 4),
                          "decode_tok_s": round(s["decode_tok_s"], 1)}), flush=True)
    summary = report.write_report(results, workdir)
    for n, info in infos.items():
        if n in summary:
            summary[n]["device_mem_total_mib"] = info.get("device_mem_total_mib")
            summary[n]["max_model_len"] = info.get("max_model_len")
    for n, d in neighbours_done.items():
        if n in summary:
            summary[n]["neighbours"] = d
    for n, d in long_ttft.items():
        if n in summary:
            summary[n]["long_prompt"] = d
    (workdir / "summary.json").write_text(json.dumps(summary, indent=1))
    line = {"metric": "serving TTFT / per-token latency, vGPU slices vs native", "model": a.model,
            "neighbours_default": default_nb,
            "runs": a.runs, "warmup": a.warmup, "max_tokens": a.max_tokens, "data": "synthetic prompt, random-init "
            "weights", "wall_s": round(time.time() - t0, 1), "configs": summary, "out_dir": str(workdir)}
    (workdir / "serving.json").write_text(json.dumps(line, indent=1))
    print(json.dumps(line))
    return 0


if __name__ == "__main__":
    sys.exit(main())
