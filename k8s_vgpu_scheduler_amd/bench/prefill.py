"""Prefill (time to first token) microbenchmark: one prompt through the
captured per-bucket prefill graph of the Qwen3 decoder, batch row 0.

    python -m k8s_vgpu_scheduler_amd.bench.prefill --len 92 --iters 20 [--eager]
Prints one JSON line (ms per prefill, tokens/s)."""

from __future__ import annotations

import argparse
import json
import time

import torch

from k8s_vgpu_scheduler_amd import ops
from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_8B, QWEN3_TINY, Qwen3Decoder


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-8b", choices=["qwen3-8b", "qwen3-tiny"])
    ap.add_argument("--len", type=int, default=92)
    ap.add_argument("--ctx", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--eager", action="store_true")
    a = ap.parse_args(argv)
    cfg = QWEN3_8B if a.model == "qwen3-8b" else QWEN3_TINY
    d = Qwen3Decoder(cfg, batch=1, max_ctx=a.ctx, device="cuda")
    if d.skinny:
        d.reserve_prefill()
    bucket = d._bucket(a.len)
    if not a.eager and bucket:
        d.capture_prefill([bucket])
    prompt = list(range(3, 3 + a.len))
    for _ in range(3):
        d.prefill(prompt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        d.prefill(prompt)
        int(d.tokens[0])          # the first token reaches the host, as in serving
    ms = (time.perf_counter() - t0) * 1e3 / a.iters
    print(json.dumps({"model": cfg.name, "prompt": a.len, "bucket": bucket, "graph": not a.eager and bool(bucket),
                      "cus": ops.visible_cus(), "ms_per_prefill": round(ms, 3),
                      "prompt_tok_s": round(a.len / ms * 1e3, 1)}))


if __name__ == "__main__":
    main()
