"""Single-process decode benchmark (one slice, no orchestration) for profiling.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- \
        python -m k8s_vgpu_scheduler_amd.bench.decode --batch 32 --steps 20
"""

from __future__ import annotations

import argparse
import json
import time

import torch

from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_8B, QWEN3_TINY, Qwen3Decoder


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-8b", choices=["qwen3-8b", "qwen3-tiny"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--gemm", default="auto", choices=["auto", "skinny", "hipblaslt"])
    a = ap.parse_args()
    cfg = QWEN3_8B if a.model == "qwen3-8b" else QWEN3_TINY
    skinny = {"auto": None, "skinny": True, "hipblaslt": False}[a.gemm]
    dec = Qwen3Decoder(cfg, batch=a.batch, max_ctx=a.ctx + a.steps + a.warmup + 16, skinny=skinny)
    dec.fill_context(a.ctx)
    if not a.no_graph:
        dec.capture(warmup=1)
    for _ in range(a.warmup):
        dec.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        dec.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    weight_bytes = cfg.param_count() * 2
    kv_bytes = 2 * cfg.layers * a.batch * cfg.kv_heads * (a.ctx + a.warmup + a.steps // 2) * cfg.head_dim * 2
    gave_up = bool(dec._chains and dec._chains[0].gave_up())
    print(json.dumps({"batch": a.batch, "ctx": a.ctx, "skinny_gemm": dec.skinny, "chain": dec.chain,
                      "chain_w": dec.chain_w if dec.chain else None, "chain_gave_up": gave_up,
                      "ms_per_step": dt / a.steps * 1e3,
                      "tok_s": a.batch * a.steps / dt,
                      "hbm_gbps_lower_bound": (weight_bytes + kv_bytes) * a.steps / dt / 1e9}))


if __name__ == "__main__":
    main()
