"""Decode-attention microbenchmark (csrc/ops/model_ops.hip): the MFMA kernel
(4 / 8 waves) and the VALU kernel's load-scheduling variants, across CU
partitions.

Qwen3-8B shape: B=32 sequences, 32 query / 8 KV heads x 128, context 1024.
Each call reads K+V of one layer (134 MB); calls rotate over ``--layers`` KV
caches (>= 1 GB) so the 256 MB Infinity Cache cannot serve repeats — in a real
decode step all other layers stream in between.  Every (variant, CU mask)
runs in a child process (the variant is read once per process, and
HSA_CU_MASK must be set before HIP initialises).

    python -m k8s_vgpu_scheduler_amd.bench.attention --out gpurun_out/attn.json
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
from pathlib import Path


def child(a):
    import math

    import torch

    from k8s_vgpu_scheduler_amd import ops

    B, Hq, Hkv, D = a.batch, 32, 8, 128
    T = a.ctx + 16
    T = -(-T // 32) * 32
    ks = [ops.k_to_cache_layout(torch.randn(B, Hkv, T, D, device="cuda").bfloat16()) for _ in range(a.layers)]
    vs = [ops.v_to_cache_layout(torch.randn(B, Hkv, T, D, device="cuda").bfloat16()) for _ in range(a.layers)]
    q = torch.randn(B, Hq, D, device="cuda").bfloat16()
    seqlens = torch.full((B,), a.ctx, dtype=torch.int32, device="cuda")
    nsplit = math.ceil(T / ops.attn_split())
    out = torch.empty(B, Hq * D, device="cuda", dtype=torch.bfloat16)
    o_part = torch.empty(B * Hq * nsplit * D, device="cuda")
    ml_part = torch.empty(B * Hq * nsplit * 2, device="cuda")
    scale = 1.0 / math.sqrt(D)

    def run(i):
        ops.decode_attention(q, ks[i % a.layers], vs[i % a.layers], seqlens, out, o_part, ml_part, Hq, Hkv, D,
                             nsplit, scale)

    for i in range(3):
        run(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(a.reps):
            run(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / a.reps
    kv_bytes = 2 * B * Hkv * a.ctx * D * 2
    print(json.dumps({"kernel": os.environ.get("MIVGPU_ATTN_KERNEL", "mfma"), "split": ops.attn_split(),
                      "nt": os.environ.get("MIVGPU_ATTN_NT", "1"),
                      "pf": os.environ.get("MIVGPU_ATTN_PF", "auto"), "cu_mask": os.environ.get("HSA_CU_MASK", ""),
                      "us": round(us, 2), "kv_TBps": round(kv_bytes / us / 1e6, 3)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--reps", type=int, default=64)
    ap.add_argument("--variants", default="mfma,mfma4,valu:auto",
                    help="mfma | mfma4 | mfma:cached | mfma4:cached | valu:<pf> with pf in 0,1,2,auto")
    ap.add_argument("--masks", default=",0:0-63,0:0-31")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.child:
        return child(a)
    rows = []
    for mask in a.masks.split(","):
        for var in a.variants.split(","):
            kernel, _, opt = var.partition(":")
            env = dict(os.environ, MIVGPU_ATTN_KERNEL=kernel)
            env.pop("MIVGPU_ATTN_PF", None)
            env.pop("MIVGPU_ATTN_NT", None)
            if opt == "cached":
                env["MIVGPU_ATTN_NT"] = "0"
            elif opt and opt != "auto":     # auto = the library's own CU-aware choice
                env["MIVGPU_ATTN_PF"] = opt
            env.pop("HSA_CU_MASK", None)
            if mask:
                env["HSA_CU_MASK"] = mask
            r = subprocess.run([sys.executable, "-m", "k8s_vgpu_scheduler_amd.bench.attention", "--child",
                                "--batch", str(a.batch), "--ctx", str(a.ctx), "--layers", str(a.layers),
                                "--reps", str(a.reps)], env=env, capture_output=True, text=True, timeout=600)
            line = next((x for x in r.stdout.splitlines() if x.startswith("{")), None)
            row = json.loads(line) if line else {"variant": var, "cu_mask": mask, "error": r.stderr[-500:]}
            print(json.dumps(row), flush=True)
            rows.append(row)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
