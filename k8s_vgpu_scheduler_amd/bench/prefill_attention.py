"""Prefill flash-attention microbenchmark (csrc/ops/prefill_attn.hip).

Qwen3-8B heads (32 query / 8 KV x 128), one sequence of L positions, causal:
useful FLOPs = 4 * D * Hq * L * (L + 1) / 2.  Against the eager path it
replaces (two batched fp32 GEMMs over the materialised L x L scores, run
where it fits in memory).

    python -m k8s_vgpu_scheduler_amd.bench.prefill_attention --lens 512,2048,8192 --out x.json
"""

from __future__ import annotations

import argparse
import json
import math
import os
import time

import torch


def _time(fn, reps: int) -> float:
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main(argv=None):
    from k8s_vgpu_scheduler_amd import ops

    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="512,2048,8192")
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--kv-heads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--eager-max", type=int, default=4096, help="largest L for the eager fp32 comparison")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    ops.require_native()
    D, Hq, Hkv = 128, a.heads, a.kv_heads
    G = Hq // Hkv
    scale = 1.0 / math.sqrt(D)
    rows = []
    for L in (int(x) for x in a.lens.split(",") if x):
        q = torch.randn(Hkv, G * L, D, device="cuda").to(torch.bfloat16)
        k = torch.randn(Hkv, L, D, device="cuda").to(torch.bfloat16)
        v = torch.randn(Hkv, L, D, device="cuda").to(torch.bfloat16)
        out = torch.empty(L, Hq * D, device="cuda", dtype=torch.bfloat16)
        flops = 4.0 * D * Hq * L * (L + 1) / 2
        t = _time(lambda: ops.prefill_attention(q, k, v, Hq, scale, out=out), a.reps)
        row = {"L": L, "heads": Hq, "kv_heads": Hkv, "flash_ms": round(t * 1e3, 3),
               "flash_tflops": round(flops / t / 1e12, 1), "cus": ops.visible_cus(),
               "vt_path": os.environ.get("MIVGPU_FA_TR", "1"), "kernel": os.environ.get("MIVGPU_FA_KERNEL", "8")}
        if L <= a.eager_max:
            i = torch.arange(L, device="cuda")
            mask = torch.zeros(L, L, device="cuda").masked_fill_(i[None, :] > i[:, None], float("-inf")).repeat(G, 1)

            def eager():
                sc = torch.baddbmm(mask.expand(Hkv, G * L, L), q.float(), k.float().transpose(1, 2), alpha=scale)
                return torch.bmm(torch.softmax(sc, dim=-1), v.float())
            te = _time(eager, max(2, a.reps // 4))
            row.update(eager_fp32_ms=round(te * 1e3, 3), speedup=round(te / t, 1))
            del mask
        rows.append(row)
        print(json.dumps(row), flush=True)
        del q, k, v, out
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
