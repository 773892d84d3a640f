"""Wide skinny GEMM plans at prompt row counts (M = 96 / 128): waves per
workgroup x inter-workgroup split, Qwen3-8B gate_up / down / qkv / o_proj,
against the auto plan and hipBLASLt.  One JSON line per shape."""
import json

import torch

from k8s_vgpu_scheduler_amd import ops
from k8s_vgpu_scheduler_amd.bench.gemm import SHAPES, _time

ops.require_native()
res = []
for name in ("gate_up", "down", "qkv", "o_proj"):
    N, K, silu = SHAPES[name]
    ws = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(max(1, -(-768 * 2 ** 20 // (N * K * 2))))]
    lins = [ops.PackedLinear(w, silu_mul=silu) for w in ws]
    nc = len(ws)
    for M in (96, 128):
        x = torch.randn(M, K, device="cuda").bfloat16()
        out = torch.empty(M, lins[0].out_features, device="cuda", dtype=torch.bfloat16)
        row = {"shape": name, "M": M, "cus": ops.visible_cus(),
               "auto_us": round(_time(lambda i: lins[i % nc](x, out=out), 20), 1)}
        for wv in (2, 4, 8):
            for S in (1, 2, 4):
                pl = ops.skinny_plan(M, K, N, lins[0].epi, 0, wv, S, ops.VARIANT_WIDE)
                if pl["variant"] != ops.VARIANT_WIDE or pl["ks"] != wv or pl["S"] != S:
                    continue
                for l in lins:
                    l._ensure_scratch(pl["scratch_floats"], pl["tickets"], x.device)
                try:
                    row[f"wv{wv}_S{S}"] = round(_time(lambda i: lins[i % nc](x, out=out, ks=wv, S=S,
                                                                              variant=ops.VARIANT_WIDE), 20), 1)
                except RuntimeError as e:
                    row[f"wv{wv}_S{S}"] = str(e)[:30]
        print(json.dumps(row), flush=True)
        res.append(row)
    del ws, lins
    torch.cuda.empty_cache()
