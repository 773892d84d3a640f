"""Prompt-sized projection GEMMs on hipBLASLt: weight [N, K] (F.linear, the
current layout) vs a [K, N] copy (torch.mm, no transpose), M = 8192 rows."""
import json

import torch
import torch.nn.functional as F

M = 8192
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gu": (24576, 4096), "down": (4096, 12288)}
out = {}
for name, (N, K) in shapes.items():
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    wt = w.t().contiguous()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    res = {}
    for tag, fn in (("linear_NK", lambda: F.linear(x, w)), ("mm_KN", lambda: torch.mm(x, wt, out=y)),
                    ("mm_NK_t", lambda: torch.mm(x, w.t(), out=y))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        res[tag] = {"us": round(ms * 1e3, 1), "tflops": round(2 * M * N * K / ms / 1e9, 1)}
    out[name] = res
    print(name, json.dumps(res), flush=True)
