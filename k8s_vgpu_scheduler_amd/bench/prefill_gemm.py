"""Prefill GEMM microbenchmark: the hand-written kernel on the packed weight
(csrc/ops/prefill_gemm.hip) against the library path it replaces (unpack the
packed weight into a scratch copy, hipBLASLt via F.linear, SiLU*up pass).

Qwen3-8B projections (qkv 6144x4096, o 4096x4096, gate_up 2x12288x4096 with
SiLU*up, down 4096x12288) at prompt lengths M:

    python -m k8s_vgpu_scheduler_amd.bench.prefill_gemm --rows 2048,8192 --out x.json
"""

from __future__ import annotations

import argparse
import json
import time

import torch

SHAPES = {"qkv": (6144, 4096, False), "o_proj": (4096, 4096, False), "gate_up": (24576, 4096, True),
          "down": (4096, 12288, False)}


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
    ap.add_argument("--rows", default="2048,8192")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    ops.require_native()
    rows = []
    for M in (int(v) for v in a.rows.split(",") if v):
        for name, (N, K, silu) in SHAPES.items():
            x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
            w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
            pl = ops.PackedLinear(w, silu_mul=silu)
            flops = 2.0 * M * N * K
            tn = _time(lambda: ops.prefill_gemm(pl.wp, x, N, K, silu_mul=silu), a.reps)

            def lib_path():
                wu = ops.unpack_weight(pl.wp, N, K, ops.unpack_scratch(N * K, x.device), deinterleave=silu)
                y = torch.nn.functional.linear(x, wu)
                return ops.silu_mul(y) if silu else y
            tl = _time(lib_path, a.reps)
            wu = ops.unpack_weight(pl.wp, N, K, ops.unpack_scratch(N * K, x.device), deinterleave=silu)
            tg = _time(lambda: torch.nn.functional.linear(x, wu), a.reps)
            row = {"M": M, "proj": name, "N": N, "K": K, "native_us": round(tn * 1e6, 1),
                   "native_tflops": round(flops / tn / 1e12, 1), "lib_path_us": round(tl * 1e6, 1),
                   "hipblaslt_gemm_only_us": round(tg * 1e6, 1), "hipblaslt_tflops": round(flops / tg / 1e12, 1),
                   "speedup_vs_lib_path": round(tl / tn, 3)}
            rows.append(row)
            print(json.dumps(row), flush=True)
            del x, w, pl, wu
            torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
