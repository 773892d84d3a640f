"""GPU-box probe: does a decode projection run faster when its weights were
just read into the 256 MB Infinity Cache (MALL)?

For each Qwen3-8B projection shape, times (hipGraph, --reps repetitions):
  flush             read a 1 GiB junk buffer (evicts the MALL)
  flush+gemm        the projection cold
  flush+pre         flush, then read the packed weight once (the prefetch)
  flush+pre+gemm    the projection with its weight just prefetched
  flush+pre||gemm   prefetch of the NEXT weight on a second stream while this one runs
and reports cold / warm GEMM time (differences) and bandwidths, for the
skinny kernel and hipBLASLt.  If warm << cold, prefetching the next layer's
weights in the HBM-idle gaps of a decode step (norms, combine, kernel tails)
pays.  Output: JSON lines.

    python scripts/probe/mall_prefetch.py --out gpurun_out/mall/mall.json
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from k8s_vgpu_scheduler_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o_proj": (4096, 4096), "down": (4096, 12288), "gate_up": (24576, 4096)}


def graph_us(fn, reps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1000.0 / reps
        best = t if best is None else min(best, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--M", type=int, default=32)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ops.require_native()
    dev = torch.device("cuda")
    junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    junk.fill_(1)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    rows = []
    side = torch.cuda.Stream()
    for name, (N, K) in SHAPES.items():
        silu = name == "gate_up"
        lin = ops.PackedLinear((torch.randn(N, K, device=dev) * 0.02).bfloat16(), silu_mul=silu)
        nxt = ops.PackedLinear((torch.randn(N, K, device=dev) * 0.02).bfloat16(), silu_mul=silu)
        w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        x = torch.randn(a.M, K, device=dev).bfloat16()
        out = torch.empty(a.M, lin.out_features, device=dev, dtype=torch.bfloat16)
        yl = torch.empty(a.M, N, device=dev, dtype=torch.bfloat16)

        def flush():
            ops.stream_read(junk, out=sink)

        def pre(t):
            ops.stream_read(t, out=sink)

        def sk():
            lin(x, out=out)

        def lib():
            torch.matmul(x, w.t(), out=yl)

        def overlapped():
            # this projection on the main stream, the next one's prefetch on a side stream
            flush()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                pre(nxt.wp)
            sk()
            torch.cuda.current_stream().wait_stream(side)

        t_flush = graph_us(flush, a.reps)
        t_cold = graph_us(lambda: (flush(), sk()), a.reps) - t_flush
        t_pre = graph_us(lambda: (flush(), pre(lin.wp)), a.reps) - t_flush
        t_warm = graph_us(lambda: (flush(), pre(lin.wp), sk()), a.reps) - t_flush - t_pre
        t_lcold = graph_us(lambda: (flush(), lib()), a.reps) - t_flush
        t_lpre = graph_us(lambda: (flush(), pre(w)), a.reps) - t_flush
        t_lwarm = graph_us(lambda: (flush(), pre(w), lib()), a.reps) - t_flush - t_lpre
        t_both = graph_us(overlapped, a.reps) - t_flush
        mb = N * K * 2 / 1e6
        row = {"shape": name, "M": a.M, "weight_MB": round(mb, 1), "flush_us": round(t_flush, 1),
               "prefetch_us": round(t_pre, 2), "prefetch_TBps": round(mb / t_pre, 2),
               "skinny_cold_us": round(t_cold, 2), "skinny_warm_us": round(t_warm, 2),
               "hipblaslt_cold_us": round(t_lcold, 2), "hipblaslt_warm_us": round(t_lwarm, 2),
               "skinny_plus_next_prefetch_us": round(t_both, 2),
               "skinny_cold_TBps": round(mb / t_cold, 2), "skinny_warm_TBps": round(mb / t_warm, 2)}
        print(json.dumps(row), flush=True)
        rows.append(row)
        del lin, nxt, w
        torch.cuda.empty_cache()
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
