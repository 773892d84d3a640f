"""Decode-projection GEMM microbenchmark: skinny MFMA kernel vs hipBLASLt (F.linear).

Shapes are the Qwen3-8B projections (qkv, o, gate_up, down, lm_head) at the
decode batch sizes the slices run.  Reports µs per call and effective weight
bandwidth (W bytes / time), each timed over a hipGraph of ``--reps`` calls.

    python -m k8s_vgpu_scheduler_amd.bench.gemm --out gpurun_out/gemm.json
"""

from __future__ import annotations

import argparse
import json
from pathlib import Path

import torch
import torch.nn.functional as F

from k8s_vgpu_scheduler_amd import ops

SHAPES = {  # name: (N, K, silu_mul)
    "qkv": (6144, 4096, False),
    "o_proj": (4096, 4096, False),
    "gate_up": (24576, 4096, True),
    "down": (4096, 12288, False),
    "lm_head": (151936, 4096, False),
}


def _time(fn, reps: int) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,32,64,128")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--sweep", action="store_true", help="also sweep nt/ks/S (at --sweep-rows)")
    ap.add_argument("--sweep-rows", default="32", help="row counts the sweep runs at (comma list)")
    ap.add_argument("--norm", action="store_true",
                    help="also time the row-norm fusion epilogues (residual update, row scales) per kernel")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ops.require_native()
    res = []
    for name in a.shapes.split(","):
        N, K, silu = SHAPES[name]
        wbytes = N * K * 2
        # rotate over enough copies (>= 768 MB) that neither kernel is served
        # from the 256 MB Infinity Cache: decode streams every weight once/step
        ncopy = max(1, -(-768 * 2 ** 20 // wbytes))
        ws = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(ncopy)]
        lins = [ops.PackedLinear(w, silu_mul=silu) for w in ws]
        w, lin = ws[0], lins[0]
        for M in map(int, a.batches.split(",")):
            x = torch.randn(M, K, device="cuda").bfloat16()
            out = torch.empty(M, lin.out_features, device="cuda", dtype=torch.bfloat16)
            if silu:
                gu = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                act = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)

                def lib_fn(i):
                    torch.matmul(x, ws[i % ncopy].t(), out=gu)
                    ops.silu_mul(gu, out=act)
            else:
                yl = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

                def lib_fn(i):
                    torch.matmul(x, ws[i % ncopy].t(), out=yl)
            t_lib = _time(lib_fn, a.reps)
            t_sk = _time(lambda i: lins[i % ncopy](x, out=out), a.reps)
            t_wide = _time(lambda i: lins[i % ncopy](x, out=out, variant=ops.VARIANT_WIDE), a.reps)
            widek = {}
            if M <= 64:
                for kw in (2, 4):
                    for S in (0, 1, 2, 4):
                        if ops.skinny_plan(M, K, N, lin.epi, 0, kw, S, ops.VARIANT_WIDEK)["variant"] != ops.VARIANT_WIDEK:
                            continue
                        widek[f"kw{kw}_S{S or 'auto'}"] = round(_time(
                            lambda i: lins[i % ncopy](x, out=out, ks=kw, S=S, variant=ops.VARIANT_WIDEK), a.reps), 2)
            row = {"plan": ops.skinny_plan(M, K, N, lin.epi), "shape": name, "M": M, "N": N, "K": K, "fused_silu": silu,
                   "wide_plan": ops.skinny_plan(M, K, N, lin.epi, variant=ops.VARIANT_WIDE),
                   "wide_us": round(t_wide, 2), "wide_TBps": round(wbytes / t_wide / 1e6, 3),
                   "hipblaslt_us": round(t_lib, 2), "skinny_us": round(t_sk, 2),
                   "hipblaslt_TBps": round(wbytes / t_lib / 1e6, 3), "skinny_TBps": round(wbytes / t_sk / 1e6, 3),
                   "speedup": round(t_lib / t_sk, 3), "weight_copies": ncopy, "widek_us": widek}
            if a.norm and M <= 64:
                # row-norm fusion: the residual update (+ sum-of-squares slots)
                # and a store with row scales from 128 slots, on the wide and the
                # K-split kernel, vs the plain store of the same kernel
                ss = torch.rand(128 * ops.SS_ROWS, device="cuda") + 1.0
                res_buf = torch.randn(M, N, device="cuda").bfloat16()
                nrm = {}
                for tag, v in (("wide", ops.VARIANT_WIDE), ("widek", ops.VARIANT_WIDEK)):
                    if ops.skinny_plan(M, K, N, lin.epi, variant=v)["variant"] != v:
                        continue
                    for L in lins:
                        L.variant = v
                    cases = {"store": lambda i: lins[i % ncopy](x, out=out),
                             "rowscale": lambda i: lins[i % ncopy].norm_call(x, out=out, row_scale=(ss, 128, K, 1e-6))}
                    if not silu:
                        cases["resid"] = lambda i: lins[i % ncopy].norm_call(x, out=res_buf, residual=True, ss_out=ss)
                    for cname, fn in cases.items():
                        try:
                            nrm[f"{tag}_{cname}"] = round(_time(fn, a.reps), 2)
                        except (RuntimeError, ValueError) as e:
                            nrm[f"{tag}_{cname}"] = str(e)[:60]
                    for L in lins:
                        L.variant = ops.VARIANT_AUTO
                row["norm_us"] = nrm
            if a.sweep and M in {int(v) for v in a.sweep_rows.split(",")}:
                sw = {}
                for variant, tag, kss in ((ops.VARIANT_CLASSIC, "", (1, 2, 4, 8)), (ops.VARIANT_WIDE, "wide_", (1, 2, 4)),
                                          (ops.VARIANT_WIDEK, "widek_", (2, 4, 8))):
                    for nt in (1, 2):
                        for ks in kss:
                            for S in (1, 2, 4, 8, 16):
                                if (silu and nt == 1) or S > K // 64 // ks:
                                    continue
                                if ops.skinny_plan(M, K, N, lin.epi, nt, ks, S, variant)["variant"] != variant:
                                    continue      # the wide kernel cannot run this split
                                try:
                                    sw[f"{tag}nt{nt}_ks{ks}_S{S}"] = round(_time(
                                        lambda i: lins[i % ncopy](x, out=out, nt=nt, ks=ks, S=S, variant=variant),
                                        a.reps), 2)
                                except RuntimeError as e:
                                    sw[f"{tag}nt{nt}_ks{ks}_S{S}"] = str(e)[:40]
                best = min((v, k) for k, v in sw.items() if isinstance(v, float))
                row["sweep_best"] = {"config": best[1], "us": best[0]}
                row["sweep_us"] = sw
            print(json.dumps(row), flush=True)
            res.append(row)
        del w, lin, ws, lins
        torch.cuda.empty_cache()
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
