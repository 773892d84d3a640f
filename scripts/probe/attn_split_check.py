"""Decode-step numerics after a prefill of L tokens (Qwen3-8B, B=1, T=4096).

One probe for the fused-attention investigation of round 2 (three one-off
scripts before):

  --mode paths   fused attention (eager), unfused (eager) and the captured
                 graph, compared by logits cosine;
  --mode rounds  three rounds of prefill -> fused step / prefill -> unfused
                 step per L: is an odd result a prefill or a decode effect?
  --mode state   split-K scratch / ticket state of the packed projections and
                 the token / position left by the prefill, per round.

Fault-free: nothing replays on an out-of-range token.

    python scripts/probe/attn_split_check.py --mode paths
"""
import argparse

import torch

from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_8B, Qwen3Decoder

ap = argparse.ArgumentParser()
ap.add_argument("--mode", choices=["paths", "rounds", "state"], default="paths")
a = ap.parse_args()

d = Qwen3Decoder(QWEN3_8B, batch=1, max_ctx=4096, device="cuda")
d.reserve_prefill()
d.prefill(list(range(3, 163)))
d.capture()
cos = torch.nn.functional.cosine_similarity


def step(fused=True, graph=False):
    with torch.no_grad():
        if graph:
            d.graph.replay()
        else:
            d.attn_fused = fused
            d._step_impl()
            d.attn_fused = True
    torch.cuda.synchronize()
    return d.logits[0].float().clone()


if a.mode == "paths":
    for L in (92, 255, 256, 257, 300, 600):
        prompt = list(range(5, 5 + L))
        out = {}
        for mode in ("fused", "unfused", "graph"):
            d.prefill(prompt)
            torch.cuda.synchronize()
            out[mode] = step(fused=mode == "fused", graph=mode == "graph")
        print(L, "fused~unfused", round(cos(out["fused"], out["unfused"], dim=0).item(), 5),
              "graph~unfused", round(cos(out["graph"], out["unfused"], dim=0).item(), 5),
              "counters", d.attn_counters.tolist(), flush=True)
elif a.mode == "rounds":
    for L in (255, 92, 255, 300, 255):
        prompt = list(range(5, 5 + L))
        ref = None
        for rnd in range(3):
            d.prefill(prompt)
            torch.cuda.synchronize()
            fused = step(fused=True)
            d.prefill(prompt)
            unfused = step(fused=False)
            ref = unfused if ref is None else ref
            print(L, rnd, "fused~ref", round(cos(fused, ref, dim=0).item(), 5),
                  "unfused~ref", round(cos(unfused, ref, dim=0).item(), 5), flush=True)
else:
    pls = d.packed_linears()
    for L in (255, 300, 255, 300, 255, 300):
        prompt = list(range(5, 5 + L))
        ref = None
        for rnd in range(4):
            d.prefill(prompt)
            torch.cuda.synchronize()
            tok, pos, sl = int(d.tokens[0]), int(d.pos[0]), int(d.seqlens[0])
            dirty = sum(int(pl.scratch.ne(0).sum()) for pl in pls if pl.scratch is not None)
            tick = sum(int(pl.tickets.ne(0).sum()) for pl in pls if pl.tickets is not None)
            lg = step(fused=True)
            ref = lg if ref is None else ref
            print(L, rnd, "tok", tok, "pos", pos, "seqlens", sl, "scratch_nonzero", dirty, "tickets_nonzero", tick,
                  "cos", round(cos(lg, ref, dim=0).item(), 4), flush=True)
