"""Bad decode steps after a prefill: is split-K state (scratch / tickets of
the packed projections) or the token left non-zero / stale when it happens?"""
import torch

from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_8B, Qwen3Decoder

d = Qwen3Decoder(QWEN3_8B, batch=1, max_ctx=4096, device="cuda")
d.reserve_prefill()
d.prefill(list(range(3, 163)))
d.capture()
cos = torch.nn.functional.cosine_similarity
pls = d.packed_linears()
for L in (255, 300, 255, 300, 255, 300):
    prompt = list(range(5, 5 + L))
    ref = None
    for rnd in range(4):
        d.prefill(prompt)
        torch.cuda.synchronize()
        tok = int(d.tokens[0]); pos = int(d.pos[0]); sl = int(d.seqlens[0])
        dirty = sum(int(pl.scratch.ne(0).sum()) for pl in pls if pl.scratch is not None)
        tick = sum(int(pl.tickets.ne(0).sum()) for pl in pls if pl.tickets is not None)
        with torch.no_grad():
            d._step_impl()
        torch.cuda.synchronize()
        lg = d.logits[0].float().clone()
        if ref is None:
            ref = lg
        print(L, rnd, "tok", tok, "pos", pos, "seqlens", sl, "scratch_nonzero", dirty, "tickets_nonzero", tick,
              "cos", round(cos(lg, ref, dim=0).item(), 4), flush=True)
