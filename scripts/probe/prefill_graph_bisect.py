"""Which part of a post-capture prefill makes the next decode-graph replay
write a garbage token (Qwen3-8B, B=1)?  Each variant builds a fresh decoder,
captures, replays once (must be clean), applies one piece of the prefill,
replays once more and reports whether tokens[0] is still a vocabulary id --
never replaying a graph whose input token is already out of range.
    python scripts/probe/prefill_graph_bisect.py <variant>"""
import sys

import torch

from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_8B, Qwen3Decoder

variant = sys.argv[1]
cfg = QWEN3_8B
d = Qwen3Decoder(cfg, batch=1, max_ctx=4096, device="cuda")
d.reserve_prefill()
d.prefill(list(range(3, 163)))
d.capture()
d.graph.replay()
torch.cuda.synchronize()
t0 = int(d.tokens[0])
assert 0 <= t0 < cfg.vocab, t0
L = 92
g = torch.Generator(device="cuda").manual_seed(0)
if variant == "full":
    d.prefill(list(range(5, 5 + L)))
elif variant == "state":
    d.tokens[0] = 777
    d.pos[0] = L
    d.seqlens[0] = L + 1
elif variant == "full_rezero":
    d.prefill(list(range(5, 5 + L)))
    for pl in d.packed_linears():
        if pl.scratch is not None:
            pl.scratch.zero_()
        if pl.tickets is not None:
            pl.tickets.zero_()
elif variant == "gemms":
    for lw in d.w.layers:
        x = torch.randn(L, cfg.hidden, device="cuda", generator=g).bfloat16()
        d._proj(lw, "qkv", x)
        act = d._proj(lw, "gu", x)
        d._proj(lw, "d", act)
elif variant == "pd_only":
    for lw in d.w.layers:
        a = (torch.randn(L, cfg.intermediate, device="cuda", generator=g) * 0.1).bfloat16()
        d._proj(lw, "d", a)
elif variant == "kv":
    for li in range(cfg.layers):
        k = torch.randn(L, cfg.kv_heads, cfg.head_dim, device="cuda", generator=g)
        d._write_kv(li, 0, k, k)
    d.pos[0] = L
    d.seqlens[0] = L + 1
elif variant == "full_counters":
    d.prefill(list(range(5, 5 + L)))
    torch.cuda.synchronize()
    print("counters after prefill", d.attn_counters.tolist(), flush=True)
elif variant == "full_eager":
    d.prefill(list(range(5, 5 + L)))
torch.cuda.synchronize()
if d.attn_counters is not None:
    print("counters before replay", d.attn_counters.tolist(), flush=True)
if variant == "full_eager":
    with torch.no_grad():
        d._step_impl()
else:
    d.graph.replay()
torch.cuda.synchronize()
t1 = int(d.tokens[0])
print(("CLEAN" if 0 <= t1 < cfg.vocab else "CORRUPT"), variant, t0, t1, int(d.pos[0]), flush=True)
