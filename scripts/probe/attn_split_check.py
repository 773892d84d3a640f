"""Decode step after a prefill of L tokens, Qwen3-8B B=1 T=4096: fused
attention (eager), unfused attention (eager) and the captured graph, compared
by logits cosine.  Fault-free: nothing replays on an out-of-range token."""
import torch

from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_8B, Qwen3Decoder

d = Qwen3Decoder(QWEN3_8B, batch=1, max_ctx=4096, device="cuda")
d.reserve_prefill()
d.prefill(list(range(3, 163)))
d.capture()
cos = torch.nn.functional.cosine_similarity
for L in (92, 255, 256, 257, 300, 600):
    prompt = list(range(5, 5 + L))
    out = {}
    for mode in ("fused", "unfused", "graph"):
        d.prefill(prompt)
        torch.cuda.synchronize()
        with torch.no_grad():
            if mode == "graph":
                d.graph.replay()
            else:
                d.attn_fused = mode == "fused"
                d._step_impl()
                d.attn_fused = True
        torch.cuda.synchronize()
        out[mode] = d.logits[0].float().clone()
    print(L, "fused~unfused", round(cos(out["fused"], out["unfused"], dim=0).item(), 5),
          "graph~unfused", round(cos(out["graph"], out["unfused"], dim=0).item(), 5),
          "counters", d.attn_counters.tolist(), flush=True)
