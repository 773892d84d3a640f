"""Is the odd fused-attention result a prefill or a decode-step effect?
For each L, three rounds of: prefill -> prefill logits; eager fused step;
prefill again -> eager unfused step.  Cosines against round 0's unfused."""
import torch

from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_8B, Qwen3Decoder

d = Qwen3Decoder(QWEN3_8B, batch=1, max_ctx=4096, device="cuda")
d.reserve_prefill()
d.prefill(list(range(3, 163)))
d.capture()
cos = torch.nn.functional.cosine_similarity
for L in (255, 92, 255, 300, 255):
    prompt = list(range(5, 5 + L))
    rows = []
    ref = None
    for rnd in range(3):
        pl = d.prefill(prompt).float().clone()
        torch.cuda.synchronize()
        with torch.no_grad():
            d._step_impl()
        torch.cuda.synchronize()
        fused = d.logits[0].float().clone()
        d.prefill(prompt)
        d.attn_fused = False
        with torch.no_grad():
            d._step_impl()
        d.attn_fused = True
        torch.cuda.synchronize()
        unf = d.logits[0].float().clone()
        if ref is None:
            ref, pref = unf, pl
        rows.append((round(cos(pl, pref, dim=0).item(), 4), round(cos(fused, ref, dim=0).item(), 4),
                     round(cos(unf, ref, dim=0).item(), 4)))
    print(L, "(prefill, fused, unfused) vs round 0:", rows, flush=True)
