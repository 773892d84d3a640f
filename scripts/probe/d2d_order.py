"""Are device-to-device copies ordered with the kernels after them on the
same stream?  Each iteration writes a fresh value into `src` (kernel), copies
it into `dst` (copy_ of a contiguous same-dtype tensor: a D2D memcpy) and
reads `dst` with a kernel into out[i]; out must equal the values written.
Also argmax(out=view) and index_select(out=), the decode graph's writers."""
import torch

N = 4000
dev = "cuda"
vals = torch.arange(N, device=dev, dtype=torch.long) * 7 + 3
res = {}

# 1) plain D2D copy of one int64
src = torch.zeros(1, dtype=torch.long, device=dev)
dst = torch.zeros(1, dtype=torch.long, device=dev)
out = torch.zeros(N, dtype=torch.long, device=dev)
for i in range(N):
    src.copy_(vals[i:i + 1] * 1)          # kernel
    dst.copy_(src)                        # D2D copy
    torch.add(dst, 0, out=out[i:i + 1])   # kernel reading dst
torch.cuda.synchronize()
res["d2d_copy_mismatches"] = int((out != vals).sum())

# 2) argmax(out=view) then a reader
tok = torch.zeros(4, dtype=torch.long, device=dev)
logits = torch.zeros(N, 512, device=dev)
logits[torch.arange(N), torch.arange(N) % 512] = 1.0
out2 = torch.zeros(N, dtype=torch.long, device=dev)
for i in range(N):
    torch.argmax(logits[i:i + 1], dim=-1, out=tok[0:1])
    torch.add(tok[0:1], 0, out=out2[i:i + 1])
torch.cuda.synchronize()
res["argmax_out_mismatches"] = int((out2 != torch.arange(N, device=dev) % 512).sum())

# 3) H2D + D2D into a slice, as prefill fills its id buffer
ids = torch.zeros(256, dtype=torch.long, device=dev)
out3 = torch.zeros(N, dtype=torch.long, device=dev)
for i in range(N):
    host = torch.tensor([i, i + 1, i + 2])
    ids[:3].copy_(host.to(dev))
    torch.sum(ids[:3], dim=0, keepdim=True, out=out3[i:i + 1])
torch.cuda.synchronize()
res["h2d_slice_mismatches"] = int((out3 != torch.arange(N, device=dev) * 3 + 3).sum())
print(res, flush=True)
