"""Out-of-bounds write check for every kernel the serving prefill runs at
Qwen3-8B shapes: each output (and in-place input) is a view in the middle of a
sentinel-filled buffer, and the sentinels on both sides must survive.  A
write past an output corrupts whatever the caching allocator placed next to
it -- e.g. state a captured hipGraph reads later -- without faulting where it
happens."""

from __future__ import annotations

import pytest
import torch

from k8s_vgpu_scheduler_amd import ops

pytestmark = pytest.mark.gpu

PAD = 1 << 20          # elements of sentinel on each side
SENT = -12345.0


def guarded(rows, cols, dtype=torch.bfloat16):
    buf = torch.full((PAD * 2 + rows * cols,), SENT, dtype=dtype, device="cuda")
    return buf, buf[PAD:PAD + rows * cols].view(rows, cols)


def intact(buf, what):
    torch.cuda.synchronize()
    lo, hi = buf[:PAD], buf[-PAD:]
    bad_lo = int((lo != SENT).sum())
    bad_hi = int((hi != SENT).sum())
    assert bad_lo == 0 and bad_hi == 0, f"{what}: {bad_lo} elements written before, {bad_hi} after the output"


@pytest.mark.parametrize("M", [1, 22, 33, 92, 128])
def test_prefill_kernels_stay_in_bounds(M):
    ops.require_native()
    torch.manual_seed(M)
    h, inter, vocab = 4096, 12288, 151936
    x = (torch.randn(M, h, device="cuda") * 0.5).bfloat16()
    w = (1 + 0.05 * torch.randn(h, device="cuda")).bfloat16()
    # norms (rows = prompt tokens)
    buf, out = guarded(M, h)
    ops.rmsnorm(x, w, 1e-6, out=out)
    intact(buf, "rmsnorm")
    rbuf, res = guarded(M, h)
    res.copy_(x)
    buf, out = guarded(M, h)
    ops.add_rmsnorm(x, res, w, 1e-6, out=out)
    intact(buf, "add_rmsnorm out")
    intact(rbuf, "add_rmsnorm residual")
    # packed projections (classic kernel above 64 rows, wide below)
    for N, K, silu in ((2 * inter, h, True), (h, inter, False), (6144, h, False), (h, h, False)):
        pl = ops.PackedLinear((torch.randn(N, K, device="cuda") * 0.02).bfloat16(), silu_mul=silu)
        pl.reserve(128)
        sbuf = torch.full((PAD * 2 + pl.scratch.numel(),), SENT, device="cuda") if pl.scratch is not None else None
        xin = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
        buf, out = guarded(M, pl.out_features)
        pl(xin, out=out)
        intact(buf, f"skinny {N}x{K} silu={silu}")
        assert sbuf is None or int((sbuf != SENT).sum()) == 0
        if pl.scratch is not None:
            torch.cuda.synchronize()
            assert int(pl.scratch.abs().sum()) == 0, "split-K scratch must be left zeroed"
            assert int(pl.tickets.abs().sum()) == 0, "split-K tickets must be left zeroed"
    # lm_head on the last row
    pl = ops.PackedLinear((torch.randn(vocab, h, device="cuda") * 0.02).bfloat16())
    pl.reserve(128)
    buf, out = guarded(1, vocab)
    pl(x[-1:].contiguous(), out=out)
    intact(buf, "lm_head")
    # library GEMMs of the whole-GPU plan (qkv, o_proj): hipBLASLt into a view
    for N in (6144, 4096):
        wl = (torch.randn(N, h, device="cuda") * 0.02).bfloat16()
        buf, out = guarded(M, N)
        torch.mm(x, wl.t(), out=out)
        intact(buf, f"hipBLASLt {M}x{N}")
