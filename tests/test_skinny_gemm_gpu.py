"""Skinny MFMA GEMM (csrc/ops/skinny_gemm.hip) against a plain fp32 PyTorch reference."""

import pytest
import torch

from k8s_vgpu_scheduler_amd import ops

pytestmark = pytest.mark.gpu


def _ref(x, w):
    return (x.float() @ w.float().t())


def _close(got, ref, tol=2e-2):
    err = (got.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err / scale < tol, (err, scale)


@pytest.mark.parametrize("variant", [ops.VARIANT_CLASSIC, ops.VARIANT_WIDE])
@pytest.mark.parametrize("M", [1, 7, 32, 33, 64, 100, 128])
@pytest.mark.parametrize("N,K", [(64, 64), (1024, 512), (4096, 4096), (6144, 4096), (4096, 12288)])
def test_skinny_gemm_matches_fp32(M, N, K, variant):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.02).bfloat16()
    lin = ops.PackedLinear(w)
    if variant == ops.VARIANT_WIDE and K >= 512:      # K = 64 is a single k-block: classic fallback
        assert ops.skinny_plan(M, K, N, ops.EPI_STORE, variant=variant)["variant"] == ops.VARIANT_WIDE
    for _ in range(2):   # split-K scratch must come back zeroed
        _close(lin(x, variant=variant), _ref(x, w))


@pytest.mark.parametrize("nt,wv,S", [(1, 1, 1), (1, 4, 1), (2, 2, 1), (2, 4, 1), (1, 4, 4), (2, 4, 2),
                                     (2, 1, 8), (1, 2, 16), (2, 4, 32)])
@pytest.mark.parametrize("M", [1, 32, 100])
def test_wide_variants(nt, wv, S, M):
    x = torch.randn(M, 4096, device="cuda").bfloat16()
    w = (torch.randn(2048, 4096, device="cuda") * 0.02).bfloat16()
    lin = ops.PackedLinear(w)
    pl = ops.skinny_plan(M, 4096, 2048, ops.EPI_STORE, nt, wv, S, ops.VARIANT_WIDE)
    assert pl["variant"] == ops.VARIANT_WIDE and (pl["nt"], pl["ks"], pl["S"]) == (nt, wv, S)
    ref = _ref(x, w)
    for _ in range(3):
        _close(lin(x, nt=nt, ks=wv, S=S, variant=ops.VARIANT_WIDE), ref)


def test_wide_lm_head_shape_and_fallbacks():
    # 151936 rows = 4748 tiles: not a multiple of 8 -> one tile per wave
    assert ops.skinny_plan(32, 4096, 151936, ops.EPI_STORE, variant=ops.VARIANT_WIDE)["nt"] == 1
    # a split that leaves no whole group per workgroup falls back to the classic kernel
    assert ops.skinny_plan(32, 4096, 2048, ops.EPI_STORE, 1, 4, 64, ops.VARIANT_WIDE)["variant"] == ops.VARIANT_CLASSIC
    # 1187 tiles (odd): one tile per wave, one wave per workgroup
    x = torch.randn(32, 4096, device="cuda").bfloat16()
    w = (torch.randn(37984, 4096, device="cuda") * 0.02).bfloat16()
    pl = ops.skinny_plan(32, 4096, 37984, ops.EPI_STORE, variant=ops.VARIANT_WIDE)
    assert (pl["variant"], pl["nt"], pl["ks"]) == (ops.VARIANT_WIDE, 1, 1)
    _close(ops.PackedLinear(w)(x, variant=ops.VARIANT_WIDE), _ref(x, w))


@pytest.mark.parametrize("nt,ks,S", [(1, 1, 1), (1, 4, 1), (2, 2, 1), (2, 8, 1), (1, 4, 4), (2, 4, 2),
                                     (1, 1, 8), (1, 8, 8), (2, 2, 3), (1, 4, 64)])
@pytest.mark.parametrize("M", [1, 32, 100])
def test_skinny_gemm_variants(nt, ks, S, M):
    x = torch.randn(M, 4096, device="cuda").bfloat16()
    w = (torch.randn(2048, 4096, device="cuda") * 0.02).bfloat16()
    lin = ops.PackedLinear(w)
    ref = _ref(x, w)
    for _ in range(3):   # the split-K scratch must come back zeroed every call
        _close(lin(x, nt=nt, ks=ks, S=S), ref)


def test_split_k_under_graph_replay():
    x = torch.randn(32, 4096, device="cuda").bfloat16()
    w = (torch.randn(4096, 4096, device="cuda") * 0.02).bfloat16()
    lin = ops.PackedLinear(w)
    # the o_proj shape splits by default on the whole chip; a CU partition (<= 96 CUs) does not split
    assert (ops.skinny_plan(32, 4096, 4096, ops.EPI_STORE)["S"] > 1) == (ops.visible_cus() > 96)
    out = torch.empty(32, 4096, device="cuda", dtype=torch.bfloat16)
    lin(x, out=out, S=4)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        lin(x, out=out, S=4)
    ref = _ref(x, w)
    for i in range(5):
        x.copy_(torch.randn(32, 4096, device="cuda").bfloat16())
        ref = _ref(x, w)
        g.replay()
        torch.cuda.synchronize()
        _close(out, ref)


def test_exact_on_integers():
    """Small integers are exact in bf16 and fp32: any k-permutation mismatch between
    the packed W and the X fragments shows up as a wrong element."""
    x = torch.randint(-3, 4, (32, 512), device="cuda").bfloat16()
    w = torch.randint(-3, 4, (256, 512), device="cuda").bfloat16()
    for variant in (ops.VARIANT_CLASSIC, ops.VARIANT_WIDE):
        assert ops.skinny_plan(32, 512, 256, ops.EPI_STORE, variant=variant)["variant"] == variant
        got = ops.PackedLinear(w)(x, variant=variant).float()
        # the fp32 sum is exact; the kernel rounds it to bf16 once (RNE), like this
        assert torch.equal(got, (x.float() @ w.float().t()).bfloat16().float())


@pytest.mark.parametrize("variant", [ops.VARIANT_CLASSIC, ops.VARIANT_WIDE])
@pytest.mark.parametrize("M", [1, 32, 64, 128])
@pytest.mark.parametrize("S", [0, 1, 4])
def test_fused_silu_mul(M, S, variant):
    inter, K = 1024, 512
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(2 * inter, K, device="cuda") * 0.05).bfloat16()
    got = ops.PackedLinear(w, silu_mul=True)(x, S=S, variant=variant)
    gu = _ref(x, w).bfloat16().float()
    ref = torch.nn.functional.silu(gu[:, :inter]) * gu[:, inter:]
    assert got.shape == (M, inter)
    _close(got, ref)


def test_strided_x_and_out():
    x_big = torch.randn(32, 1024 + 64, device="cuda").bfloat16()
    x = x_big[:, :1024]
    w = (torch.randn(256, 1024, device="cuda") * 0.02).bfloat16()
    out_big = torch.zeros(32, 512, device="cuda", dtype=torch.bfloat16)
    ops.PackedLinear(w)(x, out=out_big[:, :256])
    _close(out_big[:, :256], _ref(x, w))
    assert out_big[:, 256:].abs().max().item() == 0


def test_rejects_bad_shapes():
    with pytest.raises(ValueError):
        ops.pack_weight(torch.zeros(33, 64, device="cuda", dtype=torch.bfloat16))
    lin = ops.PackedLinear(torch.zeros(64, 64, device="cuda", dtype=torch.bfloat16))
    with pytest.raises(RuntimeError):
        lin(torch.zeros(129, 64, device="cuda", dtype=torch.bfloat16))


def _rms_ref(x, w, eps=1e-6):
    xf = x.float()
    return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()


@pytest.mark.parametrize("variant", ["wide", "widek", "widek8"])
@pytest.mark.parametrize("S", [0, 1, 4])
@pytest.mark.parametrize("M", [1, 5, 32, 48])
def test_row_norm_fusion_chain(M, S, variant):
    """o_proj-like residual call (res += X.W^T, per-slot sums of squares) then
    a gate_up-like call that applies RMSNorm through folded column weights and
    row scales from those slots, vs. add + RMSNorm + GEMM in fp32; on the wide
    kernel and on the K-split one (variant 3)."""
    g = torch.Generator(device="cuda").manual_seed(M * 13 + S)
    K, N1, N2 = 4096, 4096, 2048
    res = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    wo = (torch.randn(N1, K, device="cuda", generator=g) * 0.02).bfloat16()
    wn = (1 + 0.1 * torch.randn(K, device="cuda", generator=g)).bfloat16()
    wg = (torch.randn(N2, K, device="cuda", generator=g) * 0.02).bfloat16()
    po = ops.PackedLinear(wo)
    pg = ops.PackedLinear(wg, col_scale=wn)
    ks = 8 if variant == "widek8" else 0    # 8 k-waves per workgroup: one M-tile only
    if variant.startswith("widek"):
        po.variant = pg.variant = ops.VARIANT_WIDEK
        pl = ops.skinny_plan(M, K, N1, ops.EPI_STORE, 0, ks, S, ops.VARIANT_WIDEK)
        if ks == 8 and M > 32:
            assert pl["variant"] != ops.VARIANT_WIDEK
            return
        assert pl["variant"] == ops.VARIANT_WIDEK
    slots = po.slots(M)
    ss = torch.full((slots * ops.SS_ROWS,), float("nan"), device="cuda")   # every used slot must be written
    r1 = res.clone()
    for _ in range(2):   # split-K scratch / tickets must come back clean
        r1.copy_(res)
        po.norm_call(x, out=r1, residual=True, ss_out=ss, S=S, ks=ks)
        exp_res = res.float() + _ref(x, wo)
        _close(r1, exp_res)
        got_ss = ss.view(slots, ops.SS_ROWS)[:, :M].sum(0)
        _close(got_ss, r1.float().pow(2).sum(-1), 1e-3)
        y = torch.empty(M, N2, device="cuda", dtype=torch.bfloat16)
        pg.norm_call(r1, out=y, row_scale=(ss, slots, K, 1e-6), S=S, ks=ks)
        _close(y, _rms_ref(r1, wn) @ wg.float().t())


@pytest.mark.parametrize("M", [1, 32])
def test_row_scale_with_silu_and_single_slot(M):
    """The decoder's first norm (one slot from torch) into the SiLU*up epilogue."""
    K, inter = 1024, 2048
    res = torch.randn(M, K, device="cuda").bfloat16()
    wn = (1 + 0.1 * torch.randn(K, device="cuda")).bfloat16()
    wgu = (torch.randn(2 * inter, K, device="cuda") * 0.05).bfloat16()
    ss = torch.zeros(ops.SS_ROWS, device="cuda")
    ss[:M] = res.float().pow(2).sum(-1)
    lin = ops.PackedLinear(wgu, silu_mul=True, col_scale=wn)
    y = torch.empty(M, inter, device="cuda", dtype=torch.bfloat16)
    lin.norm_call(res, out=y, row_scale=(ss, 1, K, 1e-6))
    gu = _rms_ref(res, wn).bfloat16().float() @ wgu.float().t()
    g, u = gu[:, :inter], gu[:, inter:]
    _close(y, torch.nn.functional.silu(g) * u, 3e-2)


def test_norm_call_rejects_bad_arguments():
    lin = ops.PackedLinear((torch.randn(2048, 4096, device="cuda") * 0.02).bfloat16())
    x = torch.randn(4, 4096, device="cuda").bfloat16()
    out = torch.empty(4, 2048, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        lin.norm_call(x, out=out, residual=True)          # no ss_out
    with pytest.raises(ValueError):
        lin.norm_call(x, out=out, row_scale=(torch.zeros(8, device="cuda"), 1, 4096, 1e-6))   # slots too small


_MID_CHILD = r"""
import json, torch
from k8s_vgpu_scheduler_amd import ops
from k8s_vgpu_scheduler_amd.ops import reference as ref
out = {"cus": ops.visible_cus()}
x = torch.randn(32, 4096, device="cuda").bfloat16()
for name, N, K, silu in (("gate_up", 24576, 4096, True), ("down", 4096, 12288, False), ("lm", 65536, 4096, False)):
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    lin = ops.PackedLinear(w, silu_mul=silu)
    xx = x if K == 4096 else torch.randn(32, K, device="cuda").bfloat16()
    pl = ops.skinny_plan(32, K, N, lin.epi)
    y = lin(xx).float()
    r = xx.float() @ w.float().t()
    if silu:
        r = ref.silu_mul(r.bfloat16()).float()
    out[name] = {"plan": [pl["variant"], pl["nt"], pl["ks"], pl["S"]],
                 "err": ((y - r).abs().max() / r.abs().max()).item()}
# row-norm fusion: the down projection's 128 sum-of-squares slots into gate_up,
# whose one-wave plan here reads only 64 (the kernel takes more waves)
wn = (1 + 0.1 * torch.randn(4096, device="cuda")).bfloat16()
wg = (torch.randn(24576, 4096, device="cuda") * 0.02).bfloat16()
pg = ops.PackedLinear(wg, silu_mul=True, col_scale=wn)
ss = torch.zeros(128 * ops.SS_ROWS, device="cuda")
ss.view(128, ops.SS_ROWS)[:, :32] = (x.float().pow(2).sum(-1) / 128)[None, :]
y = torch.empty(32, 12288, device="cuda", dtype=torch.bfloat16)
pg.norm_call(x, out=y, row_scale=(ss, 128, 4096, 1e-6))
h = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-6) * wn.float()
r = ref.silu_mul((h.bfloat16().float() @ wg.float().t()).bfloat16()).float()
out["rowscale128_err"] = ((y.float() - r).abs().max() / r.abs().max()).item()
print("RESULT " + json.dumps(out))
"""


@pytest.mark.parametrize("mid", ["1", "0"])
def test_half_gpu_partition_plans(mid):
    """128-CU partition (2 slices per GPU): the mid-partition wave counts
    (MIVGPU_WIDE_MID_PLAN) are chosen and compute the same as fp32."""
    import json
    import os
    import subprocess
    import sys

    env = dict(os.environ, HSA_CU_MASK="0:0-127", MIVGPU_WIDE_MID_PLAN=mid)
    r = subprocess.run([sys.executable, "-c", _MID_CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][0][7:])
    assert out["cus"] == 128
    want = {"1": {"gate_up": [2, 2, 1, 1], "down": [2, 1, 4, 4], "lm": [2, 1, 4, 1]},
            "0": {"gate_up": [2, 2, 2, 1], "down": [2, 1, 2, 4], "lm": [2, 1, 2, 1]}}[mid]
    for k, plan in want.items():
        assert out[k]["plan"] == plan, (k, out[k])
        assert out[k]["err"] < 2e-2, (k, out[k])
    assert out["rowscale128_err"] < 3e-2, out


_SLICE_PLANS_CHILD = r"""
import json
from k8s_vgpu_scheduler_amd import ops
shapes = {"qkv": (6144, 4096, 0), "o_proj": (4096, 4096, 0), "gate_up": (24576, 4096, 1), "down": (4096, 12288, 0),
          "lm_head": (151936, 4096, 0)}
out = {"cus": ops.visible_cus()}
for k, (N, K, epi) in shapes.items():
    pl = ops.skinny_plan(32, K, N, epi)
    out[k] = [pl["variant"], pl["nt"], pl["ks"], pl["S"]]
print("RESULT " + json.dumps(out))
"""


@pytest.mark.parametrize("mask,want", [
    ("0:0-31", {"qkv": [2, 1, 2, 1], "o_proj": [2, 1, 4, 1], "gate_up": [2, 2, 4, 1], "down": [2, 1, 4, 1],
                "lm_head": [2, 1, 4, 1]}),
    ("0:0-63", {"qkv": [2, 1, 4, 1], "o_proj": [2, 1, 2, 1], "gate_up": [2, 2, 2, 1], "down": [2, 1, 2, 1],
                "lm_head": [2, 1, 4, 1]}),
])
def test_slice_partition_plans(mask, want):
    """Auto plans of the Qwen3-8B projections in the 8-slice and 4-slice
    partitions (the measured table in skinny_gemm.hip plan_wide)."""
    import json
    import os
    import subprocess
    import sys

    r = subprocess.run([sys.executable, "-c", _SLICE_PLANS_CHILD], env=dict(os.environ, HSA_CU_MASK=mask),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][0][7:])
    assert {k: out[k] for k in want} == want


@pytest.mark.parametrize("M", [33, 92, 128])
def test_prefill_row_counts_at_qwen3_8b_shapes(M):
    """The serving prefill runs the packed projections on row chunks of up to
    128 (models/qwen3.py prefill): gate_up + SiLU (24576 x 4096) and down
    (4096 x 12288) at Qwen3-8B shapes, row counts the decode path never uses."""
    torch.manual_seed(M)
    for N, K, silu in ((24576, 4096, True), (4096, 12288, False)):
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        pl = ops.PackedLinear(w, silu_mul=silu)
        pl.reserve(128)
        got = pl(x).float()
        torch.cuda.synchronize()
        gu = _ref(x, w).bfloat16().float()
        ref = torch.nn.functional.silu(gu[:, :N // 2]) * gu[:, N // 2:] if silu else gu
        _close(got, ref)
