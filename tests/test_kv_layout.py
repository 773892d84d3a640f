"""Fragment-packed KV layout (csrc/ops/model_ops.hip, MFMA decode attention):
the Python packing used by tests/benchmarks matches the kernel's index formulas
element by element.  CPU only: the library is not loaded."""

import pytest
import torch

from k8s_vgpu_scheduler_amd import ops


@pytest.fixture
def packed(monkeypatch):
    monkeypatch.setattr(ops, "kv_packed", lambda: True)


def _k_offset(key, dim):
    # qk_norm_rope_kv_kernel<true>: key = 8(r/4) + 4t + r%4, dim = 32s + 8q + e
    k = key % 32
    t, r = (k >> 2) & 1, 4 * (k >> 3) + (k & 3)
    s, q, e = dim >> 5, (dim >> 3) & 3, dim & 7
    return (key // 32), (((t * 4 + s) * 4 + q) * 16 + r) * 8 + e


def _v_offset(key, dim):
    k = key % 32
    q, e = k >> 3, k & 7
    dt, r = dim >> 4, dim & 15
    return (key // 32), ((dt * 4 + q) * 16 + r) * 8 + e


def test_pack_matches_kernel_index_formulas(packed):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, 2, 64, 128, generator=g)
    pk, pv = ops.k_to_cache_layout(x), ops.v_to_cache_layout(x)
    assert pk.shape == (1, 2, 2, 4096) and pv.shape == (1, 2, 2, 4096)
    for key in (0, 3, 4, 7, 8, 13, 31, 32, 45, 63):
        for dim in (0, 7, 8, 31, 32, 63, 64, 100, 127):
            grp, off = _k_offset(key, dim)
            assert pk[0, 1, grp, off] == x[0, 1, key, dim], (key, dim)
            grp, off = _v_offset(key, dim)
            assert pv[0, 1, grp, off] == x[0, 1, key, dim], (key, dim)


def test_pack_roundtrip_and_shape_checks(packed):
    x = torch.randn(2, 3, 96, 128)
    assert torch.equal(ops.k_from_cache_layout(ops.k_to_cache_layout(x)), x)
    assert torch.equal(ops.v_from_cache_layout(ops.v_to_cache_layout(x)), x)
    with pytest.raises(ValueError):
        ops.kv_cache_shape(1, 1, 100, 128)


def test_lane_fragments_are_mfma_operands(packed):
    """Lane l = 16q + r of slab (t, s) holds A[row r][k = 8q..8q+8] of the
    16x16x32 score MFMA: key 8(r/4) + 4t + r%4, dims 32s + 8q .. +8; lane l of
    V slab dt holds keys 8q .. +8 of dim 16dt + r."""
    x = torch.arange(32 * 128, dtype=torch.float32).view(1, 1, 32, 128)
    pk = ops.k_to_cache_layout(x).view(2, 4, 64, 8)
    pv = ops.v_to_cache_layout(x).view(8, 64, 8)
    for t in range(2):
        for s in range(4):
            for lane in (0, 5, 17, 38, 63):
                q, r = lane // 16, lane % 16
                key = 8 * (r // 4) + 4 * t + r % 4
                assert torch.equal(pk[t, s, lane], x[0, 0, key, 32 * s + 8 * q:32 * s + 8 * q + 8])
    for dt in range(8):
        for lane in (0, 9, 16, 47, 63):
            q, r = lane // 16, lane % 16
            assert torch.equal(pv[dt, lane], x[0, 0, 8 * q:8 * q + 8, 16 * dt + r])


def test_prefill_attention_reference_matches_the_masked_path():
    """ops.reference.prefill_attention (the flash kernel's numerics reference)
    agrees with the decoder's fp32 masked-GEMM prefill attention."""
    import math

    import torch

    from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_TINY, Qwen3Decoder
    from k8s_vgpu_scheduler_amd.ops import reference as ref

    d = Qwen3Decoder(QWEN3_TINY, batch=1, max_ctx=128, device="cpu", native=False)
    L, G, Hkv, D = 48, 4, 2, 128
    q = torch.randn(Hkv, G * L, D).to(torch.bfloat16)
    k = torch.randn(Hkv, L, D).to(torch.bfloat16)
    v = torch.randn(Hkv, L, D).to(torch.bfloat16)
    bufs = d._prefill_bufs(L)
    a = d._prefill_attention(q, k, v, bufs["mask"]).float()
    b = ref.prefill_attention(q, k, v, G * Hkv, 1.0 / math.sqrt(D))
    assert (a - b).abs().max().item() < 2e-2 * b.abs().max().item()
