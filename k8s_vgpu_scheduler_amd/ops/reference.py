"""Plain-PyTorch fp32 references of the HIP ops (numerics tests, CPU dev path)."""

from __future__ import annotations

import math

import torch


def rmsnorm(x, w, eps):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(x.dtype)


def add_rmsnorm(x, res, w, eps):
    res.copy_((res.float() + x.float()).to(res.dtype))
    return rmsnorm(res, w, eps)


def rope_neox(x, pos, theta):
    """x: [B, H, D] fp32, pos: [B] -> rotate-half RoPE."""
    D = x.shape[-1]
    half = D // 2
    inv_freq = theta ** (-(2.0 * torch.arange(half, dtype=torch.float32, device=x.device)) / D)
    ang = pos.float()[:, None] * inv_freq[None, :]  # [B, half]
    c, s = torch.cos(ang)[:, None, :], torch.sin(ang)[:, None, :]
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


def qk_norm_rope_kv(qkv, q_norm_w, k_norm_w, pos, q_out, k_cache, v_cache, n_q_heads, n_kv_heads,
                    head_dim, eps, theta):
    B = qkv.shape[0]
    x = qkv.float().view(B, n_q_heads + 2 * n_kv_heads, head_dim)
    q = x[:, :n_q_heads]
    k = x[:, n_q_heads:n_q_heads + n_kv_heads]
    v = x[:, n_q_heads + n_kv_heads:]

    def hn(t, w):
        return t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + eps) * w.float()

    q = rope_neox(hn(q, q_norm_w), pos, theta)
    k = rope_neox(hn(k, k_norm_w), pos, theta)
    q_out.copy_(q.to(q_out.dtype))
    for b in range(B):
        p = int(pos[b])
        k_cache[b, :, p] = k[b].to(k_cache.dtype)
        v_cache[b, :, p] = v[b].to(v_cache.dtype)


def decode_attention(q, k_cache, v_cache, seqlens, n_q_heads, n_kv_heads, head_dim, scale=None):
    """q: [B, Hq, D]; caches [B, Hkv, T, D]; returns [B, Hq, D] in q.dtype."""
    B = q.shape[0]
    G = n_q_heads // n_kv_heads
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    out = torch.empty_like(q)
    for b in range(B):
        L = int(seqlens[b])
        k = k_cache[b, :, :L].float().repeat_interleave(G, dim=0)  # [Hq, L, D]
        v = v_cache[b, :, :L].float().repeat_interleave(G, dim=0)
        s = torch.einsum("hd,hld->hl", q[b].float(), k) * scale
        p = torch.softmax(s, dim=-1)
        out[b] = torch.einsum("hl,hld->hd", p, v).to(q.dtype)
    return out


def silu_mul(gate_up):
    i = gate_up.shape[-1] // 2
    g, u = gate_up[..., :i].float(), gate_up[..., i:].float()
    return (torch.nn.functional.silu(g) * u).to(gate_up.dtype)


def prefill_attention(q, k, v, n_q_heads, scale):
    """fp32 causal GQA attention: q [Hkv, G*L, D] head-grouped, k / v [Hkv, L, D]
    -> [L, Hq*D] (the numerics reference of ops.prefill_attention)."""
    Hkv, GL, D = q.shape
    L = k.shape[1]
    G = GL // L
    qf = q.float().view(Hkv, G, L, D)
    sc = torch.einsum("hgld,hkd->hglk", qf, k.float()) * scale
    causal = torch.ones(L, L, dtype=torch.bool, device=q.device).triu(1)
    sc = sc.masked_fill(causal, float("-inf"))
    o = torch.einsum("hglk,hkd->hgld", torch.softmax(sc, dim=-1), v.float())
    return o.permute(2, 0, 1, 3).reshape(L, Hkv * G * D)
