"""ctypes bindings for ``libmivgpu_ops.so`` (hand-written gfx950 kernels).

The kernels take raw device pointers and the caller's HIP stream, so they are
captured by ``torch.cuda.CUDAGraph`` like any other launch.  On a GPU box the
library MUST load -- ops fail loudly instead of silently falling back to
PyTorch (``require_native()``); the pure-PyTorch reference implementations in
:mod:`k8s_vgpu_scheduler_amd.ops.reference` exist for numerics tests and for
CPU-only development.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

# MIVGPU_OPS_LIB points experiments at an alternative build of the same library.
_LIB_PATH = Path(os.environ.get("MIVGPU_OPS_LIB") or Path(__file__).resolve().parents[1] / "lib" / "libmivgpu_ops.so")
_lib = None


class NativeOpsUnavailable(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            raise NativeOpsUnavailable(
                f"{_LIB_PATH} missing: run `python -m k8s_vgpu_scheduler_amd.utils.build ops`")
        # torch must be initialised first so the HIP runtime it bundles
        # (SONAME libamdhip64.so.7) is the one our library binds to.
        import torch.cuda  # noqa: F401
        L = ctypes.CDLL(str(_LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.mivgpu_rmsnorm.argtypes = [vp, vp, vp, i, i, f, vp]
        L.mivgpu_add_rmsnorm.argtypes = [vp, vp, vp, vp, i, i, f, vp]
        L.mivgpu_embed_rmsnorm.argtypes = [vp, vp, vp, vp, vp, i, i, ctypes.c_longlong, f, vp, vp]
        L.mivgpu_decode_tail.argtypes = [vp, i, i, i, vp, vp, vp, vp, vp]
        L.mivgpu_qk_norm_rope_kv.argtypes = [vp, vp, vp, vp, vp, vp, vp, i, i, i, i, i, f, f, vp]
        L.mivgpu_prefill_qk_norm_rope_kv.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, i, i, i, i, i, i, f, f,
                                                     vp]
        L.mivgpu_decode_attention.argtypes = [vp, vp, vp, vp, vp, vp, vp, i, i, i, i, i, i, f, vp]
        L.mivgpu_prefill_attention.argtypes = [vp, vp, vp, vp, i, i, i, i, f, vp]
        L.mivgpu_tr_read_probe.argtypes = [vp, vp, i, vp]
        L.mivgpu_decode_attention_fused.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i, i, i, i, i,
                                                     i, f, f, f, i, vp]
        L.mivgpu_skinny_gemm_norm_xcomb.argtypes = [vp, vp, vp, vp, i, i, i, i, vp, i, i, i, i, i, i, i, vp, vp,
                                                    vp, i, f, f, vp, vp]
        L.mivgpu_silu_mul.argtypes = [vp, vp, i, i, vp]
        L.mivgpu_hwid_probe.argtypes = [vp, i, vp]
        L.mivgpu_pack_weight.argtypes = [vp, vp, i, i, vp]
        L.mivgpu_unpack_weight.argtypes = [vp, vp, i, i, i, vp]
        L.mivgpu_prefill_gemm.argtypes = [vp, vp, vp, i, i, i, i, i, i, vp]
        L.mivgpu_skinny_gemm.argtypes = [vp, vp, vp, i, i, i, i, i, i, i, i, i, i, vp, vp, vp]
        L.mivgpu_skinny_gemm_norm.argtypes = [vp, vp, vp, i, i, i, i, i, i, i, i, i, i, vp, vp, vp, i, f, f, vp, vp]
        ip, lp = ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_longlong)
        L.mivgpu_mfma_burn.argtypes = [vp, i, i, ctypes.c_uint, vp]
        L.mivgpu_mfma_burn_flops.argtypes = [i, i]
        L.mivgpu_mfma_burn_flops.restype = ctypes.c_double
        L.mivgpu_stream_copy.argtypes = [vp, vp, ctypes.c_longlong, i, vp]
        L.mivgpu_stream_read.argtypes = [vp, ctypes.c_longlong, vp, i, vp]
        L.mivgpu_skinny_plan.argtypes = [i, i, i, i, ip, ip, ip, lp, ip, ip]
        L.mivgpu_decode_chain.argtypes = [ctypes.POINTER(ChainGemm), i, vp, vp]
        for fn in ("mivgpu_rmsnorm", "mivgpu_add_rmsnorm", "mivgpu_qk_norm_rope_kv",
                   "mivgpu_decode_attention", "mivgpu_silu_mul", "mivgpu_ops_attn_split",
                   "mivgpu_hwid_probe", "mivgpu_pack_weight", "mivgpu_skinny_gemm",
                   "mivgpu_skinny_max_m", "mivgpu_skinny_plan", "mivgpu_mfma_burn",
                   "mivgpu_stream_copy", "mivgpu_stream_read", "mivgpu_ops_visible_cus",
                   "mivgpu_ops_kv_packed", "mivgpu_decode_attention_fused", "mivgpu_skinny_gemm_norm",
                   "mivgpu_prefill_qk_norm_rope_kv", "mivgpu_prefill_attention", "mivgpu_unpack_weight",
                   "mivgpu_decode_chain", "mivgpu_chain_counter_words", "mivgpu_chain_err_word",
                   "mivgpu_prefill_gemm"):
            getattr(L, fn).restype = ctypes.c_int
        _lib = L
    return _lib


class ChainGemm(ctypes.Structure):
    """One projection of mivgpu_decode_chain (csrc/ops/skinny_gemm.hip MivgpuChainGemm)."""
    _fields_ = [("wp", ctypes.c_void_p), ("x", ctypes.c_void_p), ("y", ctypes.c_void_p),
                ("M", ctypes.c_int), ("K", ctypes.c_int), ("N", ctypes.c_int), ("ldx", ctypes.c_int),
                ("ldy", ctypes.c_int), ("S", ctypes.c_int), ("scratch", ctypes.c_void_p),
                ("tickets", ctypes.c_void_p), ("rs_part", ctypes.c_void_p), ("rs_nparts", ctypes.c_int),
                ("rs_inv_dim", ctypes.c_float), ("rs_eps", ctypes.c_float), ("ss_out", ctypes.c_void_p)]


def available() -> bool:
    try:
        lib()
        return torch.cuda.is_available()
    except (NativeOpsUnavailable, OSError):
        return False


def require_native():
    """Raise unless the HIP op library is loadable and a GPU is present."""
    if not torch.cuda.is_available():
        raise NativeOpsUnavailable("no GPU visible")
    lib()


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


def _check(rc: int, name: str):
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None):
    out = torch.empty_like(x) if out is None else out
    rows, dim = x.reshape(-1, x.shape[-1]).shape
    _check(lib().mivgpu_rmsnorm(_p(x), _p(w), _p(out), rows, dim, eps, _stream()), "rmsnorm")
    return out


def add_rmsnorm(x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, eps: float,
                out: torch.Tensor | None = None):
    """res += x (in place); returns rmsnorm(res) * w."""
    out = torch.empty_like(x) if out is None else out
    rows, dim = x.reshape(-1, x.shape[-1]).shape
    _check(lib().mivgpu_add_rmsnorm(_p(x), _p(res), _p(w), _p(out), rows, dim, eps, _stream()),
           "add_rmsnorm")
    return out


def embed_rmsnorm(embed: torch.Tensor, tokens: torch.Tensor, w: torch.Tensor | None, eps: float, res: torch.Tensor,
                  out: torch.Tensor | None, ss_out: torch.Tensor | None = None):
    """Decode-step head in one launch: res = embed[tokens] (ids clamped to
    the table), out = rmsnorm(res) * w; ss_out (fp32, >= B) receives the
    rows' sums of squares (out may then be None: the norm-fused decoder)."""
    rows, dim = res.shape
    if (tokens.dtype != torch.int64 or tokens.numel() != rows or embed.shape[1] != dim
            or (out is not None and (out.shape != res.shape or not out.is_contiguous() or w is None))
            or (ss_out is not None and (ss_out.dtype != torch.float32 or ss_out.numel() < rows))
            or (out is None and ss_out is None) or not (embed.is_contiguous() and res.is_contiguous())):
        raise ValueError("embed_rmsnorm: embed [V, D], tokens int64 [B], res / out [B, D] contiguous, ss_out fp32 [B]")
    _check(lib().mivgpu_embed_rmsnorm(_p(embed), _p(tokens), _p(w) if w is not None else None, _p(res),
                                      _p(out) if out is not None else None, rows, dim, embed.shape[0], eps,
                                      _p(ss_out) if ss_out is not None else None, _stream()), "embed_rmsnorm")
    return out


def decode_tail_workspace(rows: int, device) -> torch.Tensor:
    """Zeroed workspace of decode_tail (per-row 64-bit argmax slot + ticket);
    every launch leaves it zero."""
    return torch.zeros(2 * rows, dtype=torch.int64, device=device)


def decode_tail(logits: torch.Tensor, tokens: torch.Tensor, pos: torch.Tensor, seqlens: torch.Tensor,
                work: torch.Tensor):
    """Decode-step tail in one launch: tokens = argmax(logits, -1) (first
    maximum, NaN as the maximum, as torch.argmax), pos += 1, seqlens += 1.
    ``work`` from decode_tail_workspace(rows) (not shared by concurrent calls)."""
    rows, vocab = logits.shape
    if (logits.dtype != torch.bfloat16 or logits.stride(1) != 1 or tokens.dtype != torch.int64
            or pos.dtype != torch.int32 or seqlens.dtype != torch.int32
            or min(tokens.numel(), pos.numel(), seqlens.numel()) < rows
            or work.dtype != torch.int64 or work.numel() < 2 * rows):
        raise ValueError("decode_tail: bf16 logits [B, V], int64 tokens, int32 pos / seqlens, int64 work [2B]")
    _check(lib().mivgpu_decode_tail(_p(logits), logits.stride(0), vocab, rows, _p(tokens), _p(pos), _p(seqlens),
                                    _p(work), _stream()), "decode_tail")
    return tokens


def _check_kv(k_cache, v_cache, B, n_kv_heads, head_dim):
    """Host-side check that both caches are in the layout the kernels index; returns T."""
    T = k_cache.shape[2] * (32 if kv_packed() else 1)
    want = kv_cache_shape(B, n_kv_heads, T, head_dim)
    if tuple(k_cache.shape) != want or tuple(v_cache.shape) != want \
            or not (k_cache.is_contiguous() and v_cache.is_contiguous()):
        raise ValueError(f"KV cache shapes {tuple(k_cache.shape)} / {tuple(v_cache.shape)} do not match "
                         f"the kernels' layout {want} (contiguous)")
    return T


def qk_norm_rope_kv(qkv, q_norm_w, k_norm_w, pos, q_out, k_cache, v_cache, n_q_heads, n_kv_heads,
                    head_dim, eps, theta):
    B = qkv.shape[0]
    max_ctx = _check_kv(k_cache, v_cache, B, n_kv_heads, head_dim)
    _check(lib().mivgpu_qk_norm_rope_kv(_p(qkv), _p(q_norm_w), _p(k_norm_w), _p(pos), _p(q_out),
                                        _p(k_cache), _p(v_cache), B, n_q_heads, n_kv_heads, head_dim,
                                        max_ctx, eps, theta, _stream()), "qk_norm_rope_kv")


def prefill_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, n_q_heads: int, scale: float,
                      out: torch.Tensor | None = None) -> torch.Tensor:
    """Causal GQA flash attention over one prompt (csrc/ops/prefill_attn.hip):
    q [Hkv, G*L, D] head-grouped, k / v [Hkv, L, D] bf16 -> [L, Hq*D] bf16.
    Never materialises the L x L scores."""
    Hkv, GL, D = q.shape
    L = k.shape[1]
    if D != 128 or GL != (n_q_heads // Hkv) * L or tuple(k.shape) != (Hkv, L, D) or k.shape != v.shape:
        raise ValueError(f"prefill_attention shapes q {tuple(q.shape)} k {tuple(k.shape)} v {tuple(v.shape)}")
    if n_q_heads % Hkv or (n_q_heads // Hkv) not in (1, 2, 4, 8):
        raise ValueError(f"GQA group {n_q_heads}/{Hkv} unsupported")
    for t in (q, k, v):
        if t.dtype != torch.bfloat16 or not t.is_contiguous():
            raise ValueError("q, k, v must be contiguous bf16")
    if out is None:
        out = torch.empty(L, n_q_heads * D, dtype=torch.bfloat16, device=q.device)
    if out.numel() < L * n_q_heads * D or not out.is_contiguous():
        raise ValueError("out too small")
    _check(lib().mivgpu_prefill_attention(_p(q), _p(k), _p(v), _p(out), L, n_q_heads, Hkv, D, scale, _stream()),
           "prefill_attention")
    return out


def prefill_qk_norm_rope_kv(qkv, q_norm_w, k_norm_w, pos, q_out, k_plain, v_plain, k_cache, v_cache, cache_b,
                            n_q_heads, n_kv_heads, head_dim, eps, theta):
    """Prompt tokens of one sequence (qkv [L, (Hq+2Hkv)*D], positions pos [L]
    int32) -> QK-norm + RoPE; K/V appended to cache row ``cache_b`` (positions
    >= the cache length dropped); q_out [Hkv, G*L, D] head-grouped, k_plain /
    v_plain [Hkv, L, D] (or None)."""
    L = qkv.shape[0]
    B = k_cache.shape[0]
    max_ctx = _check_kv(k_cache, v_cache, B, n_kv_heads, head_dim)
    if not 0 <= cache_b < B:
        raise ValueError(f"cache row {cache_b} outside [0, {B})")
    if qkv.shape[1] != (n_q_heads + 2 * n_kv_heads) * head_dim or not qkv.is_contiguous():
        raise ValueError(f"qkv shape {tuple(qkv.shape)} does not match the head counts")
    if pos.dtype != torch.int32 or pos.numel() < L:
        raise ValueError("pos must be int32 with one position per row")
    if q_out.numel() < L * n_q_heads * head_dim or not q_out.is_contiguous():
        raise ValueError("q_out too small")
    for t in (k_plain, v_plain):
        if t is not None and (t.numel() < L * n_kv_heads * head_dim or not t.is_contiguous()):
            raise ValueError("k_plain / v_plain too small")
    _check(lib().mivgpu_prefill_qk_norm_rope_kv(_p(qkv), _p(q_norm_w), _p(k_norm_w), _p(pos), _p(q_out),
                                                _p(k_plain) if k_plain is not None else None,
                                                _p(v_plain) if v_plain is not None else None,
                                                _p(k_cache), _p(v_cache), L, cache_b, n_q_heads, n_kv_heads,
                                                head_dim, max_ctx, eps, theta, _stream()),
           "prefill_qk_norm_rope_kv")


def visible_cus() -> int:
    """CUs this process runs on (its HSA_CU_MASK partition, else the whole GPU)."""
    return int(lib().mivgpu_ops_visible_cus())


def attn_split() -> int:
    """Keys per decode-attention partial workgroup (size the workspace with it)."""
    return int(lib().mivgpu_ops_attn_split())


def kv_packed() -> bool:
    """True when the KV caches are fragment-packed (the MFMA attention kernel,
    MIVGPU_ATTN_KERNEL != valu): per (batch, kv-head), 32-key groups of 4096
    elements laid out as the MFMA operands (csrc/ops/model_ops.hip)."""
    return bool(lib().mivgpu_ops_kv_packed())


def kv_cache_shape(B: int, Hkv: int, T: int, D: int) -> tuple:
    """Shape of a K or V cache of logical size [B, Hkv, T, D] in the kernels' layout."""
    if kv_packed():
        if T % 32 or D != 128:
            raise ValueError(f"packed KV cache needs T % 32 == 0 and D == 128 (T={T}, D={D})")
        return (B, Hkv, T // 32, 32 * D)
    return (B, Hkv, T, D)


# Logical [B, H, T, D] viewed as [B, H, g, key factors..., dim factors...] and
# permuted into the packed group order (see the kernel's layout comment):
#   K: key = 8a + 4t + c, dim = 32s + 8q + e -> [t][s][q][a c][e]
#   V: key = 8q + e,      dim = 16dt + r    -> [dt][q][r][e]
def _k_pack_view(k):
    B, H, T, D = k.shape
    return k.reshape(B, H, T // 32, 4, 2, 4, 4, 4, 8).permute(0, 1, 2, 4, 6, 7, 3, 5, 8)


def _v_pack_view(v):
    B, H, T, D = v.shape
    return v.reshape(B, H, T // 32, 4, 8, 8, 16).permute(0, 1, 2, 5, 3, 6, 4)


def k_to_cache_layout(k: torch.Tensor) -> torch.Tensor:
    """Logical [B, Hkv, T, D] K -> contiguous copy in the kernels' layout."""
    if not kv_packed():
        return k.contiguous()
    B, H, T, D = k.shape
    return _k_pack_view(k).contiguous().view(kv_cache_shape(B, H, T, D))


def v_to_cache_layout(v: torch.Tensor) -> torch.Tensor:
    """Logical [B, Hkv, T, D] V -> contiguous copy in the kernels' layout."""
    if not kv_packed():
        return v.contiguous()
    B, H, T, D = v.shape
    return _v_pack_view(v).contiguous().view(kv_cache_shape(B, H, T, D))


def k_from_cache_layout(k: torch.Tensor, D: int = 128) -> torch.Tensor:
    """Kernel-layout K cache -> logical [B, Hkv, T, D]."""
    if not kv_packed():
        return k
    B, H, G, _ = k.shape
    out = torch.empty(B, H, G * 32, D, dtype=k.dtype, device=k.device)
    _k_pack_view(out).copy_(k.view(B, H, G, 2, 4, 4, 4, 4, 8))
    return out


def v_from_cache_layout(v: torch.Tensor, D: int = 128) -> torch.Tensor:
    """Kernel-layout V cache -> logical [B, Hkv, T, D]."""
    if not kv_packed():
        return v
    B, H, G, _ = v.shape
    out = torch.empty(B, H, G * 32, D, dtype=v.dtype, device=v.device)
    _v_pack_view(out).copy_(v.view(B, H, G, 8, 4, 16, 8))
    return out


def decode_attention(q, k_cache, v_cache, seqlens, out, o_part, ml_part, n_q_heads, n_kv_heads,
                     head_dim, nsplit, scale):
    B = q.shape[0]
    max_ctx = _check_kv(k_cache, v_cache, B, n_kv_heads, head_dim)
    need = B * n_q_heads * nsplit
    if nsplit * attn_split() < max_ctx or o_part.numel() < need * head_dim or ml_part.numel() < need * 2:
        raise ValueError(f"attention workspace too small for nsplit={nsplit}, max_ctx={max_ctx}")
    _check(lib().mivgpu_decode_attention(_p(q), _p(k_cache), _p(v_cache), _p(seqlens), _p(out),
                                         _p(o_part), _p(ml_part), B, n_q_heads, n_kv_heads, head_dim,
                                         max_ctx, nsplit, scale, _stream()), "decode_attention")
    return out


def attn_fused_ok(n_q_heads: int, n_kv_heads: int, head_dim: int = 128) -> bool:
    """The one-launch attention (decode_attention_fused) needs the packed KV
    layout and one wave per query head of a group + 2 (key, value)."""
    G = n_q_heads // n_kv_heads
    return (kv_packed() and head_dim == 128 and n_q_heads % n_kv_heads == 0 and G in (1, 2, 4, 6)
            and attn_split() // 32 >= G + 2)


ATTN_MAX_SPLITS = 16
W12_MAX_CTX = 2048


def attn_w12() -> bool:
    """Twelve-wave one-split attention workgroups (mivgpu_decode_attention_fused
    with nsplit 1 and 4 query heads per kv-head); MIVGPU_ATTN_W12=0 turns them
    off (read by the C launcher too)."""
    return os.environ.get("MIVGPU_ATTN_W12", "1") != "0"


def attn_fused_splits(B: int, n_kv_heads: int, max_ctx: int, n_q_heads: int | None = None) -> int:
    """Key splits for decode_attention_fused.  One split per attn_split()
    keys (one 32-key group per wave: several workgroups share a CU and hide
    each other's load latency) up to ATTN_MAX_SPLITS; a longer context keeps
    ATTN_MAX_SPLITS splits (or enough to give every CU two workgroups) whose
    waves loop over several groups, so the workspace and the combine stay
    bounded.  One split per (b, kv-head) writes the output itself (no combine
    launch) but at batch 32 ran slower than 5 splits + combine (43 vs 31 us,
    profiles/README.md section 35).  With four query heads per kv-head and at
    least one (b, kv-head) per visible CU, ONE split on twelve-wave
    workgroups (attn_w12) merges its waves in LDS and writes the output: 25.5
    us per layer with no combine launch vs 26.0 + 4.9 at batch 32 (decode
    step 4.46 vs 4.59 ms, profiles/round6/w12/); up to W12_MAX_CTX keys of
    cache, so that one long row among short ones (continuous batching) is
    never a single workgroup's 8k-key stream.  MIVGPU_ATTN_SPLITS=n forces
    n (0 = one split per attn_split() keys)."""
    full = max(1, -(-max_ctx // attn_split()))
    env = os.environ.get("MIVGPU_ATTN_SPLITS")
    if env is not None and env.strip():
        n = int(env)
        return full if n <= 0 else n
    if (n_q_heads is not None and n_q_heads == 4 * n_kv_heads and attn_w12()
            and B * n_kv_heads >= visible_cus() and max_ctx <= W12_MAX_CTX):
        return 1
    if full <= ATTN_MAX_SPLITS:
        return full
    return min(full, max(ATTN_MAX_SPLITS, -(-2 * visible_cus() // max(1, B * n_kv_heads))))


def decode_attention_fused(qkv, q_norm_w, k_norm_w, pos, seqlens, k_cache, v_cache, out, o_part, ml_part,
                           counters, n_q_heads, n_kv_heads, head_dim, nsplit, scale, eps, theta,
                           defer_combine: bool = False):
    """One launch per layer: QK-norm + RoPE (q heads, new key), KV append at
    pos[b], attention over seqlens[b] keys, split combine -> out [B, Hq*D].
    counters: B*Hkv int32, zero before the first call (left zero after).
    defer_combine: leave only the split partials (o_part / ml_part) for
    PackedLinear.norm_call_xcomb; ``out`` is not written."""
    B = qkv.shape[0]
    max_ctx = _check_kv(k_cache, v_cache, B, n_kv_heads, head_dim)
    need = B * n_q_heads * nsplit
    # any nsplit >= 1 covers max_ctx (each wave loops over its key groups)
    if nsplit < 1 or o_part.numel() < need * head_dim or ml_part.numel() < need * 2:
        raise ValueError(f"attention workspace too small for nsplit={nsplit}, max_ctx={max_ctx}")
    if counters.dtype != torch.int32 or counters.numel() < B * n_kv_heads:
        raise ValueError("counters must be int32 with B * n_kv_heads entries")
    if qkv.shape[1] != (n_q_heads + 2 * n_kv_heads) * head_dim or not qkv.is_contiguous():
        raise ValueError(f"qkv shape {tuple(qkv.shape)} does not match the head counts")
    _check(lib().mivgpu_decode_attention_fused(_p(qkv), _p(q_norm_w), _p(k_norm_w), _p(pos), _p(seqlens),
                                               _p(k_cache), _p(v_cache), _p(out), _p(o_part), _p(ml_part),
                                               _p(counters), B, n_q_heads, n_kv_heads, head_dim, max_ctx,
                                               nsplit, scale, eps, theta, int(bool(defer_combine)), _stream()),
           "decode_attention_fused")
    return out


def silu_mul(gate_up: torch.Tensor, out: torch.Tensor | None = None):
    rows, two_i = gate_up.shape
    inter = two_i // 2
    out = torch.empty(rows, inter, dtype=gate_up.dtype, device=gate_up.device) if out is None else out
    _check(lib().mivgpu_silu_mul(_p(gate_up), _p(out), rows, inter, _stream()), "silu_mul")
    return out


def hwid_probe(blocks: int = 4096) -> torch.Tensor:
    """[blocks, 2] uint32 (HW_REG_HW_ID, HW_REG_XCC_ID) per workgroup."""
    out = torch.zeros(blocks * 2, dtype=torch.int32, device="cuda")
    _check(lib().mivgpu_hwid_probe(_p(out), blocks, _stream()), "hwid_probe")
    torch.cuda.synchronize()
    return out.view(blocks, 2).cpu()


# ------------------------------------------------------- load generators --
def mfma_burn(blocks: int, iters: int, out: torch.Tensor | None = None, seed: int = 1) -> torch.Tensor:
    """Matrix-core load: `blocks` x 4 waves x 8 MFMA chains x `iters` (see loadgen.hip)."""
    out = torch.empty(blocks * 256, dtype=torch.float32, device="cuda") if out is None else out
    _check(lib().mivgpu_mfma_burn(_p(out), blocks, iters, seed, _stream()), "mfma_burn")
    return out


def mfma_burn_flops(blocks: int, iters: int) -> float:
    return float(lib().mivgpu_mfma_burn_flops(blocks, iters))


def stream_copy(src: torch.Tensor, dst: torch.Tensor, blocks: int = 0):
    nbytes = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < nbytes:
        raise ValueError("stream_copy: dst too small")
    _check(lib().mivgpu_stream_copy(_p(src), _p(dst), nbytes, blocks, _stream()), "stream_copy")


def stream_read(src: torch.Tensor, out: torch.Tensor | None = None, blocks: int = 0) -> torch.Tensor:
    """HBM read-only sweep; returns the sum of all 32-bit words as uint64 (in an int64 tensor)."""
    out = torch.zeros(1, dtype=torch.int64, device=src.device) if out is None else out
    _check(lib().mivgpu_stream_read(_p(src), src.numel() * src.element_size(), _p(out), blocks, _stream()),
           "stream_read")
    return out


# ------------------------------------------------------------ skinny GEMM --
EPI_STORE, EPI_SILU_MUL = 0, 1


def skinny_max_m() -> int:
    return int(lib().mivgpu_skinny_max_m())


def pack_weight(w: torch.Tensor) -> torch.Tensor:
    """W[N, K] bf16 -> MFMA-fragment-packed copy (same byte size, flat bf16)."""
    N, K = w.shape
    if w.dtype != torch.bfloat16 or N % 32 or K % 64:
        raise ValueError(f"pack_weight needs bf16 [N%32, K%64], got {tuple(w.shape)} {w.dtype}")
    w = w.contiguous()
    out = torch.empty(N * K, dtype=torch.bfloat16, device=w.device)
    _check(lib().mivgpu_pack_weight(_p(w), _p(out), N, K, _stream()), "pack_weight")
    return out


# One shared row-major scratch per device for prompt-sized GEMMs on packed
# weights (PackedLinear.prompt): the largest projection's bytes, not a second
# copy of every weight (16 GB for Qwen3-8B).
_UNPACK: dict = {}


def unpack_scratch(numel: int, device) -> torch.Tensor:
    key = str(device)
    buf = _UNPACK.get(key)
    if buf is None or buf.numel() < numel:
        buf = _UNPACK[key] = torch.empty(numel, dtype=torch.bfloat16, device=device)
    return buf[:numel]


def unpack_weight(wp: torch.Tensor, N: int, K: int, out: torch.Tensor | None = None,
                  deinterleave: bool = False) -> torch.Tensor:
    """Packed W -> row-major [N, K] (the inverse of pack_weight; with
    ``deinterleave`` the gate/up blocks of interleave_gate_up are put back as
    [gate rows; up rows])."""
    if out is None:
        out = torch.empty(N, K, dtype=torch.bfloat16, device=wp.device)
    _check(lib().mivgpu_unpack_weight(_p(wp), _p(out), N, K, 1 if deinterleave else 0, _stream()),
           "unpack_weight")
    return out.view(N, K)


def interleave_gate_up(w_gu: torch.Tensor) -> torch.Tensor:
    """[2I, K] (gate rows then up rows) -> rows ordered gate[0:32], up[0:32], gate[32:64], ...
    so n-tile pair (2c, 2c+1) of the packed weight is (gate, up) of channel block c."""
    two_i, K = w_gu.shape
    inter = two_i // 2
    return w_gu.view(2, inter // 32, 32, K).transpose(0, 1).reshape(two_i, K)


VARIANT_AUTO, VARIANT_CLASSIC, VARIANT_WIDE, VARIANT_WIDEK = 0, 1, 2, 3


def skinny_plan(M: int, K: int, N: int, epi: int, nt: int = 0, ks: int = 0, S: int = 0, variant: int = 0) -> dict:
    """Launch plan the kernel will use (0 = auto) and the scratch it needs.
    variant: 1 classic (ks = waves splitting K inside a workgroup), 2 wide
    workgroups (ks = waves sharing one LDS X tile); 0 = auto.  The returned
    variant is the kernel that will run (an infeasible wide plan falls back)."""
    c = ctypes
    v_nt, v_ks, v_s, v_t, v_v = c.c_int(nt), c.c_int(ks), c.c_int(S), c.c_int(0), c.c_int(variant)
    v_f = c.c_longlong(0)
    _check(lib().mivgpu_skinny_plan(M, K, N, epi, c.byref(v_nt), c.byref(v_ks), c.byref(v_s), c.byref(v_f),
                                    c.byref(v_t), c.byref(v_v)), "skinny_plan")
    return {"nt": v_nt.value, "ks": v_ks.value, "S": v_s.value, "scratch_floats": v_f.value,
            "tickets": v_t.value, "variant": v_v.value}


EPI_RESID = 2
SS_ROWS = 128   # rows per sum-of-squares slot (csrc/ops/skinny_gemm.hip SS_ROWS)


def prefill_gemm_ok(N: int, K: int) -> bool:
    """The native prefill GEMM takes this weight (tile-major packing, N a
    multiple of 256, K of 64) and is selected (MIVGPU_PREFILL_GEMM=native).
    The default is the library path: measured on MI355X
    (profiles/round5/kern/pgemm.json) the register-staged 256x256 kernel ran
    984 TFLOP/s on the 8192-row qkv against hipBLASLt's 1505 (unpack + GEMM
    291 vs 419 us), and the 8k-token prefill took 127.4 vs 120.7 ms."""
    return (os.environ.get("MIVGPU_PREFILL_GEMM", "lib") == "native" and N % 256 == 0 and K % 64 == 0
            and os.environ.get("MIVGPU_SKINNY_KMAJOR", "0") in ("", "0", "-1"))


def prefill_gemm(wp: torch.Tensor, x: torch.Tensor, N: int, K: int, silu_mul: bool = False,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """Y = X . W^T (or SiLU(gate) * up of an interleaved gate/up weight) for
    prompt-sized X [M, K] bf16 against the fragment-packed W (pack_weight)."""
    if x.dtype != torch.bfloat16 or x.dim() != 2 or x.shape[1] != K or x.stride(1) != 1:
        raise ValueError(f"prefill_gemm: X must be [M, {K}] bf16 with unit column stride, got {tuple(x.shape)}")
    M = x.shape[0]
    cols = N // 2 if silu_mul else N
    if out is None:
        out = torch.empty(M, cols, dtype=torch.bfloat16, device=x.device)
    if out.shape[0] < M or out.shape[1] < cols or out.stride(1) != 1:
        raise ValueError("prefill_gemm: out too small")
    _check(lib().mivgpu_prefill_gemm(_p(wp), _p(x), _p(out), M, K, N, x.stride(0), out.stride(0),
                                     1 if silu_mul else 0, _stream()), "prefill_gemm")
    return out


class PackedLinear:
    """A weight held only in packed form, applied with the skinny MFMA GEMM.

    Owns the zeroed fp32 slabs + tickets of the inter-workgroup split-K
    (sized for the largest plan seen; the kernel leaves them zeroed, so graph
    replays need no memset).  Not safe to call concurrently on two streams.

    ``col_scale`` (an RMSNorm weight of length K) is folded into W's columns
    before packing, so ``norm_call(x, row_scale=...)`` computes
    RMSNorm(x) . W^T with the norm's row scales applied in the epilogue.
    """

    def __init__(self, w: torch.Tensor, silu_mul: bool = False, col_scale: torch.Tensor | None = None):
        self.N, self.K = w.shape
        self.silu_mul = silu_mul
        self.epi = EPI_SILU_MUL if silu_mul else EPI_STORE
        if col_scale is not None:
            if col_scale.shape != (self.K,):
                raise ValueError(f"col_scale must be [{self.K}], got {tuple(col_scale.shape)}")
            w = (w.float() * col_scale.float()[None, :]).to(w.dtype)
        self.wp = pack_weight(interleave_gate_up(w) if silu_mul else w)
        self.variant = VARIANT_AUTO   # kernel used when a call does not ask for one (VARIANT_WIDEK: K-split waves)
        self.scratch = None
        self.tickets = None
        # set once a hipGraph holds the slabs' addresses: growing them then
        # would free memory the graph still writes
        self.frozen = False

    def reserve(self, max_m: int):
        """Size the split-K slabs for every row count up to ``max_m`` (before a
        graph capture, when later calls may use other row counts)."""
        floats = tickets = 0
        for m in range(1, max_m + 1):
            for v in {VARIANT_AUTO, self.variant}:
                pl = skinny_plan(m, self.K, self.N, self.epi, variant=v)
                floats, tickets = max(floats, pl["scratch_floats"]), max(tickets, pl["tickets"])
        self._ensure_scratch(floats, tickets, self.wp.device)

    @property
    def out_features(self) -> int:
        return self.N // 2 if self.silu_mul else self.N

    def _ensure_scratch(self, floats: int, tickets: int, device):
        if self.frozen and ((floats and (self.scratch is None or self.scratch.numel() < floats))
                            or (tickets and (self.tickets is None or self.tickets.numel() < tickets))):
            raise RuntimeError("skinny_gemm: split-K scratch would grow under a captured graph; "
                               "reserve() the row counts before capture")
        if floats and (self.scratch is None or self.scratch.numel() < floats):
            self.scratch = torch.zeros(floats, dtype=torch.float32, device=device)
        if tickets and (self.tickets is None or self.tickets.numel() < tickets):
            self.tickets = torch.zeros(tickets, dtype=torch.int32, device=device)

    def __call__(self, x: torch.Tensor, out: torch.Tensor | None = None, nt: int = 0, ks: int = 0, S: int = 0,
                 variant: int = 0):
        M = x.shape[0]
        if x.dim() != 2 or x.shape[1] != self.K or x.stride(1) != 1:
            raise ValueError(f"skinny_gemm: x must be [M, {self.K}] row-major, got {tuple(x.shape)}")
        if out is None:
            out = torch.empty(M, self.out_features, dtype=torch.bfloat16, device=x.device)
        variant = variant or self.variant
        if 0 < M <= 128:
            pl = skinny_plan(M, self.K, self.N, self.epi, nt, ks, S, variant)
            self._ensure_scratch(pl["scratch_floats"], pl["tickets"], x.device)
        sp = _p(self.scratch) if self.scratch is not None else None
        tp = _p(self.tickets) if self.tickets is not None else None
        _check(lib().mivgpu_skinny_gemm(_p(self.wp), _p(x), _p(out), M, self.K, self.N, x.stride(0),
                                        out.stride(0), self.epi, nt, ks, S, variant, sp, tp, _stream()),
               "skinny_gemm")
        return out

    def prompt(self, x: torch.Tensor) -> torch.Tensor:
        """X . W^T for prompt-sized X (hundreds to thousands of rows), SiLU*up
        for a gate/up weight.  (A folded col_scale stays folded: the caller
        normalises X without a weight.)  The hand-written prefill GEMM
        (csrc/ops/prefill_gemm.hip) reads the packed weight directly, SiLU*up
        in its epilogue; MIVGPU_PREFILL_GEMM=lib (or a shape it does not take)
        unpacks the weight into the shared scratch and runs the library GEMM
        (hipBLASLt) instead."""
        if prefill_gemm_ok(self.N, self.K):
            return prefill_gemm(self.wp, x, self.N, self.K, silu_mul=self.silu_mul)
        w = unpack_weight(self.wp, self.N, self.K, unpack_scratch(self.N * self.K, self.wp.device),
                          deinterleave=self.silu_mul)
        y = torch.nn.functional.linear(x, w)
        return silu_mul(y) if self.silu_mul else y

    def slots(self, M: int) -> int:
        """Sum-of-squares slots a residual call (``norm_call(residual=True)``)
        writes: one per wave-group of the wide plan."""
        return (self.N // 32) // skinny_plan(M, self.K, self.N, EPI_RESID, variant=self._norm_variant())["nt"]

    def _norm_variant(self) -> int:
        # the row-norm fusion runs on the wide kernel, or the K-split one when
        # this projection is set to it
        return VARIANT_WIDEK if self.variant == VARIANT_WIDEK else VARIANT_WIDE

    def xcomb_ok(self, M: int) -> bool:
        """norm_call_xcomb can run: the K-split kernel, one row (batch 1)."""
        return (self.variant == VARIANT_WIDEK and M == 1 and not self.silu_mul and self.K % 128 == 0
                and skinny_plan(M, self.K, self.N, EPI_STORE, variant=VARIANT_WIDEK)["variant"] == VARIANT_WIDEK)

    def norm_call_xcomb(self, parts: tuple, M: int, out: torch.Tensor, residual: bool = False,
                        ss_out: torch.Tensor | None = None):
        """norm_call with X = the split combine of decode-attention partials
        (``decode_attention_fused(..., defer_combine=True)``), done in the
        kernel's X staging: ``parts = (o_part, ml_part, seqlens, nsplit,
        split_keys, max_ctx, n_q_heads)``; K must be n_q_heads * 128."""
        o_part, ml_part, seqlens, nsplit, split_keys, max_ctx, hq = parts
        if not self.xcomb_ok(M) or self.K != hq * 128 or o_part.dtype != torch.float32 or ml_part.dtype != torch.float32:
            raise ValueError("norm_call_xcomb needs the K-split kernel, M <= 4, K = Hq * 128, fp32 partials")
        epi = EPI_RESID if residual else self.epi
        if residual and (ss_out is None or ss_out.numel() < self.slots(M) * SS_ROWS or tuple(out.shape) != (M, self.N)):
            raise ValueError("residual call needs out [M, N], ss_out of slots(M) * SS_ROWS floats")
        pl = skinny_plan(M, self.K, self.N, EPI_STORE, variant=VARIANT_WIDEK)
        self._ensure_scratch(pl["scratch_floats"], pl["tickets"], out.device)
        sp = _p(self.scratch) if self.scratch is not None else None
        tp = _p(self.tickets) if self.tickets is not None else None
        _check(lib().mivgpu_skinny_gemm_norm_xcomb(_p(self.wp), _p(o_part), _p(ml_part), _p(seqlens), nsplit,
                                                   split_keys, max_ctx, hq, _p(out), M, self.K, self.N,
                                                   out.stride(0), epi, 0, 0, sp, tp, None, 0, 0.0, 0.0,
                                                   _p(ss_out) if residual else None, _stream()),
               "skinny_gemm_norm_xcomb")
        return out

    def norm_call(self, x: torch.Tensor, out: torch.Tensor, row_scale: tuple | None = None,
                  residual: bool = False, ss_out: torch.Tensor | None = None, ks: int = 0, S: int = 0):
        """Wide-kernel call with the row-norm fusion (csrc/ops/skinny_gemm.hip):
        * ``row_scale=(slots, nparts, dim, eps)``: multiply row m of X.W^T by
          rsqrt(sum of the nparts sum-of-squares slots / dim + eps);
        * ``residual=True``: ``out`` is the residual stream, updated in place
          (out += X.W^T), and ``ss_out`` receives ``slots(M)`` slots of the new
          rows' sums of squares ([slots * SS_ROWS] fp32)."""
        M = x.shape[0]
        if x.dim() != 2 or x.shape[1] != self.K or x.stride(1) != 1 or not 0 < M <= 128:
            raise ValueError(f"skinny_gemm: x must be [M <= 128, {self.K}] row-major, got {tuple(x.shape)}")
        epi = EPI_RESID if residual else self.epi
        if residual and (self.silu_mul or ss_out is None or ss_out.numel() < self.slots(M) * SS_ROWS
                         or tuple(out.shape) != (M, self.N)):
            raise ValueError("residual call needs out [M, N], ss_out of slots(M) * SS_ROWS floats, no SiLU")
        variant = self._norm_variant()
        pl = skinny_plan(M, self.K, self.N, EPI_STORE if residual else epi, 0, ks, S, variant=variant)
        if pl["variant"] not in (VARIANT_WIDE, VARIANT_WIDEK):
            raise ValueError(f"row-norm fusion needs the wide or K-split kernel; plan {pl}")
        self._ensure_scratch(pl["scratch_floats"], pl["tickets"], x.device)
        sp = _p(self.scratch) if self.scratch is not None else None
        tp = _p(self.tickets) if self.tickets is not None else None
        rs, nparts, inv_dim, eps = None, 0, 0.0, 0.0
        if row_scale is not None:
            part, nparts, dim, eps = row_scale
            if part.dtype != torch.float32 or part.numel() < nparts * SS_ROWS or nparts <= 0:
                raise ValueError("row_scale slots must be fp32 [nparts * SS_ROWS]")
            rs, inv_dim = _p(part), 1.0 / dim
        _check(lib().mivgpu_skinny_gemm_norm(_p(self.wp), _p(x), _p(out), M, self.K, self.N, x.stride(0),
                                             out.stride(0), epi, 0, ks, S, variant, sp, tp, rs, nparts,
                                             inv_dim, eps, _p(ss_out) if residual else None, _stream()),
               "skinny_gemm_norm")
        return out


# ------------------------------------------------------ chained launch --
def chain_counter_words() -> int:
    return int(lib().mivgpu_chain_counter_words())


def chain_counters(device) -> torch.Tensor:
    """Zeroed counters of one chained launch sequence (left zero by every
    launch except the give-up flag, chain_err_word(): nonzero = a wait timed
    out)."""
    return torch.zeros(chain_counter_words(), dtype=torch.int32, device=device)


def chain_err_word() -> int:
    return int(lib().mivgpu_chain_err_word())


class DecodeChain:
    """o_proj (+ residual) -> gate_up (+ SiLU*up) -> down (+ residual) -> the
    next layer's qkv as ONE launch (csrc/ops/skinny_gemm.hip
    decode_chain_kernel): each projection's workgroups are dispatched in the
    previous one's tail, issue their first weight loads, and wait in-kernel
    for the producers of their inputs -- one ramp and drain instead of four.
    Every buffer is bound at construction (static decode buffers), so a call
    is one C call (and one node of a captured graph).

    Each projection is ``(pl, x, y)`` plus ``rs=(slots, nparts, dim, eps)``
    (row scales, gate_up / qkv) or ``ss=slots`` (residual update, o_proj /
    down); ``None`` leaves it out.  ``W``: waves per workgroup (2 or 4);
    ``down_splits``: the down projection's inter-workgroup k-split."""

    def __init__(self, o=None, gu=None, d=None, qkv=None, W: int = 2, down_splits: int = 4, ctr=None):
        self.W = W
        arr = (ChainGemm * 4)()
        self._keep = []
        for i, spec in enumerate((o, gu, d, qkv)):
            if spec is None:
                continue
            pl, x, y = spec["pl"], spec["x"], spec["y"]
            M = x.shape[0]
            S = down_splits if i == 2 else 1
            if S > 1:
                plan = skinny_plan(M, pl.K, pl.N, EPI_STORE, nt=1, ks=W, S=S, variant=VARIANT_WIDE)
                pl._ensure_scratch(plan["scratch_floats"], plan["tickets"], x.device)
            g = arr[i]
            g.wp, g.x, g.y = self._ptr(pl.wp), self._ptr(x), self._ptr(y)
            g.M, g.K, g.N, g.ldx, g.ldy, g.S = M, pl.K, pl.N, x.stride(0), y.stride(0), S
            g.scratch = self._ptr(pl.scratch) if S > 1 else None
            g.tickets = self._ptr(pl.tickets) if S > 1 else None
            if spec.get("rs") is not None:
                part, nparts, dim, eps = spec["rs"]
                g.rs_part, g.rs_nparts, g.rs_inv_dim, g.rs_eps = self._ptr(part), nparts, 1.0 / dim, eps
            if spec.get("ss") is not None:
                g.ss_out = self._ptr(spec["ss"])
            self._keep.append(spec)
        self.arr = arr
        dev = (o or gu or d or qkv)["x"].device
        self.ctr = chain_counters(dev) if ctr is None else ctr

    def _ptr(self, t):
        self._keep.append(t)
        return t.data_ptr()

    def __call__(self):
        _check(lib().mivgpu_decode_chain(self.arr, self.W, _p(self.ctr), _stream()), "decode_chain")

    def gave_up(self) -> bool:
        return int(self.ctr[chain_err_word()].item()) != 0
