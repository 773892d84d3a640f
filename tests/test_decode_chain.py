"""Chained decode launch (csrc/ops/skinny_gemm.hip decode_chain_kernel): the
ctypes mirror of its argument struct and the host-side plan checks, on the
CPU (the library loads without a GPU; no launch happens on these paths)."""

import ctypes

import pytest

torch = pytest.importorskip("torch")

from k8s_vgpu_scheduler_amd import ops  # noqa: E402


@pytest.fixture(scope="module")
def L():
    try:
        return ops.lib()
    except (ops.NativeOpsUnavailable, OSError) as e:
        pytest.skip(f"ops library unavailable: {e}")


def test_chain_struct_layout_matches_c(L):
    out = (ctypes.c_longlong * 12)()
    L.mivgpu_chain_gemm_layout(out)
    G = ops.ChainGemm
    want = [ctypes.sizeof(G)] + [getattr(G, f).offset for f in
                                 ("wp", "x", "y", "M", "S", "scratch", "tickets", "rs_part", "rs_nparts", "rs_eps",
                                  "ss_out")]
    assert list(out) == want


def test_counter_words(L):
    # 12 counters, each on its own 128-byte line; the give-up flag is the 4th
    assert ops.chain_counter_words() == 12 * 32
    assert ops.chain_err_word() == 3 * 32


def _gemm(wp, x, y, M, K, N, S=1, rs=0, ss=0):
    g = ops.ChainGemm()
    g.wp, g.x, g.y = wp, x, y
    g.M, g.K, g.N, g.ldx, g.ldy, g.S = M, K, N, K, N if not rs else N // 2, S
    if rs:
        g.rs_part, g.rs_nparts, g.rs_inv_dim, g.rs_eps = rs, 128, 1 / 4096, 1e-6
    if ss:
        g.ss_out = ss
    return g


def _call(L, gemms, W=2):
    arr = (ops.ChainGemm * 4)(*gemms)
    ctr = (ctypes.c_int * (12 * 32))()
    return L.mivgpu_decode_chain(arr, W, ctypes.cast(ctr, ctypes.c_void_p), None)


# fake device addresses: the plan checks compare and never dereference them
RES, ACT, ATTN, SSA, SSB, WO, WGU, WD = (0x1000 * (i + 1) for i in range(8))


def test_chain_rejects_broken_links(L):
    o = _gemm(WO, ATTN, RES, 32, 4096, 4096, ss=SSB)
    gu = _gemm(WGU, RES, ACT, 32, 4096, 24576, rs=SSB)
    gu.ldy = 12288
    bad = _gemm(WGU, ATTN, ACT, 32, 4096, 24576, rs=SSB)   # gate_up must read o_proj's output
    bad.ldy = 12288
    none = ops.ChainGemm()
    assert _call(L, [o, bad, none, none]) != 0
    bad_rs = _gemm(WGU, RES, ACT, 32, 4096, 24576, rs=SSA)   # ... and its slots
    bad_rs.ldy = 12288
    assert _call(L, [o, bad_rs, none, none]) != 0
    # down must read gate_up's output with K = N_gu / 2
    d = _gemm(WD, RES, RES, 32, 12288, 4096, S=4, ss=SSA)
    d.scratch, d.tickets = 0x9000, 0xa000
    assert _call(L, [o, gu, d, none]) != 0


def test_chain_rejects_unsupported_shapes(L):
    none = ops.ChainGemm()
    # more than 32 rows, waves other than 2 / 4, a split without scratch
    assert _call(L, [_gemm(WO, ATTN, RES, 64, 4096, 4096, ss=SSB), none, none, none]) != 0
    assert _call(L, [_gemm(WO, ATTN, RES, 32, 4096, 4096, ss=SSB), none, none, none], W=3) != 0
    d = _gemm(WD, ACT, RES, 32, 12288, 4096, S=4, ss=SSA)
    assert _call(L, [none, none, d, none]) != 0
    # o_proj needs its slots buffer
    assert _call(L, [_gemm(WO, ATTN, RES, 32, 4096, 4096), none, none, none]) != 0
