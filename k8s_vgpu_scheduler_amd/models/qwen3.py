"""Qwen3-architecture decoder for the isolation benchmark (random-init weights).

The reference's only benchmark is vLLM serving Qwen3-8B bf16 at TP=1
(benchmarks/ai-benchmark/Dockerfile:7-9, benchmark.py:72-75) inside a HAMi
slice vs. natively.  This module is the MI355X-native stand-in for that
workload: a Qwen3-8B-shaped decoder (GQA 32q/8kv x 128, per-head QK RMSNorm,
NeoX RoPE theta 1e6, SwiGLU 12288, vocab 151936) whose decode step runs
  * every weight-streaming projection of the decode step (qkv, o_proj,
    gate_up with SiLU*up fused into its epilogue, down, lm_head) on the
    hand-written skinny MFMA GEMM (csrc/ops/skinny_gemm.hip) over
    fragment-packed weights, for batch <= 32: the wide variant (workgroups
    sharing an LDS X tile) for gate_up / down / lm_head, the K-split variant
    (skinny_widek_kernel) for qkv and o_proj (the kernel trace,
    profiles/round4/bench/decode_trace_b32.json);
  * the prompt (prefill) projections: up to 1023 rows in 128-row chunks on
    the skinny kernels, longer prompts on the packed weight unpacked once
    into a shared scratch and hipBLASLt (PackedLinear.prompt; the hand-written
    packed-weight GEMM, csrc/ops/prefill_gemm.hip, with
    MIVGPU_PREFILL_GEMM=native), the causal attention on the flash kernel
    (csrc/ops/prefill_attn.hip);
  * every other op on the hand-written gfx950 kernels of libmivgpu_ops.so,
  * the whole step captured in one hipGraph (launch overhead -> one replay).
No network: weights are random normal(0, 0.02) of the exact architecture.
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from k8s_vgpu_scheduler_amd import ops
from k8s_vgpu_scheduler_amd.ops import reference as ref


@dataclass(frozen=True)
class Qwen3Config:
    name: str = "Qwen3-8B"
    hidden: int = 4096
    layers: int = 36
    heads: int = 32
    kv_heads: int = 8
    head_dim: int = 128
    intermediate: int = 12288
    vocab: int = 151936
    rope_theta: float = 1_000_000.0
    eps: float = 1e-6
    tie_embeddings: bool = False

    @property
    def qkv_dim(self) -> int:
        return (self.heads + 2 * self.kv_heads) * self.head_dim

    def param_count(self) -> int:
        h, l = self.hidden, self.layers
        per_layer = (self.qkv_dim * h + self.heads * self.head_dim * h + 2 * self.intermediate * h
                     + self.intermediate * h + 2 * h + 2 * self.head_dim)
        emb = self.vocab * h * (1 if self.tie_embeddings else 2)
        return l * per_layer + emb + h


QWEN3_8B = Qwen3Config()
# Same family, tiny: CPU tests and GPU smoke.
QWEN3_TINY = Qwen3Config(name="Qwen3-tiny", hidden=512, layers=2, heads=8, kv_heads=2,
                         head_dim=128, intermediate=1024, vocab=4096)


class Qwen3Weights:
    def __init__(self, cfg: Qwen3Config, device, dtype=torch.bfloat16, seed: int = 0):
        g = torch.Generator(device=device)
        g.manual_seed(seed)
        std = 0.02

        def rnd(*shape):
            return (torch.randn(*shape, generator=g, device=device, dtype=torch.float32) * std).to(dtype)

        def ones(n):
            # Norm weights around 1 so activations stay O(1) through 36 layers.
            return (1.0 + 0.05 * torch.randn(n, generator=g, device=device)).to(dtype)

        h = cfg.hidden
        self.embed = rnd(cfg.vocab, h)
        self.layers = []
        for _ in range(cfg.layers):
            self.layers.append(dict(
                ln1=ones(h), ln2=ones(h),
                wqkv=rnd(cfg.qkv_dim, h),
                q_norm=ones(cfg.head_dim), k_norm=ones(cfg.head_dim),
                wo=rnd(h, cfg.heads * cfg.head_dim),
                wgu=rnd(2 * cfg.intermediate, h),
                wd=rnd(h, cfg.intermediate),
            ))
        self.final_norm = ones(h)
        self.lm_head = self.embed if cfg.tie_embeddings else rnd(cfg.vocab, h)


def _gpu_shared() -> bool:
    """This process runs on part of a GPU: a CU mask, or a core limit the
    temporal governor enforces (the device plugin's grant)."""
    if os.environ.get("HSA_CU_MASK"):
        return True
    lim = os.environ.get("HIP_DEVICE_CORE_LIMIT", "")
    try:
        return bool(lim) and 0 < float(lim) < 100
    except ValueError:
        return False


class Qwen3Decoder:
    """Static-shape batched decoder with a persistent KV cache.

    ``native=True`` runs the HIP kernels (required on GPU); ``native=False``
    uses the fp32 PyTorch references (CPU tests).
    """

    def __init__(self, cfg: Qwen3Config, batch: int, max_ctx: int, device="cuda",
                 native: bool | None = None, seed: int = 0, skinny: bool | None = None):
        self.cfg = cfg
        self.B = batch
        self.device = torch.device(device)
        self.native = (self.device.type == "cuda") if native is None else native
        # KV length padded to whole 32-key groups (the packed KV layout)
        self.T = -(-max_ctx // 32) * 32
        if self.native:
            ops.require_native()
        self.w = Qwen3Weights(cfg, self.device, seed=seed)
        shapes_ok = cfg.hidden % 64 == 0 and cfg.intermediate % 64 == 0 and cfg.vocab % 64 == 0
        if skinny is None:
            skinny = os.environ.get("MIVGPU_SKINNY_GEMM", "1") != "0"
            skinny = skinny and self.native and batch <= 32 and shapes_ok
        self.skinny = skinny
        # The wide-workgroup skinny kernel (X staged once per workgroup in LDS)
        # beats hipBLASLt on gate_up (+SiLU fused), down and lm_head at 64 and
        # 256 CUs, and on o_proj inside a CU partition; qkv stays on hipBLASLt
        # (profiles/gemm_wide_*.json).
        self.skinny_gate_up = skinny
        # o_proj on the whole chip: the wide kernel up to 8 rows (1 row 10.4 vs
        # 15.5 us, 8 rows 11.3 vs 15.7), hipBLASLt from 32 (13.3 vs 15.2,
        # profiles/gemm_wide_plan_full.json) -- batch-1 serving takes the former
        self.skinny_o = skinny and (ops.visible_cus() <= int(os.environ.get("MIVGPU_SLICE_PLAN_CUS", "96"))
                                    or batch <= 16)
        # qkv joins them in partitions: hipBLASLt vs wide kernel at 32 CUs
        # 50.7 vs 40.7 us, 64 CUs 27.9 vs 29.6, 128 CUs 20.9 vs 17.5, whole
        # GPU 15.2 vs 17.0 (profiles/cu32/, cu128/, gemm_wide_plan_*.json).
        self.skinny_qkv = skinny and ops.visible_cus() <= int(os.environ.get("MIVGPU_QKV_WIDE_CUS", "160"))
        # Row-norm fusion (MIVGPU_NORM_FUSED=1; off by default): every
        # projection on the wide kernel; the RMSNorm weights are folded into
        # the columns of qkv / gate_up / lm_head, o_proj and down update the
        # residual stream in their epilogue and write per-row sums of squares,
        # and the next projection applies rsqrt(mean + eps) per row in its
        # epilogue -- no add+RMSNorm launches (csrc/ops/skinny_gemm.hip).
        # Round 2, with qkv / o_proj on the wide kernel: 64-CU slice 8.85 vs
        # 8.87 ms/step, whole GPU 4.97 vs 4.92 (profiles/README.md section 14).
        # Default on since the residual epilogue sums its squares through LDS
        # (was 80 cross-lane shuffles per lane: +3 us per call): whole GPU
        # 4.62 vs 4.80 ms at batch 32, 3.36 vs 3.52 at batch 1, 64 CUs 8.63 vs
        # 8.75, 32 CUs 14.45 vs 14.59 (profiles/README.md section 36).
        self.norm_fused = skinny and os.environ.get("MIVGPU_NORM_FUSED", "1") == "1"
        if self.norm_fused:
            self.skinny_o = True
        # K-split wide kernel (csrc/ops/skinny_gemm.hip skinny_widek_kernel) for
        # the small projections on the whole chip, where the wide kernel leaves
        # CUs idle and hipBLASLt is slower: qkv 13.6 vs 15.1 us, o_proj 12.2 vs
        # 13.3 at 32 rows; 11.6 vs 14.3 / 10.0 vs 10.6 at 1 row
        # (profiles/round3/widek_gemm.json).  Inside a CU partition the tuned
        # wide plans stay.  MIVGPU_WIDEK=qkv,o,down,gu picks the set, "off" none.
        # A half-GPU partition (97-160 CUs) takes o_proj only: 128 CUs decode
        # 5.80 ms vs 6.00 with the wide kernel, qkv there loses (6.09,
        # profiles/README.md section 36).
        wk_env = os.environ.get("MIVGPU_WIDEK")
        if wk_env is None:
            cus = ops.visible_cus() if self.native else 0
            wk_env = "qkv,o" if cus > 160 else ("o" if cus > 96 else "")
        widek = {p for p in wk_env.split(",") if p and p != "off"} if skinny else set()
        if "qkv" in widek:
            self.skinny_qkv = True
        if "o" in widek:
            self.skinny_o = True
        if self.skinny:
            # Keep only the packed copies (no duplicate 16 GB of weights).
            # batch-1 serving on the whole chip keeps the plain gate_up too, for
            # prompts (hipBLASLt + SiLU 58 vs wide 93 us at 128 rows; +201
            # MB/layer); qkv keeps it wherever it runs on the K-split kernel
            # (hipBLASLt 25 vs wide 50 us at 128 rows; +50 MB/layer).  With the
            # norm fusion the packed copies carry the RMSNorm weight in their
            # columns and the plain ones stay unscaled (prefill normalises first).
            keep_gu = batch <= 16 and ops.visible_cus() > int(os.environ.get("MIVGPU_SLICE_PLAN_CUS", "96"))
            keep_qkv = "qkv" in widek and ops.visible_cus() > 160
            for lw in self.w.layers:
                if self.norm_fused:
                    lw["pqkv"] = ops.PackedLinear(lw["wqkv"] if keep_qkv else lw.pop("wqkv"), col_scale=lw["ln1"])
                    lw["pgu"] = ops.PackedLinear(lw["wgu"] if keep_gu else lw.pop("wgu"), silu_mul=True,
                                                 col_scale=lw["ln2"])
                else:
                    if self.skinny_gate_up:
                        lw["pgu"] = ops.PackedLinear(lw["wgu"] if keep_gu else lw.pop("wgu"), silu_mul=True)
                    if self.skinny_qkv:
                        lw["pqkv"] = ops.PackedLinear(lw["wqkv"] if keep_qkv else lw.pop("wqkv"))
                if self.skinny_o:
                    # on the whole chip the plain copy stays for prompt-sized
                    # GEMMs (hipBLASLt 24.6 vs wide 46 us at 128 rows; +34 MB/layer)
                    keep = ops.visible_cus() > int(os.environ.get("MIVGPU_SLICE_PLAN_CUS", "96"))
                    lw["po"] = ops.PackedLinear(lw["wo"] if keep else lw.pop("wo"))
                # the plain down weight too where gate_up keeps its own: an
                # 8192-token prompt otherwise unpacks it for the library GEMM
                # in every layer (+100 MB/layer)
                keep_d = keep_gu and os.environ.get("MIVGPU_KEEP_PLAIN_DOWN", "1") == "1"
                lw["pd"] = ops.PackedLinear(lw["wd"] if keep_d else lw.pop("wd"))
                for key, name in (("pqkv", "qkv"), ("po", "o"), ("pd", "down"), ("pgu", "gu")):
                    if name in widek and key in lw:
                        lw[key].variant = ops.VARIANT_WIDEK
            # lm_head stays unscaled under the norm fusion: its 2374 workgroups
            # would each reduce the last down projection's 128 sum-of-squares
            # slots (204.6 vs 191.7 us); one RMSNorm launch (5 us) is cheaper
            self.p_lm = ops.PackedLinear(self.w.lm_head)
            if not cfg.tie_embeddings:
                self.w.lm_head = None
            torch.cuda.empty_cache()
        dt = torch.bfloat16
        kvshape = (batch, cfg.kv_heads, self.T, cfg.head_dim)
        # K/V in the attention kernel's layout (fragment-packed 32-key groups
        # for the MFMA kernel: ops.kv_cache_shape); the fp32 reference path
        # keeps [B, Hkv, T, D] rows.
        self.kv_native_layout = self.native and ops.kv_packed()
        pshape = ops.kv_cache_shape(*kvshape) if self.native else kvshape
        self.k_cache = [torch.zeros(pshape, dtype=dt, device=self.device) for _ in range(cfg.layers)]
        self.v_cache = [torch.zeros(pshape, dtype=dt, device=self.device) for _ in range(cfg.layers)]
        self.tokens = torch.zeros(batch, dtype=torch.long, device=self.device)
        self.pos = torch.zeros(batch, dtype=torch.int32, device=self.device)
        self.seqlens = torch.ones(batch, dtype=torch.int32, device=self.device)
        h = cfg.hidden
        # Static activation buffers (graph-capture friendly).
        self.res = torch.zeros(batch, h, dtype=dt, device=self.device)
        self.h = torch.zeros(batch, h, dtype=dt, device=self.device)
        self.q = torch.zeros(batch, cfg.heads, cfg.head_dim, dtype=dt, device=self.device)
        self.attn = torch.zeros(batch, cfg.heads * cfg.head_dim, dtype=dt, device=self.device)
        self.act = torch.zeros(batch, cfg.intermediate, dtype=dt, device=self.device)
        self.mlp_out = torch.zeros(batch, h, dtype=dt, device=self.device)
        self.o_out = torch.zeros(batch, h, dtype=dt, device=self.device)
        self.logits = torch.zeros(batch, cfg.vocab, dtype=dt, device=self.device)
        if self.norm_fused or self.skinny_qkv:
            self.qkv_buf = torch.zeros(batch, cfg.qkv_dim, dtype=dt, device=self.device)
        # Chained projections (MIVGPU_CHAIN=1, norm fusion, batch <= 32):
        # o_proj -> gate_up -> down -> the next layer's qkv as one launch whose
        # workgroups wait in-kernel for their inputs (ops.DecodeChain), two
        # launches per layer with the attention.  MIVGPU_CHAIN_W: waves per
        # workgroup (2: gate_up / down at their tuned wide plans, o_proj / qkv
        # on 2-wave K-split workgroups); MIVGPU_CHAIN_DOWN_S: down's k-split.
        # MIVGPU_CHAIN=gd chains gate_up -> down only (o_proj / qkv stay on
        # their own 4-wave K-split launches).
        self.chain_mode = os.environ.get("MIVGPU_CHAIN", "0")
        self.chain = self.norm_fused and batch <= 32 and self.chain_mode in ("1", "gd")
        if self.chain and _gpu_shared():
            # the chain's workgroups wait in-kernel for their producers: on a
            # CU-masked or time-shared GPU they may never be co-resident, the
            # kernel gives up after its spin timeout and the step is wrong
            # (ADVICE r4), so it is refused there
            import warnings
            warnings.warn("MIVGPU_CHAIN ignored: the GPU is partitioned or time-shared (HSA_CU_MASK / core limit)")
            self.chain = False
        self.chain_w = int(os.environ.get("MIVGPU_CHAIN_W", "2"))
        self.chain_down_s = int(os.environ.get("MIVGPU_CHAIN_DOWN_S", "4"))
        if self.norm_fused:
            l0 = self.w.layers[0]
            self.slots_o, self.slots_d = l0["po"].slots(batch), l0["pd"].slots(batch)
            n = max(self.slots_o, self.slots_d, 1) * ops.SS_ROWS
            if self.chain:
                # the chain's o_proj (K-split) and down (wide, one tile per
                # wave) write one slot per 32-column tile
                self.chain_slots_o, self.chain_slots_d = l0["po"].N // 32, l0["pd"].N // 32
                n = max(n, self.chain_slots_o * ops.SS_ROWS, self.chain_slots_d * ops.SS_ROWS)
            self.ss_a = torch.zeros(n, dtype=torch.float32, device=self.device)   # before qkv / lm_head
            self.ss_b = torch.zeros(n, dtype=torch.float32, device=self.device)   # before gate_up
            self.ss_pf = torch.zeros(ops.SS_ROWS, dtype=torch.float32, device=self.device)   # prefill chunks
        # One launch per layer for QK-norm + RoPE + KV append + attention +
        # split combine (csrc/ops/model_ops.hip decode_attn_fused_kernel);
        # MIVGPU_ATTN_FUSED=0 runs the three separate kernels.
        self.attn_fused = (self.native and os.environ.get("MIVGPU_ATTN_FUSED", "1") != "0"
                           and ops.attn_fused_ok(cfg.heads, cfg.kv_heads, cfg.head_dim))
        # key splits: the fused kernel covers the context with any count
        # (ops.attn_fused_splits); the unfused one needs attn_split() keys each
        if self.attn_fused:
            self.nsplit = ops.attn_fused_splits(batch, cfg.kv_heads, self.T, cfg.heads)
        else:
            self.nsplit = max(1, math.ceil(self.T / (ops.attn_split() if self.native else 256)))
        self.o_part = torch.zeros(batch * cfg.heads * self.nsplit * cfg.head_dim, dtype=torch.float32,
                                  device=self.device)
        self.ml_part = torch.zeros(batch * cfg.heads * self.nsplit * 2, dtype=torch.float32,
                                   device=self.device)
        self.attn_counters = (torch.zeros(batch * cfg.kv_heads, dtype=torch.int32, device=self.device)
                              if self.attn_fused else None)
        # Batch 1 under the norm fusion with o_proj on the K-split kernel: the
        # attention leaves its split partials and o_proj builds the combined
        # row in LDS before its W loop (csrc/ops/skinny_gemm.hip xcomb_row),
        # one launch fewer per layer: o_proj 13.2 us vs 11.4 + 4.9 for the
        # combine launch (profiles/README.md section 36).  MIVGPU_ATTN_XCOMB=0
        # keeps the combine kernel.
        self.xcomb = None
        if (self.norm_fused and self.attn_fused and 1 < self.nsplit <= 8 and not self.chain
                and self.nsplit == math.ceil(self.T / ops.attn_split())
                and os.environ.get("MIVGPU_ATTN_XCOMB", "1") != "0"
                and self.w.layers[0]["po"].xcomb_ok(batch)):
            self.xcomb = (self.o_part, self.ml_part, self.seqlens, self.nsplit, ops.attn_split(), self.T, cfg.heads)
        # plan overrides of the two big projections, "waves,split" (A/B runs;
        # unset = the planner's choice)
        def plan_env(name):
            v = os.environ.get(name, "")
            if not v:
                return {}
            wv, sp = (int(x) for x in v.split(","))
            return {"ks": wv, "S": sp}
        self._gu_plan, self._d_plan = plan_env("MIVGPU_GU_PLAN"), plan_env("MIVGPU_DOWN_PLAN")
        if self.native and (self._gu_plan or self._d_plan):
            for lw in self.w.layers:
                for key, pl in (("pgu", self._gu_plan), ("pd", self._d_plan)):
                    if pl and key in lw:
                        plan = ops.skinny_plan(batch, lw[key].K, lw[key].N, lw[key].epi, ks=pl["ks"], S=pl["S"],
                                               variant=ops.VARIANT_WIDE)
                        lw[key]._ensure_scratch(plan["scratch_floats"], plan["tickets"], self.device)
        self._chains = self._build_chains() if self.chain else None
        self.graph = None
        self._tail_work = ops.decode_tail_workspace(batch, self.device) if self.native else None
        self._pf = {}          # prefill bucket length -> static buffers (+ captured graph)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        # RMSNorm without a weight (the packed copies carry it folded in)
        self._ones = torch.ones(cfg.hidden, dtype=torch.bfloat16, device=self.device)

    # ------------------------------------------------------------- setup --
    def fill_context(self, ctx_len: int, seed: int = 1):
        """Synthetic prompt state: random KV for the first ctx_len positions."""
        assert 0 < ctx_len < self.T
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        shape = (self.B, self.cfg.kv_heads, ctx_len, self.cfg.head_dim)
        full = torch.zeros(self.B, self.cfg.kv_heads, self.T, self.cfg.head_dim, dtype=torch.bfloat16,
                           device=self.device)
        for kc, vc in zip(self.k_cache, self.v_cache):
            # drawn in the logical [B, Hkv, ctx, D] order whatever the cache
            # layout, so native and reference decoders see the same context
            for c, to_layout in ((kc, ops.k_to_cache_layout), (vc, ops.v_to_cache_layout)):
                x = torch.randn(shape, generator=g, device=self.device, dtype=torch.float32).to(c.dtype)
                if self.kv_native_layout:
                    full[:, :, :ctx_len] = x
                    c.copy_(to_layout(full))
                else:
                    c[:, :, :ctx_len] = x
        self.pos.fill_(ctx_len)
        self.seqlens.fill_(ctx_len + 1)
        self.tokens.copy_(torch.randint(0, self.cfg.vocab, (self.B,), generator=g, device=self.device))

    # -------------------------------------------------------------- step --
    def _attention(self, li, lw, qkv, defer_combine: bool = False):
        cfg = self.cfg
        if self.attn_fused:
            ops.decode_attention_fused(qkv, lw["q_norm"], lw["k_norm"], self.pos, self.seqlens,
                                       self.k_cache[li], self.v_cache[li], self.attn, self.o_part,
                                       self.ml_part, self.attn_counters, cfg.heads, cfg.kv_heads,
                                       cfg.head_dim, self.nsplit, self.scale, cfg.eps, cfg.rope_theta,
                                       defer_combine=defer_combine)
        else:
            ops.qk_norm_rope_kv(qkv, lw["q_norm"], lw["k_norm"], self.pos, self.q,
                                self.k_cache[li], self.v_cache[li], cfg.heads, cfg.kv_heads,
                                cfg.head_dim, cfg.eps, cfg.rope_theta)
            ops.decode_attention(self.q, self.k_cache[li], self.v_cache[li], self.seqlens,
                                 self.attn, self.o_part, self.ml_part, cfg.heads, cfg.kv_heads,
                                 cfg.head_dim, self.nsplit, self.scale)

    def _step_norm_fused(self):
        """Decode step with the row-norm fusion: six launches per layer
        (qkv, attention, combine, o_proj+residual, gate_up+SiLU, down+residual)."""
        cfg, w = self.cfg, self.w
        h, eps = cfg.hidden, cfg.eps
        # gather + the first norm's sums of squares (one slot) in one launch;
        # later slots come from the epilogues
        ops.embed_rmsnorm(w.embed, self.tokens, None, cfg.eps, res=self.res, out=None, ss_out=self.ss_a)
        na = 1
        for li, lw in enumerate(w.layers):
            qkv = lw["pqkv"].norm_call(self.res, out=self.qkv_buf, row_scale=(self.ss_a, na, h, eps))
            if self.xcomb:
                # small batch: o_proj combines the attention splits in its X
                # staging (no combine launch)
                self._attention(li, lw, qkv, defer_combine=True)
                lw["po"].norm_call_xcomb(self.xcomb, self.B, out=self.res, residual=True, ss_out=self.ss_b)
            else:
                self._attention(li, lw, qkv)
                lw["po"].norm_call(self.attn, out=self.res, residual=True, ss_out=self.ss_b)
            lw["pgu"].norm_call(self.res, out=self.act, row_scale=(self.ss_b, self.slots_o, h, eps), **self._gu_plan)
            lw["pd"].norm_call(self.act, out=self.res, residual=True, ss_out=self.ss_a, **self._d_plan)
            na = self.slots_d
        ops.rmsnorm(self.res, w.final_norm, eps, out=self.h)
        logits = self.p_lm(self.h, out=self.logits)
        self._tail(logits)
        return logits

    def _build_chains(self) -> list:
        """One ops.DecodeChain per layer: [o_proj, gate_up, down] of layer li
        and the qkv of layer li + 1 (the last layer's chain ends at down)."""
        cfg, h, eps = self.cfg, self.cfg.hidden, self.cfg.eps
        ctr = ops.chain_counters(self.device)
        chains = []
        for li, lw in enumerate(self.w.layers):
            nxt = self.w.layers[li + 1] if li + 1 < cfg.layers else None
            if self.chain_mode == "gd":
                chains.append(ops.DecodeChain(
                    gu=dict(pl=lw["pgu"], x=self.res, y=self.act, rs=(self.ss_b, self.slots_o, h, eps)),
                    d=dict(pl=lw["pd"], x=self.act, y=self.res, ss=self.ss_a),
                    W=self.chain_w, down_splits=self.chain_down_s, ctr=ctr))
                continue
            chains.append(ops.DecodeChain(
                o=dict(pl=lw["po"], x=self.attn, y=self.res, ss=self.ss_b),
                gu=dict(pl=lw["pgu"], x=self.res, y=self.act, rs=(self.ss_b, self.chain_slots_o, h, eps)),
                d=dict(pl=lw["pd"], x=self.act, y=self.res, ss=self.ss_a),
                qkv=(dict(pl=nxt["pqkv"], x=self.res, y=self.qkv_buf, rs=(self.ss_a, self.chain_slots_d, h, eps))
                     if nxt is not None else None),
                W=self.chain_w, down_splits=self.chain_down_s, ctr=ctr))
        return chains

    def _step_chained(self):
        """Norm-fused decode step with chained projections: per layer the
        attention launch and one chain launch (o_proj, gate_up, down, next qkv)."""
        cfg, w = self.cfg, self.w
        h, eps = cfg.hidden, cfg.eps
        ops.embed_rmsnorm(w.embed, self.tokens, None, cfg.eps, res=self.res, out=None, ss_out=self.ss_a)
        if self.chain_mode == "gd":
            na = 1
            for li, lw in enumerate(w.layers):
                lw["pqkv"].norm_call(self.res, out=self.qkv_buf, row_scale=(self.ss_a, na, h, eps))
                self._attention(li, lw, self.qkv_buf)
                lw["po"].norm_call(self.attn, out=self.res, residual=True, ss_out=self.ss_b)
                self._chains[li]()
                na = self.chain_slots_d
            ops.rmsnorm(self.res, w.final_norm, eps, out=self.h)
            logits = self.p_lm(self.h, out=self.logits)
            self._tail(logits)
            return logits
        w.layers[0]["pqkv"].norm_call(self.res, out=self.qkv_buf, row_scale=(self.ss_a, 1, h, eps))
        for li, lw in enumerate(w.layers):
            self._attention(li, lw, self.qkv_buf)
            self._chains[li]()
        ops.rmsnorm(self.res, w.final_norm, eps, out=self.h)
        logits = self.p_lm(self.h, out=self.logits)
        self._tail(logits)
        return logits

    def _step_impl(self):
        if self.chain:
            return self._step_chained()
        if self.norm_fused:
            return self._step_norm_fused()
        cfg, w = self.cfg, self.w
        # every graph node a kernel: the step's state moves through kernels that
        # write their outputs in place (index_select / argmax with out=), never
        # through a device-to-device copy node -- replayed after a prefill, a
        # captured copy of the argmax result raced the argmax kernel on this
        # stack and fed the next step a garbage token (AMD_SERIALIZE_KERNEL=3
        # hid it; scripts/probe/prefill_graph_bisect.py)
        L = cfg.layers
        if self.native:
            # gather + first RMSNorm in one launch (csrc/ops/model_ops.hip embed_rmsnorm_kernel)
            ops.embed_rmsnorm(w.embed, self.tokens, w.layers[0]["ln1"], cfg.eps, res=self.res, out=self.h)
        else:
            torch.index_select(w.embed, 0, self.tokens, out=self.res)
            self.h.copy_(ref.rmsnorm(self.res, w.layers[0]["ln1"], cfg.eps))
        for li, lw in enumerate(w.layers):
            qkv = lw["pqkv"](self.h, out=self.qkv_buf) if self.skinny_qkv else F.linear(self.h, lw["wqkv"])
            if self.native:
                self._attention(li, lw, qkv)
            else:
                ref.qk_norm_rope_kv(qkv, lw["q_norm"], lw["k_norm"], self.pos, self.q,
                                    self.k_cache[li], self.v_cache[li], cfg.heads, cfg.kv_heads,
                                    cfg.head_dim, cfg.eps, cfg.rope_theta)
                self.attn.copy_(ref.decode_attention(self.q, self.k_cache[li], self.v_cache[li],
                                                     self.seqlens, cfg.heads, cfg.kv_heads,
                                                     cfg.head_dim, self.scale).view(self.B, -1))
            o = lw["po"](self.attn, out=self.o_out) if self.skinny_o else F.linear(self.attn, lw["wo"])
            if self.native:
                ops.add_rmsnorm(o, self.res, lw["ln2"], cfg.eps, out=self.h)
            else:
                self.h.copy_(ref.add_rmsnorm(o, self.res, lw["ln2"], cfg.eps))
            if self.skinny:
                if self.skinny_gate_up:
                    lw["pgu"](self.h, out=self.act)      # gate_up GEMM + SiLU*up epilogue
                else:
                    ops.silu_mul(F.linear(self.h, lw["wgu"]), out=self.act)
                d = lw["pd"](self.act, out=self.mlp_out)
            else:
                gu = F.linear(self.h, lw["wgu"])
                if self.native:
                    ops.silu_mul(gu, out=self.act)
                else:
                    self.act.copy_(ref.silu_mul(gu))
                d = F.linear(self.act, lw["wd"])
            nxt = w.layers[li + 1]["ln1"] if li + 1 < L else w.final_norm
            if self.native:
                ops.add_rmsnorm(d, self.res, nxt, cfg.eps, out=self.h)
            else:
                self.h.copy_(ref.add_rmsnorm(d, self.res, nxt, cfg.eps))
        logits = self.p_lm(self.h, out=self.logits) if self.skinny else F.linear(self.h, w.lm_head)
        self._tail(logits)
        return logits

    def _tail(self, logits):
        if self.native and logits.dtype == torch.bfloat16:
            # argmax + pos / seqlens advance in one launch (decode_tail_kernel)
            if self._tail_work is None:
                self._tail_work = ops.decode_tail_workspace(self.B, self.device)
            ops.decode_tail(logits, self.tokens, self.pos, self.seqlens, self._tail_work)
            return
        torch.argmax(logits, dim=-1, out=self.tokens)
        self.pos.add_(1)
        self.seqlens.add_(1)

    # ---------------------------------------------------------- prefill --
    # Prompt processing for serving (serve/engine.py): all prompt positions of
    # one batch row in one pass, padded to a bucket length so each bucket runs
    # as one captured hipGraph (HIP graphs instead of thousands of eager
    # launches: the prompt of a chat request is latency-bound, not
    # FLOP-bound).  Per layer: RMSNorm (HIP), qkv (hipBLASLt or the packed
    # skinny kernel in <= 128-row chunks), QK-norm + RoPE + KV append to the
    # cache row + head-grouped q (one HIP kernel), causal GQA flash attention
    # (csrc/ops/prefill_attn.hip: online softmax over 32-key tiles, no L x L
    # scores), o_proj, add+RMSNorm, gate_up+SiLU, down, add+RMSNorm.  Pad
    # positions >= L write K/V the decode steps overwrite before reading (and
    # causality keeps them out of every real position's attention).  Buckets
    # reach the reference benchmark's --max-model-len 8192
    # (benchmarks/ai-benchmark/Dockerfile:7-9).
    PREFILL_CHUNK = 128
    PREFILL_BUCKETS = (32, 64, 128, 256, 512, 1024, 2048, 4096, 8192)
    # prompts of at least this many rows run packed-only projections as
    # unpack-once + library GEMM (PackedLinear.prompt) instead of 128-row chunks
    PROMPT_UNPACK_ROWS = int(os.environ.get("MIVGPU_PROMPT_UNPACK_ROWS", "1024"))

    def _rows(self, pl, x, out=None):
        M = x.shape[0]
        if out is None:
            out = torch.empty(M, pl.out_features, dtype=torch.bfloat16, device=x.device)
        for s in range(0, M, self.PREFILL_CHUNK):
            e = min(M, s + self.PREFILL_CHUNK)
            pl(x[s:e], out=out[s:e])
        return out

    def _rows_normed(self, pl, x, out=None):
        """RMSNorm(x) . W^T for a packed weight with the norm folded into its
        columns (norm-fused decoder): per <= 128-row chunk, the rows' sums of
        squares in one slot, applied as row scales by the kernel."""
        M = x.shape[0]
        if out is None:
            out = torch.empty(M, pl.out_features, dtype=torch.bfloat16, device=x.device)
        for s in range(0, M, self.PREFILL_CHUNK):
            e = min(M, s + self.PREFILL_CHUNK)
            torch.sum(x[s:e].float().pow(2), dim=-1, out=self.ss_pf[:e - s])
            pl.norm_call(x[s:e], out=out[s:e], row_scale=(self.ss_pf, 1, self.cfg.hidden, self.cfg.eps))
        return out

    def _normed_proj(self, lw, name, x, ln, h=None):
        """Norm-fused decoder, prefill: RMSNorm(x) . W^T (SiLU*up for gate_up)
        on the plain weight after a separate norm where one is kept and the
        rows are prompt-sized, on the packed copy unpacked for the library GEMM
        for long prompts (its folded norm weight: X normalised without one),
        else on the packed copy with the folded norm and row scales.  ``h``:
        the normalised rows _add_then_norm already produced for this call."""
        packed, plain = {"qkv": ("pqkv", "wqkv"), "gu": ("pgu", "wgu")}[name]
        if plain in lw and x.shape[0] > 64:
            y = F.linear(self._norm(x, ln) if h is None else h, lw[plain])
            return ops.silu_mul(y) if name == "gu" else y
        if x.shape[0] >= self.PROMPT_UNPACK_ROWS:
            return lw[packed].prompt(self._norm(x, self._ones) if h is None else h)
        return self._rows_normed(lw[packed], x)     # gate_up: SiLU*up fused in the epilogue

    def _add_then_norm(self, lw, name, y, res, ln):
        """res += y in place and, where the next _normed_proj(name) normalises
        the whole rows first, that norm in the same launch (add_rmsnorm: one
        pass over the residual instead of an add and a norm kernel, 2 x 64 MB
        less traffic per layer at 8192 rows).  Returns those rows or None."""
        packed, plain = {"qkv": ("pqkv", "wqkv"), "gu": ("pgu", "wgu")}[name]
        rows = res.shape[0]
        if self.native and plain in lw and rows > 64:
            return ops.add_rmsnorm(y, res, ln, self.cfg.eps)
        if self.native and rows >= self.PROMPT_UNPACK_ROWS:
            return ops.add_rmsnorm(y, res, self._ones, self.cfg.eps)
        res.add_(y)
        return None

    def _gemm_into_residual(self, lw, name, x, res, nxt, nxt_name):
        """res += x . W^T inside the library GEMM (beta = 1, C = res), then the
        next projection's whole-row RMSNorm as its own pass where
        _add_then_norm would have fused it: at 8192 rows 64 MB less traffic
        per call than writing y and running add_rmsnorm -- 8k prefill 116.21
        vs 116.96 ms, faster in 5 of 5 interleaved pairs
        (profiles/round6/addmm/).  MIVGPU_PREFILL_ADDMM=0 writes y.  Returns
        (handled, normalised rows or None)."""
        plain = {"o": "wo", "d": "wd"}[name]
        if not (self.native and self._pf_addmm and plain in lw and x.shape[0] > 64):
            return False, None
        res.addmm_(x, lw[plain].t())
        if nxt is None:
            return True, None
        ln = nxt["ln1"] if nxt_name == "qkv" else nxt["ln2"]
        if {"qkv": "wqkv", "gu": "wgu"}[nxt_name] in nxt:
            return True, ops.rmsnorm(res, ln, self.cfg.eps)
        if res.shape[0] >= self.PROMPT_UNPACK_ROWS:
            return True, ops.rmsnorm(res, self._ones, self.cfg.eps)
        return True, None

    def _prefill_impl_norm_fused(self, bufs: dict, b: int):
        cfg, w = self.cfg, self.w
        self._pf_addmm = os.environ.get("MIVGPU_PREFILL_ADDMM", "1") == "1"
        res = torch.index_select(w.embed, 0, bufs["ids"])
        h = None
        for li, lw in enumerate(w.layers):
            qkv = self._normed_proj(lw, "qkv", res, lw["ln1"], h)
            q, k, v = self._prefill_qk(li, lw, qkv, bufs["pos"], b)
            att = self._prefill_attention(q, k, v, bufs["mask"])
            done, h = self._gemm_into_residual(lw, "o", att, res, lw, "gu")
            if not done:
                o = self._proj(lw, "o", att)
                h = self._add_then_norm(lw, "gu", o, res, lw["ln2"])
            act = self._normed_proj(lw, "gu", res, lw["ln2"], h)
            nxt = w.layers[li + 1] if li + 1 < len(w.layers) else None
            done, h = self._gemm_into_residual(lw, "d", act, res, nxt, "qkv")
            if done:
                continue
            d = self._proj(lw, "d", act)
            if nxt is not None:
                h = self._add_then_norm(nxt, "qkv", d, res, nxt["ln1"])
            else:
                res.add_(d)
        last = torch.index_select(res, 0, bufs["last"])
        logits = self._rows(self.p_lm, self._norm(last, w.final_norm))
        torch.argmax(logits, dim=-1, out=self.tokens[b:b + 1])
        torch.add(bufs["plen"], 0, out=self.pos[b:b + 1])
        torch.add(bufs["plen"], 1, out=self.seqlens[b:b + 1])
        return logits

    def _proj(self, lw, name, x):
        packed, plain = {"qkv": ("pqkv", "wqkv"), "o": ("po", "wo"), "gu": ("pgu", "wgu"),
                         "d": ("pd", "wd")}[name]
        if packed in lw and not (plain in lw and x.shape[0] > 64):
            if x.shape[0] >= self.PROMPT_UNPACK_ROWS:
                return lw[packed].prompt(x)      # long prompt: unpack once, library GEMM
            return self._rows(lw[packed], x)     # gate_up: SiLU*up fused in the epilogue
        y = F.linear(x, lw[plain])
        if name == "gu":
            return ops.silu_mul(y) if self.native else ref.silu_mul(y)
        return y

    def _norm(self, x, w):
        return ops.rmsnorm(x, w, self.cfg.eps) if self.native else ref.rmsnorm(x, w, self.cfg.eps)

    def _add_norm(self, x, res, w):
        if self.native:
            return ops.add_rmsnorm(x, res, w, self.cfg.eps)
        return ref.add_rmsnorm(x, res, w, self.cfg.eps)

    def _prefill_qk(self, li, lw, qkv, pos, b):
        """-> q [Hkv, G*L, D], k / v [Hkv, L, D] (bf16); K/V appended to cache row b."""
        cfg = self.cfg
        L, Hq, Hkv, D = qkv.shape[0], cfg.heads, cfg.kv_heads, cfg.head_dim
        G = Hq // Hkv
        if self.native:
            q = torch.empty(Hkv, G * L, D, dtype=torch.bfloat16, device=qkv.device)
            k = torch.empty(Hkv, L, D, dtype=torch.bfloat16, device=qkv.device)
            v = torch.empty_like(k)
            ops.prefill_qk_norm_rope_kv(qkv, lw["q_norm"], lw["k_norm"], pos, q, k, v, self.k_cache[li],
                                        self.v_cache[li], b, Hq, Hkv, D, cfg.eps, cfg.rope_theta)
            return q, k, v
        x = qkv.float().view(L, Hq + 2 * Hkv, D)

        def head_norm(t, wn):
            return t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + cfg.eps) * wn.float()

        qf = ref.rope_neox(head_norm(x[:, :Hq], lw["q_norm"]), pos, cfg.rope_theta)
        kf = ref.rope_neox(head_norm(x[:, Hq:Hq + Hkv], lw["k_norm"]), pos, cfg.rope_theta)
        k = kf.transpose(0, 1).to(torch.bfloat16)                         # [Hkv, L, D]
        v = x[:, Hq + Hkv:].transpose(0, 1).to(torch.bfloat16)
        n = min(L, self.T)
        self.k_cache[li][b, :, :n] = k[:, :n]
        self.v_cache[li][b, :, :n] = v[:, :n]
        q = qf.view(L, Hkv, G, D).permute(1, 2, 0, 3).reshape(Hkv, G * L, D).to(torch.bfloat16)
        return q, k, v

    def _prefill_attention(self, q, k, v, mask):
        """Causal GQA attention: q [Hkv, G*L, D], k/v [Hkv, L, D] -> [L, Hq*D] bf16."""
        if self.native:
            return ops.prefill_attention(q, k, v, self.cfg.heads, self.scale)
        Hkv, GL, D = q.shape
        L = k.shape[1]
        sc = torch.baddbmm(mask.expand(Hkv, GL, L), q.float(), k.float().transpose(1, 2), alpha=self.scale)
        o = torch.bmm(torch.softmax(sc, dim=-1), v.float())                # [Hkv, G*L, D]
        return o.view(Hkv, GL // L, L, D).permute(2, 0, 1, 3).reshape(L, Hkv * (GL // L) * D).to(torch.bfloat16)

    def _prefill_bufs(self, Lb: int) -> dict:
        bufs = self._pf.get(Lb)
        if bufs is None:
            G = self.cfg.heads // self.cfg.kv_heads
            i = torch.arange(Lb, device=self.device)
            mask = None
            if not self.native:     # the fp32 path's additive mask (the HIP kernel masks itself)
                causal = torch.zeros(Lb, Lb, device=self.device).masked_fill_(i[None, :] > i[:, None],
                                                                              float("-inf"))
                mask = causal.repeat(G, 1)
            bufs = dict(ids=torch.zeros(Lb, dtype=torch.long, device=self.device),
                        pos=i.to(torch.int32), mask=mask,
                        last=torch.zeros(1, dtype=torch.long, device=self.device),
                        plen=torch.zeros(1, dtype=torch.int32, device=self.device), graph=None)
            self._pf[Lb] = bufs
        return bufs

    def _prefill_impl(self, bufs: dict, b: int):
        if self.norm_fused:
            return self._prefill_impl_norm_fused(bufs, b)
        cfg, w = self.cfg, self.w
        res = torch.index_select(w.embed, 0, bufs["ids"])
        h = self._norm(res, w.layers[0]["ln1"])
        for li, lw in enumerate(w.layers):
            q, k, v = self._prefill_qk(li, lw, self._proj(lw, "qkv", h), bufs["pos"], b)
            o = self._proj(lw, "o", self._prefill_attention(q, k, v, bufs["mask"]))
            h = self._add_norm(o, res, lw["ln2"])
            d = self._proj(lw, "d", self._proj(lw, "gu", h))
            nxt = w.layers[li + 1]["ln1"] if li + 1 < len(w.layers) else w.final_norm
            h = self._add_norm(d, res, nxt)
        last = torch.index_select(h, 0, bufs["last"])
        logits = self._rows(self.p_lm, last) if self.skinny else F.linear(last, w.lm_head)
        # in-place kernels only (no copy nodes in a captured graph)
        torch.argmax(logits, dim=-1, out=self.tokens[b:b + 1])
        torch.add(bufs["plen"], 0, out=self.pos[b:b + 1])
        torch.add(bufs["plen"], 1, out=self.seqlens[b:b + 1])
        return logits

    def _bucket(self, L: int) -> int | None:
        for Lb in self.PREFILL_BUCKETS:
            if L <= Lb <= self.T:
                return Lb
        return None

    @torch.no_grad()
    def capture_prefill(self, buckets=None, b: int = 0):
        """Capture the prefill of row ``b`` for each bucket length (<= T)."""
        assert self.device.type == "cuda"
        for Lb in (buckets or self.PREFILL_BUCKETS):
            if Lb > self.T:
                continue
            bufs = self._prefill_bufs(Lb)
            bufs["plen"].fill_(1)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._prefill_impl(bufs, b)                     # warm: library plans, allocator
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                bufs["logits"] = self._prefill_impl(bufs, b)
            bufs["graph"] = g
        torch.cuda.synchronize()

    @torch.no_grad()
    def prefill(self, prompt, b: int = 0) -> torch.Tensor:
        """Process the prompt token ids into batch row ``b`` (KV for positions
        0..L-1), set that row's next token to the greedy choice and its
        position to L, and return the last position's logits [vocab]."""
        ids = torch.as_tensor(prompt, dtype=torch.long).view(-1)
        L = ids.numel()
        if not 0 < L < self.T:
            raise ValueError(f"prompt of {L} tokens does not fit a context of {self.T}")
        Lb = self._bucket(L) if self.device.type == "cuda" else None
        bufs = self._prefill_bufs(Lb or L)
        bufs["ids"].zero_()
        bufs["ids"][:L].copy_(ids.to(self.device, non_blocking=False))
        bufs["plen"].fill_(L)
        bufs["last"].fill_(L - 1)
        if bufs["graph"] is not None:
            bufs["graph"].replay()
            return bufs["logits"][0]
        return self._prefill_impl(bufs, b)[0]

    def packed_linears(self) -> list:
        out = [pl for lw in self.w.layers for pl in lw.values() if isinstance(pl, ops.PackedLinear)]
        return out + ([self.p_lm] if self.skinny else [])

    def reserve_prefill(self):
        """Size every packed projection's scratch for prefill row chunks, so a
        prompt after capture() never reallocates under the graph."""
        for pl in self.packed_linears():
            pl.reserve(self.PREFILL_CHUNK)

    def capture(self, warmup: int = 2):
        """Capture one decode step into a hipGraph (state advances per replay)."""
        assert self.device.type == "cuda"
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._step_impl()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._step_impl()
        torch.cuda.synchronize()
        for pl in self.packed_linears():
            pl.frozen = True

    def step(self):
        if self.graph is not None:
            self.graph.replay()
            out = None
        else:
            out = self._step_impl()
        if self.chain and any(c.gave_up() for c in self._chains[:1]):
            # a chain that timed out left wrong projections: never return them
            raise RuntimeError("decode chain gave up waiting for its producers (workgroups not co-resident); "
                               "run without MIVGPU_CHAIN")
        return out
