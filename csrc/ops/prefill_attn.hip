// Causal GQA flash attention for prompt prefill (gfx950, MFMA 32x32x16 bf16).
//
// The reference's benchmark serves Qwen3-8B with --max-model-len 8192
// (benchmarks/ai-benchmark/Dockerfile:7-9); a prompt of that length through
// two batched fp32 GEMMs materialised 8192 x 8192 scores per head group (8.6 GB
// per layer).  This kernel never materialises them: per 32-row query block it
// walks the 32-key tiles up to the diagonal with an online softmax.
//
//   q   [Hkv][G][L][128]  (head-grouped: row g*L + l of kv head hk = q head hk*G+g)
//   k,v [Hkv][L][128]
//   out [L][Hq*128]       (o_proj's input layout)
//
// grid = (ceil(L/32) query blocks, heaviest first; Hkv), G waves per workgroup:
// wave g takes q head hk*G + g over the block's 32 positions, so the G waves
// share every K/V tile the workgroup stages in LDS.  Per 32-key tile a wave
// runs 16 MFMAs:
//   S^T (32 keys x 32 q) = K . Q^T       8 k-steps over D; the scores of query
//       column r sit on lanes r and r+32 (16 keys each): the row max and the
//       exponentials stay lane-local (one cross-half exchange for the max);
//   O^T (128 x 32 q) += V^T . P^T        4 d-blocks x 2 k-steps; P^T is the
//       score accumulator converted to bf16 in place (its rows are the
//       reduction index: no lane movement, cdna_hip_programming.md section 3),
//       V^T comes from the row-major V tile through ds_read_b64_tr_b16.
// LDS (32 KB, double-buffered; the next tile's loads are in flight during
// the current tile's MFMAs): K rows with the 16-byte chunk XOR (row & 15) --
// conflict-free row reads for 16 distinct rows per 16-lane group; V rows with
// chunk ^ ((row & 3) << 2) -- the 4 rows of a transposed read land in 4
// different 64-byte slots, conflict-free.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace {

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) short i16x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

constexpr int FA_D = 128;
constexpr int FA_BQ = 32;    // query rows per wave
constexpr int FA_BK = 32;    // keys per tile
constexpr int FA_TILE = FA_BK * FA_D;     // elements per K (or V) tile
constexpr int FA_CHUNKS = FA_TILE / 8;    // 16-byte chunks per tile

__device__ __forceinline__ int k_off(int row, int ch) { return row * FA_D + ((ch ^ (row & 15)) << 3); }
__device__ __forceinline__ int v_off(int row, int ch) { return row * FA_D + ((ch ^ ((row & 3) << 2)) << 3); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even (finite inputs)
  return (bf16_t)(u >> 16);
}

// V^T for the P.V MFMAs: TR = the row-major V tile through the hardware
// transposed read (ds_read_b64_tr_b16; the default, OPAQUE: MIVGPU_FA_TR=2);
// !TR = V staged transposed in LDS ([128 dims][32 keys + 8 pad], one 2-byte
// write per element) and read with plain 8-byte reads (MIVGPU_FA_TR=0).
constexpr int FA_VT_PITCH = FA_BK + 8;

template <int G, bool TR, bool OPAQUE = false>
__global__ void __launch_bounds__(G * 64)
prefill_flash_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                     bf16_t* __restrict__ out, int L, int Hq, float scale_log2) {
  constexpr int NT = G * 64;
  constexpr int PER = FA_CHUNKS / NT;      // 16-byte chunks per thread per tile (K and V each)
  static_assert(PER * NT == FA_CHUNKS, "G must divide 8");
  __shared__ __attribute__((aligned(16))) bf16_t ks[2][FA_TILE];
  __shared__ __attribute__((aligned(16))) bf16_t vs[2][TR ? FA_TILE : FA_D * FA_VT_PITCH];

  const int nqb = (L + FA_BQ - 1) / FA_BQ;
  const int qb = nqb - 1 - (int)blockIdx.x;       // heaviest (longest) blocks first
  const int hk = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int l0 = qb * FA_BQ;
  const int ntiles = qb + 1;                      // keys 0 .. l0+31 (the last tile is the diagonal)

  const bf16_t* kb = k + (size_t)hk * L * FA_D;
  const bf16_t* vb = v + (size_t)hk * L * FA_D;

  // Q^T fragments (B operand of S^T = K.Q^T): lane holds Q[l0+r][16s + 8h .. +8]
  bf16x8_t qf[8];
  {
    const int qrow = min(l0 + r, L - 1);
    const bf16_t* qp = q + (((size_t)hk * G + w) * L + qrow) * FA_D + 8 * h;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8_t*>(qp + 16 * s);
  }

  // tile staging: chunk c = t + i*NT -> row c >> 4, 16-byte chunk c & 15
  // (16 consecutive threads read one 256-byte key row: coalesced)
  uint4 kreg[PER], vreg[PER];
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = t + i * NT;
      const int row = min(kt * FA_BK + (c >> 4), L - 1);   // rows past L: masked (causal)
      kreg[i] = *reinterpret_cast<const uint4*>(kb + (size_t)row * FA_D + (c & 15) * 8);
      vreg[i] = *reinterpret_cast<const uint4*>(vb + (size_t)row * FA_D + (c & 15) * 8);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = t + i * NT;
      *reinterpret_cast<uint4*>(&ks[buf][k_off(c >> 4, c & 15)]) = kreg[i];
      if constexpr (TR) {
        *reinterpret_cast<uint4*>(&vs[buf][v_off(c >> 4, c & 15)]) = vreg[i];
      } else {   // transposed: vs[d][key]
        const int key = c >> 4, d0 = (c & 15) * 8;
        const bf16_t* e = reinterpret_cast<const bf16_t*>(&vreg[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) vs[buf][(d0 + j) * FA_VT_PITCH + key] = e[j];
      }
    }
  };

  f32x16_t o[4];
#pragma unroll
  for (int dc = 0; dc < 4; ++dc)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dc][i] = 0.f;
  float m = -INFINITY, lsum = 0.f;
  const int qpos = l0 + r;

  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < ntiles) load_tile(kt + 1);     // in flight during this tile's MFMAs

    // ---- S^T = K . Q^T (32 keys x 32 queries)
    f32x16_t s;
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = 0.f;
    const bf16_t* kt_lds = ks[buf];
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&kt_lds[k_off(r, 2 * st + h)]);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[st], s, 0, 0, 0);
    }

    // ---- online softmax (query column r: lanes r and r+32 hold 16 keys each)
    const int key0 = kt * FA_BK + 4 * h;
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = key0 + (i & 3) + 8 * (i >> 2);
      const float x = key <= qpos ? s[i] * scale_log2 : -INFINITY;
      s[i] = x;
      mx = fmaxf(mx, x);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mnew = fmaxf(m, mx);
    const float alpha = exp2f(m - mnew);          // 0 on the first tile (m = -inf)
    m = mnew;
    float psum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = exp2f(s[i] - mnew);
      s[i] = p;
      psum += p;
    }
    lsum = lsum * alpha + psum;
#pragma unroll
    for (int dc = 0; dc < 4; ++dc)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[dc][i] *= alpha;

    // P^T as the B operand: registers 8u .. 8u+7 are the fragment of k-step u
    bf16x8_t pf[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[u][j] = (__bf16)s[8 * u + j];

    // ---- O^T += V^T . P^T; the A operand (V^T[d][key]) through transposed reads:
    // lane 4q'+p' of its 16-lane group gives the address of key row q' of the
    // group's 4-key block, columns 4p' .. 4p'+3 of its 16-column block
    const bf16_t* vt_lds = vs[buf];
    const int gi = lane & 15, qq = gi >> 2, pp = gi & 3;
    const int colblk = 16 * ((lane >> 4) & 1);
#pragma unroll
    for (int dc = 0; dc < 4; ++dc) {
      const int col = 32 * dc + colblk + 4 * pp;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int row_lo = 16 * u + 4 * h + qq, row_hi = row_lo + 8;
        if constexpr (!TR) {
          // lane (r, h): V^T[32dc + r][keys 16u + 4h .. +4 and 16u + 4h + 8 .. +4]
          const bf16_t* vrow = vt_lds + (32 * dc + r) * FA_VT_PITCH + 16 * u + 4 * h;
          const uint2 lo2 = *reinterpret_cast<const uint2*>(vrow);
          const uint2 hi2 = *reinterpret_cast<const uint2*>(vrow + 8);
          const uint4 a4 = make_uint4(lo2.x, lo2.y, hi2.x, hi2.y);
          o[dc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a4), pf[u], o[dc], 0, 0, 0);
          continue;
        }
        int olo = v_off(row_lo, col >> 3) + (col & 7), ohi = v_off(row_hi, col >> 3) + (col & 7);
        if constexpr (OPAQUE) {   // no constant part the compiler could fold into the offset field
          asm volatile("" : "+v"(olo));
          asm volatile("" : "+v"(ohi));
        }
        const i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) i16x4_t*)(&vt_lds[olo]));
        const i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) i16x4_t*)(&vt_lds[ohi]));
        // the operand from whole 32-bit lanes: built element-wise (a[j] =
        // bit_cast<__bf16>(lo[j])) hipcc kept only the first dword of each
        // read, permuted and duplicated -- the "wrong sums" of this variant
        const uint2 l2 = __builtin_bit_cast(uint2, lo), h2 = __builtin_bit_cast(uint2, hi);
        const uint4 a4 = make_uint4(l2.x, l2.y, h2.x, h2.y);
        o[dc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a4), pf[u], o[dc], 0, 0, 0);
      }
    }

    if (kt + 1 < ntiles) store_tile(buf ^ 1);
    __syncthreads();
  }

  // ---- normalise and store: O^T reg i of block dc is d = 32dc + (i&3) + 8(i>>2) + 4h
  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  const float inv = 1.f / ltot;
  if (qpos < L) {
    bf16_t* op = out + (size_t)qpos * Hq * FA_D + (size_t)(hk * G + w) * FA_D;
#pragma unroll
    for (int dc = 0; dc < 4; ++dc)
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const int d = 32 * dc + 8 * i4 + 4 * h;
        uint2 pk;
        pk.x = (uint32_t)f2bf(o[dc][4 * i4 + 0] * inv) | ((uint32_t)f2bf(o[dc][4 * i4 + 1] * inv) << 16);
        pk.y = (uint32_t)f2bf(o[dc][4 * i4 + 2] * inv) | ((uint32_t)f2bf(o[dc][4 * i4 + 3] * inv) << 16);
        *reinterpret_cast<uint2*>(op + d) = pk;
      }
  }
}

// ============================================================================
// Eight-wave variant (the default for G <= 8): 64-key tiles, 32 * RT query
// rows per workgroup (RT = 8 / G row tiles of 32, so every workgroup has 8
// waves: two per SIMD, one wave's softmax beside its partner's MFMAs), every
// wave one (head, row tile).  Measured on the kernel above (32-key tiles, 4
// waves, one per SIMD): 307 TFLOP/s at L = 8192 -- the softmax's vector work
// per 32x32 MFMA gap (scale, mask, max, exp, sum, the O rescale: ~680 cycles
// of issue against the ~384 the 16 MFMAs of a tile hide, MI355X_MICROARCH.md
// 'vector-instruction ISSUE cost') set the pace.  Here:
//   * the scale goes into the exponent's FMA (one v_fma + one v_exp per
//     score), the max is taken on the raw scores;
//   * masks only on the diagonal half-tile; halves wholly above a wave's
//     diagonal skip their MFMAs;
//   * the O / l rescale runs only when some row's max grew by more than 8
//     (log2 units; the stale max keeps every p <= 256, exact in fp32 and
//     bf16 range): after the first tiles it is almost never taken;
//   * 64-key tiles: half the barriers and max exchanges per key;
//   * one barrier per tile: the next tile's K/V land in registers during this
//     tile's MFMAs and are stored into the other LDS buffer after them.
constexpr int F2_BK = 64;
constexpr int F2_TILE = F2_BK * FA_D;     // elements per K (or V) tile: 16 KB
constexpr int F2_CHUNKS = F2_TILE / 8;    // 1024 16-byte chunks
constexpr float F2_RESCALE = 8.f;         // lazy O rescale threshold (log2 units)

template <int G, int RT, bool XCD = false>
__global__ void __launch_bounds__(G * RT * 64, 2)
prefill_flash8_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                      bf16_t* __restrict__ out, int L, int Hq, float scale_log2) {
  constexpr int NW = G * RT, NT = NW * 64;
  constexpr int PER = F2_CHUNKS / NT;      // 16-byte chunks per thread per tile (K and V each)
  static_assert(PER * NT == F2_CHUNKS && NW == 8, "eight waves, the tile split evenly");
  constexpr int ROWS = 32 * RT;
  __shared__ __attribute__((aligned(16))) bf16_t ks[2][F2_TILE];
  __shared__ __attribute__((aligned(16))) bf16_t vs[2][F2_TILE];

  const int nqb = (L + ROWS - 1) / ROWS;
  // XCD-aware order (XCD: a 1-D grid): workgroup b runs on XCD b mod 8, so
  // kv head b mod Hkv keeps every query block of a head on one XCD (Hkv = 8:
  // each XCD's L2 holds one head's K/V, 4 MB at 8192 positions, not slices of
  // all eight); heaviest (longest) blocks first within each head.  Measured:
  // 854-858 vs 676-686 TFLOP/s at 8192 positions, 8k prefill 106.8 vs 115.6
  // ms (profiles/round6/fa_xcd/)
  const int hkv = Hq / G;
  const int qb = XCD ? nqb - 1 - (int)blockIdx.x / hkv : nqb - 1 - (int)blockIdx.x;
  const int hk = XCD ? (int)blockIdx.x % hkv : (int)blockIdx.y;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = w % G, rt = w / G;                // head of the group, row tile
  const int r = lane & 31, h = lane >> 5;
  const int l0 = qb * ROWS + 32 * rt;             // this wave's first query row
  const int blk_end = min(L, (qb + 1) * ROWS);    // the block needs keys < blk_end
  const int ntiles = (blk_end + F2_BK - 1) / F2_BK;

  const bf16_t* kb = k + (size_t)hk * L * FA_D;
  const bf16_t* vb = v + (size_t)hk * L * FA_D;

  bf16x8_t qf[8];
  {
    const int qrow = min(l0 + r, L - 1);
    const bf16_t* qp = q + (((size_t)hk * G + g) * L + qrow) * FA_D + 8 * h;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8_t*>(qp + 16 * s);
  }

  // the next tile in registers: two 16-byte chunks of K and of V per thread
  // (named values, not an array: an array here was kept in scratch and LDS)
  static_assert(PER == 2, "two chunks per thread");
  const int c0 = t, c1 = t + NT;                  // chunk c -> row c >> 4, 16-byte chunk c & 15
  const int ko0 = k_off(c0 >> 4, c0 & 15), ko1 = k_off(c1 >> 4, c1 & 15);
  const int vo0 = v_off(c0 >> 4, c0 & 15), vo1 = v_off(c1 >> 4, c1 & 15);
  uint4 k0r, k1r, v0r, v1r;
  auto load_tile = [&](int kt) {
    const int r0 = min(kt * F2_BK + (c0 >> 4), L - 1);   // rows past L: masked (causal)
    const int r1 = min(kt * F2_BK + (c1 >> 4), L - 1);
    k0r = *reinterpret_cast<const uint4*>(kb + (size_t)r0 * FA_D + (c0 & 15) * 8);
    v0r = *reinterpret_cast<const uint4*>(vb + (size_t)r0 * FA_D + (c0 & 15) * 8);
    k1r = *reinterpret_cast<const uint4*>(kb + (size_t)r1 * FA_D + (c1 & 15) * 8);
    v1r = *reinterpret_cast<const uint4*>(vb + (size_t)r1 * FA_D + (c1 & 15) * 8);
  };
  auto store_tile = [&](int buf) {
    *reinterpret_cast<uint4*>(&ks[buf][ko0]) = k0r;
    *reinterpret_cast<uint4*>(&vs[buf][vo0]) = v0r;
    *reinterpret_cast<uint4*>(&ks[buf][ko1]) = k1r;
    *reinterpret_cast<uint4*>(&vs[buf][vo1]) = v1r;
  };

  f32x16_t o[4];
#pragma unroll
  for (int dc = 0; dc < 4; ++dc)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dc][i] = 0.f;
  float m = -INFINITY, lsum = 0.f;
  // Round 6, measured and left out (profiles/README.md section 41): static
  // priority for waves 4-7 (s_setprio 1 before the loop) 708-713 vs 714-718
  // TFLOP/s at 8192; a software-pipelined loop (P.V of tile kt-1 beside the
  // softmax of tile kt, V triple-buffered) 688 vs 714.

  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < ntiles) load_tile(kt + 1);     // in flight during this tile's MFMAs
    const int kbase = kt * F2_BK;
    if (kbase <= l0 + 31) {                     // some key of the tile is visible to this wave
      // halves of 32 keys: visible (kbase + 32hf <= l0), diagonal when equal
      const bool act1 = kbase + 32 <= l0;
      const bf16_t* kt_lds = ks[buf];
      f32x16_t s0, s1;
#pragma unroll
      for (int i = 0; i < 16; ++i) s0[i] = 0.f, s1[i] = 0.f;
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&kt_lds[k_off(r, 2 * st + h)]);
        s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[st], s0, 0, 0, 0);
      }
      if (act1) {
#pragma unroll
        for (int st = 0; st < 8; ++st) {
          const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&kt_lds[k_off(32 + r, 2 * st + h)]);
          s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[st], s1, 0, 0, 0);
        }
      }
      // causal mask on the diagonal half only: key (i&3) + 8(i>>2) + 4h of the
      // half against query r of the row tile
      if (kbase == l0) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if ((i & 3) + 8 * (i >> 2) + 4 * h > r) s0[i] = -INFINITY;
      } else if (act1 && kbase + 32 == l0) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if ((i & 3) + 8 * (i >> 2) + 4 * h > r) s1[i] = -INFINITY;
      }
      float mx = s0[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) mx = fmaxf(mx, s0[i]);
      if (act1) {
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s1[i]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mt = mx * scale_log2;         // finite: key kbase <= every query of the wave
      if (__ballot(mt > m + F2_RESCALE)) {
        const float mnew = fmaxf(m, mt);
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);   // 0 on the first tile (m = -inf)
        m = mnew;
        lsum *= alpha;
#pragma unroll
        for (int dc = 0; dc < 4; ++dc)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[dc][i] *= alpha;
      }
      float psum = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s0[i], scale_log2, -m));
        s0[i] = p;
        psum += p;
      }
      if (act1) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s1[i], scale_log2, -m));
          s1[i] = p;
          psum += p;
        }
      }
      lsum += psum;

      // O^T += V^T . P^T over the visible 16-key k-steps; V^T by transposed reads
      const bf16_t* vt_lds = vs[buf];
      const int gi = lane & 15, qq = gi >> 2, pp = gi & 3;
      const int colblk = 16 * ((lane >> 4) & 1);
      auto pv = [&](const f32x16_t& sh, int u) {
        bf16x8_t pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (__bf16)sh[8 * (u & 1) + j];
        const int row_lo = 16 * u + 4 * h + qq, row_hi = row_lo + 8;
#pragma unroll
        for (int dc = 0; dc < 4; ++dc) {
          const int col = 32 * dc + colblk + 4 * pp;
          const int olo = v_off(row_lo, col >> 3) + (col & 7), ohi = v_off(row_hi, col >> 3) + (col & 7);
          const i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) i16x4_t*)(&vt_lds[olo]));
          const i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) i16x4_t*)(&vt_lds[ohi]));
          const uint2 l2 = __builtin_bit_cast(uint2, lo), h2 = __builtin_bit_cast(uint2, hi);
          const uint4 a4 = make_uint4(l2.x, l2.y, h2.x, h2.y);
          o[dc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a4), pf, o[dc], 0, 0, 0);
        }
      };
      pv(s0, 0);
      pv(s0, 1);
      if (act1) {
        pv(s1, 2);
        pv(s1, 3);
      }
    }
    if (kt + 1 < ntiles) store_tile(buf ^ 1);
    __syncthreads();
  }

  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  const float inv = 1.f / ltot;
  const int qpos = l0 + r;
  if (qpos < L) {
    bf16_t* op = out + (size_t)qpos * Hq * FA_D + (size_t)(hk * G + g) * FA_D;
#pragma unroll
    for (int dc = 0; dc < 4; ++dc)
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const int d = 32 * dc + 8 * i4 + 4 * h;
        uint2 pk;
        pk.x = (uint32_t)f2bf(o[dc][4 * i4 + 0] * inv) | ((uint32_t)f2bf(o[dc][4 * i4 + 1] * inv) << 16);
        pk.y = (uint32_t)f2bf(o[dc][4 * i4 + 2] * inv) | ((uint32_t)f2bf(o[dc][4 * i4 + 3] * inv) << 16);
        *reinterpret_cast<uint2*>(op + d) = pk;
      }
  }
}

// ds_read_b64_tr_b16 semantics probe: LDS holds element e = e; lane l reads
// at element offset addr[l]; out[4l + i] = element i it received.
// OFF: a constant element offset the compiler folds into the instruction's
// offset field (the probe's addresses otherwise come from memory: none).
template <int OFF>
__global__ void __launch_bounds__(64) tr_read_probe_kernel(const int* __restrict__ addr, int* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[8192];
  for (int i = threadIdx.x; i < 8192; i += 64) lds[i] = (bf16_t)i;
  __syncthreads();
  const i16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) i16x4_t*)(&lds[addr[threadIdx.x] + OFF]));
#pragma unroll
  for (int i = 0; i < 4; ++i) out[4 * threadIdx.x + i] = (int)(uint16_t)v[i];
}

// V^T path, read per launch (prompt-sized launches; tests switch it in one
// process): 1 = transposed reads (default); 0 = V staged transposed, plain
// reads; 2 = transposed reads from opaque addresses (no folded offsets).
int fa_tr() {
  const char* e = getenv("MIVGPU_FA_TR");
  return e && *e ? atoi(e) : 1;
}

// Which kernel: 8 = the eight-wave 64-key-tile kernel (default), 4 = the
// 32-key-tile kernel (A/B; also taken whenever MIVGPU_FA_TR asks for one of
// its V^T variants).
int fa_kernel() {
  const char* e = getenv("MIVGPU_FA_KERNEL");
  if (e && *e) return atoi(e);
  const char* tr = getenv("MIVGPU_FA_TR");
  return tr && *tr && atoi(tr) != 1 ? 4 : 8;
}

}  // namespace

extern "C" {

// offset_elems: 0 or 1024 (folded into the instruction's offset field)
int mivgpu_tr_read_probe(const int* addr, int* out, int offset_elems, hipStream_t s) {
  if (offset_elems == 0)
    hipLaunchKernelGGL(tr_read_probe_kernel<0>, dim3(1), dim3(64), 0, s, addr, out);
  else if (offset_elems == 1024)
    hipLaunchKernelGGL(tr_read_probe_kernel<1024>, dim3(1), dim3(64), 0, s, addr, out);
  else
    return -1;
  return (int)hipGetLastError();
}

// Causal prefill attention of one sequence of L positions (q head-grouped, see
// above).  scale: the softmax scale (1/sqrt(D)).  G = Hq / Hkv in {1, 2, 4, 8}.
int mivgpu_prefill_attention(const void* q, const void* k, const void* v, void* out, int L, int Hq, int Hkv,
                             int head_dim, float scale, hipStream_t s) {
  if (head_dim != FA_D || L <= 0 || Hkv <= 0 || Hq % Hkv) return -1;
  const int G = Hq / Hkv;
  const dim3 grid((L + FA_BQ - 1) / FA_BQ, Hkv);
  const float sl2 = scale * 1.4426950408889634f;
  const bf16_t *qq = (const bf16_t*)q, *kk = (const bf16_t*)k, *vv = (const bf16_t*)v;
  bf16_t* oo = (bf16_t*)out;
#define MIVGPU_FA(GG, TRV, OPQ) \
  hipLaunchKernelGGL((prefill_flash_kernel<GG, TRV, OPQ>), grid, dim3(64 * GG), 0, s, qq, kk, vv, oo, L, Hq, sl2)
#define MIVGPU_FA_G(GG)                                  \
  case GG:                                               \
    if (tr == 1) MIVGPU_FA(GG, true, false);             \
    else if (tr == 2) MIVGPU_FA(GG, true, true);         \
    else MIVGPU_FA(GG, false, false);                    \
    break;
  if (fa_kernel() == 8) {
    const int rows = 32 * (8 / G);
    const dim3 grid8((L + rows - 1) / rows, Hkv);
    // XCD-aware order: a 1-D grid of nqb * Hkv workgroups; MIVGPU_FA_XCD=0
    // keeps the 2-D (query block, kv head) grid
    const char* xe = getenv("MIVGPU_FA_XCD");
    const bool xcd = !(xe && *xe == '0');
    const dim3 grid1(grid8.x * grid8.y, 1);
#define MIVGPU_FA8(GG, RR)                                                                                       \
  do {                                                                                                         \
    if (xcd) hipLaunchKernelGGL((prefill_flash8_kernel<GG, RR, true>), grid1, dim3(512), 0, s, qq, kk, vv, oo, L,  \
                                Hq, sl2);                                                                      \
    else hipLaunchKernelGGL((prefill_flash8_kernel<GG, RR, false>), grid8, dim3(512), 0, s, qq, kk, vv, oo, L, Hq, \
                            sl2);                                                                              \
  } while (0)
    switch (G) {
      case 1: MIVGPU_FA8(1, 8); break;
      case 2: MIVGPU_FA8(2, 4); break;
      case 4: MIVGPU_FA8(4, 2); break;
      case 8: MIVGPU_FA8(8, 1); break;
      default: return -1;
    }
#undef MIVGPU_FA8
    return (int)hipGetLastError();
  }
  const int tr = fa_tr();
  switch (G) {
    MIVGPU_FA_G(1)
    MIVGPU_FA_G(2)
    MIVGPU_FA_G(4)
    MIVGPU_FA_G(8)
    default: return -1;
  }
#undef MIVGPU_FA_G
#undef MIVGPU_FA
  return (int)hipGetLastError();
}

}  // extern "C"
