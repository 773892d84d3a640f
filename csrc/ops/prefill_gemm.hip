// Prompt-sized ("prefill") GEMM on gfx950 matrix cores:  Y[M][N] = X[M][K] . W^T
// with W in the decode kernels' fragment-packed layout (skinny_gemm.hip):
//   16-byte chunk ((t*KB + kb)*4 + j)*64 + l  =  W[32t + (l&31)][64kb + 32(l>>5) + 8j .. +8]
// so a slice keeps ONE copy of its weights: the library path it replaces
// (PackedLinear.prompt) unpacked every projection into a row-major scratch
// copy per call (read + write of the whole weight) before hipBLASLt, and ran
// SiLU*up as a separate pass.
//
// Tile: 256 x 256 per workgroup, K in 64-wide k-blocks, 8 waves (2 per SIMD)
// as 4 (M) x 2 (N), each wave 64 rows x 128 columns = 2 x 4 accumulators of
// v_mfma_f32_32x32x16_bf16 (128 VGPRs).  Per k-block the workgroup stages X
// [256][64] (row-major, 16-byte chunks XOR-swizzled by (row >> 1) & 7 so the
// A-fragment ds_read_b128s of a 16-lane group hit distinct banks) and the
// packed W of its 8 n-tiles (already in fragment order: every B-fragment read
// is 64 lanes x 16 contiguous bytes) in LDS, double-buffered (128 KB); the next
// k-block's 64 KB land in registers during this block's 32 MFMAs per wave and
// go to the other buffer after them, one barrier per k-block.  Arithmetic
// intensity 128 FLOP per staged byte: at the bf16 MFMA rate a CU takes in
// ~75 GB/s, served from L2 / the Infinity Cache (X and W of one projection fit
// in its 256 MB).  Workgroups are dealt to XCDs round-robin (b % 8); each
// XCD's share is walked in groups of 4 M-panels across all N so its L2 holds
// the panels it re-reads.
//
// Epilogues: store bf16, or SiLU(gate) * up for the interleaved gate/up
// weight (n-tile 2c = gate rows, 2c+1 = up rows of channel block c: a wave's
// 4 n-tiles are 2 whole pairs) -> Y[M][N/2].
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace {

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

constexpr int PG_BM = 256, PG_BN = 256, PG_NT = PG_BN / 32;   // 8 n-tiles of 32 columns
constexpr int PG_THREADS = 512;
constexpr int PG_A_ELEMS = PG_BM * 64;                       // one X k-block: 32 KB
constexpr int PG_W_CHUNKS = PG_NT * 256;                     // one W k-block: 8 tiles x 4 KB
constexpr int PG_GM = 4;                                     // M-panels per XCD group

__device__ __forceinline__ int a_off(int row, int c) { return row * 64 + ((c ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

template <int EPI>
__global__ void __launch_bounds__(PG_THREADS, 2)
prefill_gemm_kernel(const uint4* __restrict__ wp, const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int M,
                    int K, int N, int ldx, int ldy) {
  __shared__ __attribute__((aligned(16))) bf16_t as[2][PG_A_ELEMS];
  __shared__ __attribute__((aligned(16))) uint4 ws[2][PG_W_CHUNKS];

  // tile of this workgroup: XCD-grouped order (blocks b, b+8, ... share an XCD)
  const int nM = (M + PG_BM - 1) / PG_BM, nN = N / PG_BN;
  const int nb = nM * nN;
  const int b = blockIdx.x;
  const int per_xcd = (nb + 7) / 8;
  int u = (b & 7) * per_xcd + (b >> 3);
  if ((b & 7) * per_xcd + (b >> 3) >= nb || (b >> 3) >= per_xcd) u = b;   // ragged tail: identity
  const int group = u / (PG_GM * nN), within = u % (PG_GM * nN);
  const int gm = min(PG_GM, nM - group * PG_GM);
  const int mb = group * PG_GM + within % gm, nbk = within / gm;
  const int m0 = mb * PG_BM, t0 = nbk * PG_NT;                 // first row, first n-tile

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w & 3, wn = w >> 2;
  const int r = lane & 31, h = lane >> 5;
  const int KB = K >> 6;

  // staging: 4 X chunks + 4 W chunks of 16 B per thread per k-block
  uint4 xa0, xa1, xa2, xa3, wa0, wa1, wa2, wa3;
  const int q0 = tid, q1 = tid + PG_THREADS, q2 = tid + 2 * PG_THREADS, q3 = tid + 3 * PG_THREADS;
  auto xsrc = [&](int q, int kb) {
    const int row = min(m0 + (q >> 3), M - 1);   // rows past M: never stored
    return reinterpret_cast<const uint4*>(x + (size_t)row * ldx + kb * 64 + (q & 7) * 8);
  };
  auto wsrc = [&](int q, int kb) { return wp + ((size_t)(t0 + (q >> 8)) * KB + kb) * 256 + (q & 255); };
  auto load = [&](int kb) {
    xa0 = *xsrc(q0, kb);
    xa1 = *xsrc(q1, kb);
    xa2 = *xsrc(q2, kb);
    xa3 = *xsrc(q3, kb);
    wa0 = *wsrc(q0, kb);
    wa1 = *wsrc(q1, kb);
    wa2 = *wsrc(q2, kb);
    wa3 = *wsrc(q3, kb);
  };
  auto store = [&](int buf) {
    *reinterpret_cast<uint4*>(&as[buf][a_off(q0 >> 3, q0 & 7)]) = xa0;
    *reinterpret_cast<uint4*>(&as[buf][a_off(q1 >> 3, q1 & 7)]) = xa1;
    *reinterpret_cast<uint4*>(&as[buf][a_off(q2 >> 3, q2 & 7)]) = xa2;
    *reinterpret_cast<uint4*>(&as[buf][a_off(q3 >> 3, q3 & 7)]) = xa3;
    ws[buf][q0] = wa0;
    ws[buf][q1] = wa1;
    ws[buf][q2] = wa2;
    ws[buf][q3] = wa3;
  };

  f32x16_t acc[2][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mt][i][e] = 0.f;

  load(0);
  store(0);
  __syncthreads();
  for (int kb = 0; kb < KB; ++kb) {
    const int buf = kb & 1;
    if (kb + 1 < KB) load(kb + 1);
    const bf16_t* a_l = as[buf];
    const uint4* w_l = ws[buf];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x8_t af[2], bfr[4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
        af[mt] = *reinterpret_cast<const bf16x8_t*>(&a_l[a_off(wm * 64 + mt * 32 + r, j + 4 * h)]);
#pragma unroll
      for (int i = 0; i < 4; ++i) bfr[i] = __builtin_bit_cast(bf16x8_t, w_l[(wn * 4 + i) * 256 + j * 64 + lane]);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[mt][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mt], bfr[i], acc[mt][i], 0, 0, 0);
    }
    if (kb + 1 < KB) store(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds column r of each 32x32 tile, rows (e&3) + 8(e>>2) + 4h
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int rbase = m0 + wm * 64 + mt * 32 + 4 * h;
    if constexpr (EPI == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = (t0 + wn * 4 + i) * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = rbase + (e & 3) + 8 * (e >> 2);
          if (row < M) y[(size_t)row * ldy + col] = f2bf(acc[mt][i][e]);
        }
      }
    } else {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int c = (t0 + wn * 4) / 2 + p;          // channel block of the gate/up pair
        const int col = c * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = rbase + (e & 3) + 8 * (e >> 2);
          const float g = acc[mt][2 * p][e], up = acc[mt][2 * p + 1][e];
          if (row < M) y[(size_t)row * ldy + col] = f2bf(g / (1.f + __expf(-g)) * up);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Version 2 (MIVGPU_PREFILL_GEMM=native, the default variant): the same tile,
// waves and epilogues, staged by LDS-DMA in a four-deep ring of 32-wide
// k-slices.  Version 1 staged 64-wide k-blocks through registers with one
// k-block in flight: the next block's loads had ~1 k-block of MFMAs (about
// the L2/MALL latency under load) to land, and the kernel ran at 39 % of the
// MFMA peak (984 TFLOP/s, qkv at 8192 rows).  Here every wave issues four
// 16-byte global_load_lds per slice (two X, two W: 1 KB each, lane-linear in
// LDS), three slices ahead; a slice is retired by the wave's own counted
// s_waitcnt vmcnt (never 0 in the loop) and one raw s_barrier, after which
// the ring slot read one slice earlier is refilled.  All LDS is one array (a
// second __shared__ object makes hipcc wait vmcnt(0) before every ds_read).
//   X slice (kb, half hs): per row the 16-byte chunks {2hs, 2hs+1, 4+2hs,
//     5+2hs} of the 64-wide k-block -- MFMA step jj in {0,1} of the slice
//     reads chunk jj + 2h, the same k-permutation as the packed W -- 64 B per
//     row, chunk cc stored at slot cc ^ ((row >> 2) & 3): a ds_read_b128
//     group of 16 rows covers all 16 slots of a 256-B bank row; the DMA's
//     per-lane SOURCE address realises the swizzle.
//   W slice: for each of the 8 n-tiles the packed chunks j = 2hs, 2hs+1 (2 x
//     1 KB, already in fragment order).
constexpr int PG2_STAGES = 4;
constexpr int PG2_SLICE_U4 = 2048;                    // uint4 per slice: X 1024 + W 1024 (32 KB)

template <int EPI, int ST = PG2_STAGES, bool PRIO = false>
__global__ void __launch_bounds__(PG_THREADS, 2)
prefill_gemm2_kernel(const uint4* __restrict__ wp, const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int M,
                     int K, int N, int ldx, int ldy) {
  static_assert(ST == 4 || ST == 5, "ring of 4 (128 KB) or 5 (160 KB) slices");
  __shared__ __attribute__((aligned(16))) uint4 ring[ST * PG2_SLICE_U4];

  const int nM = (M + PG_BM - 1) / PG_BM, nN = N / PG_BN;
  const int nb = nM * nN;
  const int b = blockIdx.x;
  // XCD-grouped order, bijective for any grid (blocks b, b+8, ... share an XCD)
  const int q = nb / 8, rr = nb % 8, xcd = b & 7;
  const int u = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
  const int group = u / (PG_GM * nN), within = u % (PG_GM * nN);
  const int gm = min(PG_GM, nM - group * PG_GM);
  const int mb = group * PG_GM + within % gm, nbk = within / gm;
  const int m0 = mb * PG_BM, t0 = nbk * PG_NT;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w & 3, wn = w >> 2;
  const int r = lane & 31, h = lane >> 5;
  const int KB = K >> 6;
  const int S = 2 * KB;                                 // 32-wide k-slices

  // this lane's DMA sources: X rows 32w + 16i + lane/4 (i = 0, 1), slot lane%4
  const int xs_row0 = 32 * w + (lane >> 2);
  const int xcc = (lane & 3) ^ ((lane >> 4) & 3);      // in-slice chunk of the slot (row>>2 & 3 = lane>>4 & 3)
  const int xg = (xcc & 1) + 4 * (xcc >> 1);           // + 2hs: chunk of the 64-wide k-block
  const bf16_t* xsrc0 = x + (size_t)min(m0 + xs_row0, M - 1) * ldx + xg * 8;
  const bf16_t* xsrc1 = x + (size_t)min(m0 + xs_row0 + 16, M - 1) * ldx + xg * 8;
  // W: this wave's n-tile w, both halves of the slice
  const uint4* wsrc = wp + ((size_t)(t0 + w) * KB) * 256 + lane;

  auto issue = [&](int sl) {
    const int kb = sl >> 1, hs = sl & 1;
    uint4* dst = ring + (sl % ST) * PG2_SLICE_U4;
    // X: rows 32w .. 32w + 31 (two 16-row DMAs), W: tile w, j = 2hs, 2hs + 1
    __builtin_amdgcn_global_load_lds(xsrc0 + kb * 64 + hs * 16, dst + (32 * w) * 4, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(xsrc1 + kb * 64 + hs * 16, dst + (32 * w + 16) * 4, 16, 0, 0);
    const uint4* ws = wsrc + (kb * 4 + 2 * hs) * 64;
    __builtin_amdgcn_global_load_lds(ws, dst + 1024 + (2 * w) * 64, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(ws + 64, dst + 1024 + (2 * w + 1) * 64, 16, 0, 0);
  };

  f32x16_t acc[2][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mt][i][e] = 0.f;

  // A-fragment LDS slots of this lane (uint4 index within a slice): row
  // wm*64 + mt*32 + r, in-slice chunk jj + 2h, swizzled by (row >> 2) & 3
  int aidx[2][2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int row = wm * 64 + mt * 32 + r;
      aidx[mt][jj] = row * 4 + ((jj + 2 * h) ^ ((row >> 2) & 3));
    }

  for (int p = 0; p < ST - 1; ++p)
    if (p < S) issue(p);
  for (int sl = 0; sl < S; ++sl) {
    // retire slice sl: this wave's loads of the (up to) ST - 2 later slices stay in flight
    const int ahead = min(ST - 2, S - 1 - sl);
    if (ahead >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // every wave is past its reads of slice sl - 1: refill that slot
    if (sl + ST - 1 < S) issue(sl + ST - 1);
    const uint4* cur = ring + (sl % ST) * PG2_SLICE_U4;
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      bf16x8_t af[2], bfr[4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) af[mt] = __builtin_bit_cast(bf16x8_t, cur[aidx[mt][jj]]);
#pragma unroll
      for (int i = 0; i < 4; ++i) bfr[i] = __builtin_bit_cast(bf16x8_t, cur[1024 + ((wn * 4 + i) * 2 + jj) * 64 + lane]);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[mt][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mt], bfr[i], acc[mt][i], 0, 0, 0);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  }

#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int rbase = m0 + wm * 64 + mt * 32 + 4 * h;
    if constexpr (EPI == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = (t0 + wn * 4 + i) * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = rbase + (e & 3) + 8 * (e >> 2);
          if (row < M) y[(size_t)row * ldy + col] = f2bf(acc[mt][i][e]);
        }
      }
    } else {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int c = (t0 + wn * 4) / 2 + p;
        const int col = c * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = rbase + (e & 3) + 8 * (e >> 2);
          const float g = acc[mt][2 * p][e], up = acc[mt][2 * p + 1][e];
          if (row < M) y[(size_t)row * ldy + col] = f2bf(g / (1.f + __expf(-g)) * up);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Version 3: v2's ring with the two wave groups in ping-pong.  v2 ran 16
// MFMAs per wave between barriers and every wave issued its fragment reads
// right after the barrier: both waves of a SIMD waited on LDS at once (the
// ring depth and wave priority did not move it, profiles §40).  Here group 0
// (waves 0-3, n-columns 0-127) and group 1 (waves 4-7, 128-255) -- one wave of
// each per SIMD -- alternate: two barriers per slice, and between them one
// group's wave runs its 16 MFMAs (raised priority) while the other's reads
// the fragments it multiplies next.
//   phase A_s: group 0 MFMAs on slice s (fragments read in B_{s-1}),
//              group 1 reads slice s;
//   phase B_s: group 1 MFMAs on slice s, group 0 reads slice s + 1.
// Every wave retires its own DMA of slice s + 1 (counted vmcnt) before B_s,
// so slice s + 1 is complete for both readers after that barrier; the slot
// of slice s - 1 is refilled after A_s, when both groups are past it.
template <int EPI>
__global__ void __launch_bounds__(PG_THREADS, 2)
prefill_gemm3_kernel(const uint4* __restrict__ wp, const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int M,
                     int K, int N, int ldx, int ldy) {
  constexpr int ST = PG2_STAGES;
  __shared__ __attribute__((aligned(16))) uint4 ring[ST * PG2_SLICE_U4];

  const int nM = (M + PG_BM - 1) / PG_BM, nN = N / PG_BN;
  const int nb = nM * nN;
  const int b = blockIdx.x;
  const int q = nb / 8, rr = nb % 8, xcd = b & 7;
  const int u = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
  const int group = u / (PG_GM * nN), within = u % (PG_GM * nN);
  const int gm = min(PG_GM, nM - group * PG_GM);
  const int mb = group * PG_GM + within % gm, nbk = within / gm;
  const int m0 = mb * PG_BM, t0 = nbk * PG_NT;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w & 3, wn = w >> 2;   // wn: the ping-pong group
  const int r = lane & 31, h = lane >> 5;
  const int KB = K >> 6;
  const int S = 2 * KB;

  const int xs_row0 = 32 * w + (lane >> 2);
  const int xcc = (lane & 3) ^ ((lane >> 4) & 3);
  const int xg = (xcc & 1) + 4 * (xcc >> 1);
  const bf16_t* xsrc0 = x + (size_t)min(m0 + xs_row0, M - 1) * ldx + xg * 8;
  const bf16_t* xsrc1 = x + (size_t)min(m0 + xs_row0 + 16, M - 1) * ldx + xg * 8;
  const uint4* wsrc = wp + ((size_t)(t0 + w) * KB) * 256 + lane;

  auto issue = [&](int sl) {
    const int kb = sl >> 1, hs = sl & 1;
    uint4* dst = ring + (sl % ST) * PG2_SLICE_U4;
    __builtin_amdgcn_global_load_lds(xsrc0 + kb * 64 + hs * 16, dst + (32 * w) * 4, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(xsrc1 + kb * 64 + hs * 16, dst + (32 * w + 16) * 4, 16, 0, 0);
    const uint4* ws = wsrc + (kb * 4 + 2 * hs) * 64;
    __builtin_amdgcn_global_load_lds(ws, dst + 1024 + (2 * w) * 64, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(ws + 64, dst + 1024 + (2 * w + 1) * 64, 16, 0, 0);
  };
  // retire this wave's DMA of slice `sl` (slices up to sl + ST - 2 issued)
  auto retire = [&](int sl) {
    const int later = min(ST - 2, S - 1 - sl);   // slices issued after sl
    if (later >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  f32x16_t acc[2][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mt][i][e] = 0.f;
  int aidx[2][2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int row = wm * 64 + mt * 32 + r;
      aidx[mt][jj] = row * 4 + ((jj + 2 * h) ^ ((row >> 2) & 3));
    }
  // fragments of one slice: A (2 row tiles) and B (4 column tiles) for both 16-wide k-steps
  bf16x8_t a00, a01, a10, a11, b00, b01, b02, b03, b10, b11, b12, b13;
#define PG3_READ(SL)                                                                              \
  do {                                                                                            \
    const uint4* cur_ = ring + ((SL) % ST) * PG2_SLICE_U4;                                        \
    const uint4* bw_ = cur_ + 1024 + (wn * 4 * 2) * 64 + lane;                                    \
    a00 = __builtin_bit_cast(bf16x8_t, cur_[aidx[0][0]]);                                         \
    a01 = __builtin_bit_cast(bf16x8_t, cur_[aidx[1][0]]);                                         \
    a10 = __builtin_bit_cast(bf16x8_t, cur_[aidx[0][1]]);                                         \
    a11 = __builtin_bit_cast(bf16x8_t, cur_[aidx[1][1]]);                                         \
    b00 = __builtin_bit_cast(bf16x8_t, bw_[0 * 128]);                                             \
    b01 = __builtin_bit_cast(bf16x8_t, bw_[1 * 128]);                                             \
    b02 = __builtin_bit_cast(bf16x8_t, bw_[2 * 128]);                                             \
    b03 = __builtin_bit_cast(bf16x8_t, bw_[3 * 128]);                                             \
    b10 = __builtin_bit_cast(bf16x8_t, bw_[0 * 128 + 64]);                                        \
    b11 = __builtin_bit_cast(bf16x8_t, bw_[1 * 128 + 64]);                                        \
    b12 = __builtin_bit_cast(bf16x8_t, bw_[2 * 128 + 64]);                                        \
    b13 = __builtin_bit_cast(bf16x8_t, bw_[3 * 128 + 64]);                                        \
  } while (0)
#define PG3_MFMA(A, B, C) C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, C, 0, 0, 0)
#define PG3_MMA()                                                                                 \
  do {                                                                                            \
    __builtin_amdgcn_s_setprio(1);                                                                \
    PG3_MFMA(a00, b00, acc[0][0]); PG3_MFMA(a00, b01, acc[0][1]);                                 \
    PG3_MFMA(a00, b02, acc[0][2]); PG3_MFMA(a00, b03, acc[0][3]);                                 \
    PG3_MFMA(a01, b00, acc[1][0]); PG3_MFMA(a01, b01, acc[1][1]);                                 \
    PG3_MFMA(a01, b02, acc[1][2]); PG3_MFMA(a01, b03, acc[1][3]);                                 \
    PG3_MFMA(a10, b10, acc[0][0]); PG3_MFMA(a10, b11, acc[0][1]);                                 \
    PG3_MFMA(a10, b12, acc[0][2]); PG3_MFMA(a10, b13, acc[0][3]);                                 \
    PG3_MFMA(a11, b10, acc[1][0]); PG3_MFMA(a11, b11, acc[1][1]);                                 \
    PG3_MFMA(a11, b12, acc[1][2]); PG3_MFMA(a11, b13, acc[1][3]);                                 \
    __builtin_amdgcn_s_setprio(0);                                                                \
  } while (0)

  // One loop body for both groups; group 1 runs it one barrier behind group 0
  // (an extra barrier after the prologue; group 0 adds one at the end):
  //   body k:  barrier X_k . issue slice k + ST - 1 + g . MMA(k) . retire
  //            slice k + 1 + g . barrier Y_k . READ(k + 1)
  // Group 0's X_k / Y_k are the workgroup's barriers 2k+1 / 2k+2, group 1's
  // are 2k+2 / 2k+3, so group 1 READs slice k while group 0 MMAs on it, and
  // the other way round.  Slice k is read in [Y_{k-1}, X_k] by group 0 and
  // in [X_k, Y_k] by group 1 (global barriers): every wave retires it before
  // Y_{k-1} (group 1 one barrier earlier, hence k + 1 + g), and its slot is
  // refilled only after Y_k (group 1 issues one slice further, hence + g).
  const int g = wn;
  for (int p = 0; p < ST - 1 + g; ++p)
    if (p < S) issue(p);
  // retire slice 0: (ST - 2 + g) later slices stay in flight
  if (g) {
    if (S >= 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (S == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (S == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    retire(0);
  }
  barrier();                                   // P: slice 0 complete
  if (g) barrier();                            // group 1: one barrier behind
  PG3_READ(0);
  for (int k = 0; k < S; ++k) {
    barrier();                                 // X_k
    if (k + ST - 1 + g < S) issue(k + ST - 1 + g);
    PG3_MMA();
    {
      // retire slice k + 1 + g: the slices issued after it stay in flight
      const int top = min(S - 1, k + ST - 1 + g);   // last slice issued so far
      const int later = top - (k + 1 + g);
      if (later >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (later == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();                                 // Y_k
    if (k + 1 < S) PG3_READ(k + 1);
  }
  if (!g) barrier();                           // group 0 matches group 1's last barrier
#undef PG3_READ
#undef PG3_MFMA
#undef PG3_MMA

#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int rbase = m0 + wm * 64 + mt * 32 + 4 * h;
    if constexpr (EPI == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = (t0 + wn * 4 + i) * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = rbase + (e & 3) + 8 * (e >> 2);
          if (row < M) y[(size_t)row * ldy + col] = f2bf(acc[mt][i][e]);
        }
      }
    } else {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int c = (t0 + wn * 4) / 2 + p;
        const int col = c * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = rbase + (e & 3) + 8 * (e >> 2);
          const float g = acc[mt][2 * p][e], up = acc[mt][2 * p + 1][e];
          if (row < M) y[(size_t)row * ldy + col] = f2bf(g / (1.f + __expf(-g)) * up);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Version 4 (A/B, MIVGPU_PREFILL_GEMM_V=4): the same ring and tile with FOUR
// waves, one per SIMD, each 128 x 128 (4 x 4 accumulators: 256 fp32 registers,
// the 512-register file of a lone wave) -- the shape of hipBLASLt's kernel on
// these GEMMs (profiles §40): per MFMA half the LDS fragment reads of the
// 64 x 128 waves (16 reads feed 32 MFMAs per slice) and one barrier per 32
// MFMAs.  Each wave DMAs 64 X rows and two W tiles per slice (8 x 1 KB).
template <int EPI>
__global__ void __launch_bounds__(256, 1)
prefill_gemm4_kernel(const uint4* __restrict__ wp, const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int M,
                     int K, int N, int ldx, int ldy) {
  constexpr int ST = PG2_STAGES;
  __shared__ __attribute__((aligned(16))) uint4 ring[ST * PG2_SLICE_U4];

  const int nM = (M + PG_BM - 1) / PG_BM, nN = N / PG_BN;
  const int nb = nM * nN;
  const int b = blockIdx.x;
  const int q = nb / 8, rr = nb % 8, xcd = b & 7;
  const int u = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
  const int group = u / (PG_GM * nN), within = u % (PG_GM * nN);
  const int gm = min(PG_GM, nM - group * PG_GM);
  const int mb = group * PG_GM + within % gm, nbk = within / gm;
  const int m0 = mb * PG_BM, t0 = nbk * PG_NT;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w & 1, wn = w >> 1;
  const int r = lane & 31, h = lane >> 5;
  const int KB = K >> 6;
  const int S = 2 * KB;

  // DMA sources: X rows 64w + 16i + lane/4 (i = 0..3), W tiles 2w, 2w + 1
  const int xcc = (lane & 3) ^ ((lane >> 4) & 3);
  const int xg = (xcc & 1) + 4 * (xcc >> 1);
  const bf16_t* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) xsrc[i] = x + (size_t)min(m0 + 64 * w + 16 * i + (lane >> 2), M - 1) * ldx + xg * 8;
  const uint4* wsrc0 = wp + ((size_t)(t0 + 2 * w) * KB) * 256 + lane;
  const uint4* wsrc1 = wp + ((size_t)(t0 + 2 * w + 1) * KB) * 256 + lane;

  auto issue = [&](int sl) {
    const int kb = sl >> 1, hs = sl & 1;
    uint4* dst = ring + (sl % ST) * PG2_SLICE_U4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds(xsrc[i] + kb * 64 + hs * 16, dst + (64 * w + 16 * i) * 4, 16, 0, 0);
    const int wo = (kb * 4 + 2 * hs) * 64;
    __builtin_amdgcn_global_load_lds(wsrc0 + wo, dst + 1024 + (4 * w) * 64, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(wsrc0 + wo + 64, dst + 1024 + (4 * w + 1) * 64, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(wsrc1 + wo, dst + 1024 + (4 * w + 2) * 64, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(wsrc1 + wo + 64, dst + 1024 + (4 * w + 3) * 64, 16, 0, 0);
  };

  f32x16_t acc[4][4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mt][i][e] = 0.f;
  int aidx[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int row = wm * 128 + mt * 32 + r;
      aidx[mt][jj] = row * 4 + ((jj + 2 * h) ^ ((row >> 2) & 3));
    }

  for (int p = 0; p < ST - 1; ++p)
    if (p < S) issue(p);
  for (int sl = 0; sl < S; ++sl) {
    const int later = min(ST - 2, S - 1 - sl);   // 8 DMAs per slice per wave
    if (later >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (sl + ST - 1 < S) issue(sl + ST - 1);
    const uint4* cur = ring + (sl % ST) * PG2_SLICE_U4;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) af[mt] = __builtin_bit_cast(bf16x8_t, cur[aidx[mt][jj]]);
#pragma unroll
      for (int i = 0; i < 4; ++i) bfr[i] = __builtin_bit_cast(bf16x8_t, cur[1024 + ((wn * 4 + i) * 2 + jj) * 64 + lane]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[mt][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mt], bfr[i], acc[mt][i], 0, 0, 0);
    }
  }

#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int rbase = m0 + wm * 128 + mt * 32 + 4 * h;
    if constexpr (EPI == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = (t0 + wn * 4 + i) * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = rbase + (e & 3) + 8 * (e >> 2);
          if (row < M) y[(size_t)row * ldy + col] = f2bf(acc[mt][i][e]);
        }
      }
    } else {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int c = (t0 + wn * 4) / 2 + p;
        const int col = c * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = rbase + (e & 3) + 8 * (e >> 2);
          const float g = acc[mt][2 * p][e], up = acc[mt][2 * p + 1][e];
          if (row < M) y[(size_t)row * ldy + col] = f2bf(g / (1.f + __expf(-g)) * up);
        }
      }
    }
  }
}

// v2 build (A/B): MIVGPU_PREFILL_GEMM_ST = 4 or 5 ring slices,
// MIVGPU_PREFILL_GEMM_PRIO = 1 raises the wave priority over its MFMAs
int prefill_gemm2_cfg() {
  static const int c = [] {
    const char* st = getenv("MIVGPU_PREFILL_GEMM_ST");
    const char* pr = getenv("MIVGPU_PREFILL_GEMM_PRIO");
    return (st && atoi(st) == 5 ? 1 : 0) | (pr && atoi(pr) == 1 ? 2 : 0);
  }();
  return c;
}

template <int EPI>
void launch_gemm2(int blocks, hipStream_t s, const uint4* wp, const bf16_t* x, bf16_t* y, int M, int K, int N, int ldx,
                  int ldy) {
  switch (prefill_gemm2_cfg()) {
    case 1:
      hipLaunchKernelGGL((prefill_gemm2_kernel<EPI, 5, false>), dim3(blocks), dim3(PG_THREADS), 0, s, wp, x, y, M, K, N,
                         ldx, ldy);
      break;
    case 2:
      hipLaunchKernelGGL((prefill_gemm2_kernel<EPI, 4, true>), dim3(blocks), dim3(PG_THREADS), 0, s, wp, x, y, M, K, N,
                         ldx, ldy);
      break;
    case 3:
      hipLaunchKernelGGL((prefill_gemm2_kernel<EPI, 5, true>), dim3(blocks), dim3(PG_THREADS), 0, s, wp, x, y, M, K, N,
                         ldx, ldy);
      break;
    default:
      hipLaunchKernelGGL((prefill_gemm2_kernel<EPI, 4, false>), dim3(blocks), dim3(PG_THREADS), 0, s, wp, x, y, M, K,
                         N, ldx, ldy);
  }
}

int prefill_gemm_version() {
  static const int v = [] {
    const char* e = getenv("MIVGPU_PREFILL_GEMM_V");
    const int n = e ? atoi(e) : 3;
    return n == 1 || n == 2 || n == 4 ? n : 3;
  }();
  return v;
}

}  // namespace

extern "C" {

// Y[M][N] (epi 0) or Y[M][N/2] = SiLU(gate) * up (epi 1, interleaved gate/up
// weight) from X[M][K] (row stride ldx) and the fragment-packed W (tile-major
// layout only).  N a multiple of 256, K of 64; any M >= 1.
int mivgpu_prefill_gemm(const void* wp, const void* x, void* y, int M, int K, int N, int ldx, int ldy, int epi,
                        hipStream_t s) {
  if (M <= 0 || K <= 0 || (K & 63) || N <= 0 || (N % PG_BN) || ldx < K || (ldx & 7) || (epi != 0 && epi != 1))
    return (int)hipErrorInvalidValue;
  if (ldy < (epi ? N / 2 : N)) return (int)hipErrorInvalidValue;
  const int blocks = ((M + PG_BM - 1) / PG_BM) * (N / PG_BN);
  if (prefill_gemm_version() == 4) {
    if (epi == 0)
      hipLaunchKernelGGL(prefill_gemm4_kernel<0>, dim3(blocks), dim3(256), 0, s, (const uint4*)wp, (const bf16_t*)x,
                         (bf16_t*)y, M, K, N, ldx, ldy);
    else
      hipLaunchKernelGGL(prefill_gemm4_kernel<1>, dim3(blocks), dim3(256), 0, s, (const uint4*)wp, (const bf16_t*)x,
                         (bf16_t*)y, M, K, N, ldx, ldy);
    return (int)hipGetLastError();
  }
  if (prefill_gemm_version() == 3) {
    if (epi == 0)
      hipLaunchKernelGGL(prefill_gemm3_kernel<0>, dim3(blocks), dim3(PG_THREADS), 0, s, (const uint4*)wp,
                         (const bf16_t*)x, (bf16_t*)y, M, K, N, ldx, ldy);
    else
      hipLaunchKernelGGL(prefill_gemm3_kernel<1>, dim3(blocks), dim3(PG_THREADS), 0, s, (const uint4*)wp,
                         (const bf16_t*)x, (bf16_t*)y, M, K, N, ldx, ldy);
    return (int)hipGetLastError();
  }
  if (prefill_gemm_version() == 2) {
    if (epi == 0)
      launch_gemm2<0>(blocks, s, (const uint4*)wp, (const bf16_t*)x, (bf16_t*)y, M, K, N, ldx, ldy);
    else
      launch_gemm2<1>(blocks, s, (const uint4*)wp, (const bf16_t*)x, (bf16_t*)y, M, K, N, ldx, ldy);
    return (int)hipGetLastError();
  }
  if (epi == 0)
    hipLaunchKernelGGL(prefill_gemm_kernel<0>, dim3(blocks), dim3(PG_THREADS), 0, s, (const uint4*)wp,
                       (const bf16_t*)x, (bf16_t*)y, M, K, N, ldx, ldy);
  else
    hipLaunchKernelGGL(prefill_gemm_kernel<1>, dim3(blocks), dim3(PG_THREADS), 0, s, (const uint4*)wp,
                       (const bf16_t*)x, (bf16_t*)y, M, K, N, ldx, ldy);
  return (int)hipGetLastError();
}

}  // extern "C"
