// Decode-shaped ("skinny") GEMM on gfx950 matrix cores:  Y[M, N] = X[M, K] · W[N, K]^T
//
// Decode projections have M = batch (≤ 128) rows against multi-hundred-MB
// weight matrices: pure HBM streaming of W.  Library GEMMs tile for large M
// and reach 2.3–5 TB/s on these shapes (profiles/decode_b32,
// profiles/gemm); this kernel is built to stream W once at the HBM roofline:
//
//  * W is pre-packed once at load time into MFMA B-fragment order, so every
//    wave-wide load is 1 KiB contiguous (64 lanes x 16 B) and is issued
//    non-temporal (streamed once, must not evict X from L2):
//       16-byte chunk ((t*KB + kb)*4 + j)*64 + l  =  W[32t + (l&31)][64kb + 32(l>>5) + 8j .. +8]
//    for n-tile t (32 rows), k-block kb (64 columns), sub-step j (0..3), lane l.
//  * X stays row-major and L2-resident; lane (r, h) reads 64 contiguous bytes
//    X[r][64kb + 32h .. +32] per k-block and feeds sub-step j with its j-th
//    8-element piece.  The MFMA sums over its 16 k's in any order, so the same
//    (h, j) -> k permutation on both operands gives the exact product.
//  * v_mfma_f32_32x32x16_bf16, fp32 accumulation; each wave owns MT M-tiles x
//    NT n-tiles (W fragments reused MT times, X fragments NT times).
//  * Loads go out in groups of U k-blocks (≈128 VGPRs of fragments per wave in
//    flight) pinned ahead of their MFMAs with a scheduling barrier.
//  * Split-K two ways so that every one of the 256 CUs streams even when the
//    projection has only 128–192 n-tiles:
//      - KS waves of a workgroup split the k-range of the workgroup and
//        reduce with ds_add_f32 into one MT*NT*4 KiB LDS tile;
//      - S workgroups split K further; they add their tile into a zeroed fp32
//        slab with device-scope float atomics and take a ticket: the last
//        arriver applies the epilogue, then re-zeroes slab and ticket (the
//        kernel leaves them clean for the next call / graph replay).
//  * Epilogues: plain bf16 store, or SiLU(gate)*up for an interleaved gate/up
//    weight (n-tile 2c = gate rows, 2c+1 = up rows of channel block c), which
//    removes the separate activation kernel and the [M, 2I] round trip.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;

namespace {

__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (bf16_t)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}
__device__ __forceinline__ float round_bf(float f) { return __uint_as_float((uint32_t)f2bf(f) << 16); }

enum { EPI_STORE = 0, EPI_SILU_MUL = 1, EPI_RESID = 2 };

// Row-norm fusion (wide kernel):
//  * EPI_RESID: Y is the residual stream, updated in place, Y = bf16(Y + X.W^T),
//    and each wave-group writes its columns' share of every row's sum of
//    squares of the new Y to ss_out[vgroup * SS_ROWS + row] (plain stores: no
//    atomics, no zeroing; one slot per wave-group).
//  * row scale: with rs_part != nullptr the accumulator of row m is multiplied
//    by rsqrt(sum_p rs_part[p * SS_ROWS + m] * rs_inv_dim + rs_eps) before the
//    epilogue.  Together with an RMSNorm weight folded into W's columns this
//    is Y = RMSNorm(X) . W^T, with the norm's reduction done by the producer
//    of X and its scale applied here: no separate RMSNorm launch.
constexpr int SS_ROWS = 128;

// k-blocks per load group: ~128 VGPRs of fragments in flight per wave
// (16 VGPRs per M- or N-tile per k-block).
constexpr int unroll_of(int mt, int nt) {
  return 128 / (16 * (mt + nt)) >= 4 ? 4 : (128 / (16 * (mt + nt)) >= 2 ? 2 : 1);
}

// Double-buffered schedule (DB): two groups of U k-blocks, the next one's loads
// issued before the current one's MFMAs, so at least one group is always in
// flight.  Both buffers live in registers: 2*U*(MT+NT)*16 VGPRs <= 256.
constexpr int unroll_db(int mt, int nt) {
  return 256 / (32 * (mt + nt)) >= 4 ? 4 : (256 / (32 * (mt + nt)) >= 2 ? 2 : 1);
}

// Strides (in 16-byte chunks) of the packed W between consecutive n-tiles and
// consecutive k-blocks.  Tile-major: a tile's k-blocks are contiguous.
// K-block-major: a k-block's tiles are contiguous, so the waves of a launch,
// all near the same k-block, read one contiguous front that spreads over every
// HBM channel, instead of as many separate streams as there are waves.
struct WStride {
  size_t tile;
  size_t kb;
};

template <int MT, int NT>
struct Frag {
  u32x4_t a[MT][4];
  u32x4_t b[NT][4];
};

// Rows >= M of the A operand only feed rows >= M of C, which are never
// stored, so padded lanes simply re-read row M-1: no masks, no branches around
// loads (a predicated load hides from the compiler's vmcnt bookkeeping and
// serialises the pipeline).
template <int MT, int NT>
__device__ __forceinline__ void load_kblock(Frag<MT, NT>& f, const u32x4_t* __restrict__ wp, WStride ws,
                                            const bf16_t* const* xrow, int kb, int lane) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const u32x4_t* src = wp + t * ws.tile + (size_t)kb * ws.kb + lane;
#pragma unroll
    for (int j = 0; j < 4; ++j) f.b[t][j] = __builtin_nontemporal_load(src + j * 64);
  }
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const u32x4_t* src = (const u32x4_t*)(xrow[m] + kb * 64);
#pragma unroll
    for (int j = 0; j < 4; ++j) f.a[m][j] = src[j];
  }
}

// Split halves of load_kblock for the double-buffered schedule: W (HBM
// stream) and X (L2-resident) fragments.
template <int MT, int NT>
__device__ __forceinline__ void load_w_kblock(Frag<MT, NT>& f, const u32x4_t* __restrict__ wp, WStride ws,
                                              int kb, int lane) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const u32x4_t* src = wp + t * ws.tile + (size_t)kb * ws.kb + lane;
#pragma unroll
    for (int j = 0; j < 4; ++j) f.b[t][j] = __builtin_nontemporal_load(src + j * 64);
  }
}

template <int MT, int NT>
__device__ __forceinline__ void load_x_kblock(Frag<MT, NT>& f, const bf16_t* const* xrow, int kb) {
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const u32x4_t* src = (const u32x4_t*)(xrow[m] + kb * 64);
#pragma unroll
    for (int j = 0; j < 4; ++j) f.a[m][j] = src[j];
  }
}

template <int MT, int NT>
__device__ __forceinline__ void mma_kblock(const Frag<MT, NT>& f, f32x16_t (&acc)[MT][NT]) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[m][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, f.a[m][j]),
                                                            __builtin_bit_cast(bf16x8_t, f.b[t][j]), acc[m][t],
                                                            0, 0, 0);
}

// LDS tile index of C element (row, col) of n-tile t.
// 32x32x16 accumulator layout: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
template <int NT>
__device__ __forceinline__ int red_index(int row, int t, int col) {
  const int m = row >> 5, rr = row & 31;
  const int reg = (rr & 3) + 4 * (rr >> 3);
  return ((m * NT + t) * 16 + reg) * 64 + col + 32 * ((rr >> 2) & 1);
}

__device__ __forceinline__ void store8(bf16_t* dst, const float* v) {
  uint32_t pk[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) pk[e] = (uint32_t)f2bf(v[2 * e]) | ((uint32_t)f2bf(v[2 * e + 1]) << 16);
  *(uint4*)dst = make_uint4(pk[0], pk[1], pk[2], pk[3]);
}

// Final epilogue over a 32*MT x 32*NT tile whose fp32 sums are read through
// `get(row, t, col)` (LDS for S == 1, the global scratch for S > 1).
template <int MT, int NT, int KS, int EPI, class Get>
__device__ __forceinline__ void epilogue(Get get, bf16_t* __restrict__ y, int M, int ldy, int tile0, int group) {
  const int tid = threadIdx.x;
  if (EPI == EPI_STORE) {
    constexpr int C8 = NT * 4;  // 8-column pieces per row
    for (int it = tid; it < MT * 32 * C8; it += 64 * KS) {
      const int row = it / C8, c8 = it % C8;
      if (row >= M) continue;
      const int t = c8 >> 2, col = (c8 & 3) * 8;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = get(row, t, col + e);
      store8(y + (size_t)row * ldy + (size_t)(tile0 + t) * 32 + col, v);
    }
  } else {  // EPI_SILU_MUL (NT == 2): t 0 = gate, t 1 = up of channel block `group`
    for (int it = tid; it < MT * 32 * 4; it += 64 * KS) {
      const int row = it >> 2, col = (it & 3) * 8;
      if (row >= M) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        // round gate/up to bf16 first: matches an unfused bf16 GEMM + silu_mul
        const float g = round_bf(get(row, 0, col + e)), u = round_bf(get(row, 1, col + e));
        v[e] = g / (1.f + __expf(-g)) * u;
      }
      store8(y + (size_t)row * ldy + (size_t)group * 32 + col, v);
    }
  }
}

// Scheduling + compiler barrier: sched_barrier pins the machine schedule, the
// empty asm with a memory clobber keeps IR passes from hoisting the next
// buffer's (restrict, hence freely movable) loads above the MFMAs still reading
// the registers they would overwrite -- which forces renamed registers and
// loop-end copies that wait for every load (vmcnt(0)).
#define DB_FENCE()                          \
  do {                                      \
    __builtin_amdgcn_sched_barrier(0);      \
    asm volatile("" ::: "memory");          \
  } while (0)

template <int MT, int NT, int KS, int EPI, bool DB>
__global__ void __launch_bounds__(64 * KS)
skinny_gemm_kernel(const u32x4_t* __restrict__ wp, const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int M,
                   int K, int N, int ldx, int ldy, int S, float* __restrict__ scratch, int* __restrict__ tickets,
                   int kmajor) {
  __shared__ float red[MT * NT * 16 * 64];
  __shared__ int last;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int KB = K >> 6;
  const int group = blockIdx.x / S, split = blockIdx.x % S;
  const int tile0 = group * NT;
  const WStride ws = kmajor ? WStride{256, (size_t)(N >> 5) * 256} : WStride{(size_t)KB * 256, 256};
  const u32x4_t* wbase = wp + (size_t)tile0 * ws.tile;

  for (int i = tid; i < MT * NT * 16 * 64; i += 64 * KS) red[i] = 0.f;

  const bf16_t* xrow[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) xrow[m] = x + (size_t)min(m * 32 + r, M - 1) * ldx + 32 * h;
  // k-block range: split of the workgroup, then wave of the split
  const int sb0 = (int)((long long)KB * split / S), sb1 = (int)((long long)KB * (split + 1) / S);
  const int kb0 = sb0 + (int)((long long)(sb1 - sb0) * wave / KS);
  const int kb1 = sb0 + (int)((long long)(sb1 - sb0) * (wave + 1) / KS);

  f32x16_t acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[m][t][e] = 0.f;

  int kb = kb0;
  if constexpr (DB) {
    // W (the HBM stream) alternates between two register buffers, the next
    // group's loads issued before the current group's MFMAs, with no branch
    // around a load in the steady state.  X comes from L2 just in time for its
    // group and is issued *before* the W prefetch (vmcnt retires in issue
    // order: waiting for X must not wait for the prefetch), so no X fragment is
    // loop-carried (a loop-carried X buffer gets
    // renamed by the register allocator and copied back at the loop end behind
    // a vmcnt(0) that drains the whole pipeline).  The last one or two groups
    // are peeled.
    constexpr int U = unroll_db(MT, NT);
    const int G = (kb1 - kb0) / U;
    if (G > 0) {
      Frag<MT, NT> fa[U], fb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) load_w_kblock<MT, NT>(fa[u], wbase, ws, kb + u, lane);
      int g = 0;
      for (; g + 3 <= G; g += 2, kb += 2 * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) load_x_kblock<MT, NT>(fa[u], xrow, kb + u);
#pragma unroll
        for (int u = 0; u < U; ++u) load_w_kblock<MT, NT>(fb[u], wbase, ws, kb + U + u, lane);
        DB_FENCE();
#pragma unroll
        for (int u = 0; u < U; ++u) mma_kblock<MT, NT>(fa[u], acc);
        DB_FENCE();
#pragma unroll
        for (int u = 0; u < U; ++u) load_x_kblock<MT, NT>(fb[u], xrow, kb + U + u);
#pragma unroll
        for (int u = 0; u < U; ++u) load_w_kblock<MT, NT>(fa[u], wbase, ws, kb + 2 * U + u, lane);
        DB_FENCE();
#pragma unroll
        for (int u = 0; u < U; ++u) mma_kblock<MT, NT>(fb[u], acc);
        DB_FENCE();
      }
      if (G - g == 2) {
#pragma unroll
        for (int u = 0; u < U; ++u) load_x_kblock<MT, NT>(fa[u], xrow, kb + u);
#pragma unroll
        for (int u = 0; u < U; ++u) load_w_kblock<MT, NT>(fb[u], wbase, ws, kb + U + u, lane);
        DB_FENCE();
#pragma unroll
        for (int u = 0; u < U; ++u) mma_kblock<MT, NT>(fa[u], acc);
        DB_FENCE();
#pragma unroll
        for (int u = 0; u < U; ++u) load_x_kblock<MT, NT>(fb[u], xrow, kb + U + u);
        DB_FENCE();
#pragma unroll
        for (int u = 0; u < U; ++u) mma_kblock<MT, NT>(fb[u], acc);
        kb += 2 * U;
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) load_x_kblock<MT, NT>(fa[u], xrow, kb + u);
        DB_FENCE();
#pragma unroll
        for (int u = 0; u < U; ++u) mma_kblock<MT, NT>(fa[u], acc);
        kb += U;
      }
    }
  } else {
    // Groups of U k-blocks: every load of the group is issued before the first
    // MFMA, which then consume them in order behind decreasing vmcnt waits.
    // (A rotated one-ahead pipeline gets re-serialised by the compiler.)
    constexpr int U = unroll_of(MT, NT);
    for (; kb + U <= kb1; kb += U) {
      Frag<MT, NT> f[U];
#pragma unroll
      for (int u = 0; u < U; ++u) load_kblock<MT, NT>(f[u], wbase, ws, xrow, kb + u, lane);
      // keep the whole group in flight: the occupancy-driven scheduler would
      // otherwise sink loads behind MFMAs (≈2 loads in flight per wave)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) mma_kblock<MT, NT>(f[u], acc);
    }
  }
  for (; kb < kb1; ++kb) {
    Frag<MT, NT> f;
    load_kblock<MT, NT>(f, wbase, ws, xrow, kb, lane);
    mma_kblock<MT, NT>(f, acc);
  }
  __syncthreads();  // red[] zeroed
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) atomicAdd(&red[((m * NT + t) * 16 + e) * 64 + lane], acc[m][t][e]);
  __syncthreads();

  if (S == 1) {
    epilogue<MT, NT, KS, EPI>([&](int row, int t, int col) { return red[red_index<NT>(row, t, col)]; }, y, M, ldy,
                              tile0, group);
    return;
  }
  // Inter-workgroup split: add this split's tile into the zeroed fp32 slab
  // scratch[group][MT*32][C] with device-scope float atomics, take a ticket,
  // and the last of the S workgroups runs the epilogue from the slab, then
  // re-zeroes slab and ticket for the next call / graph replay.  The atomics
  // are performed at the coherence point, so draining them (vmcnt(0)) before
  // the ticket is all the ordering needed.  Measured alternatives, both slower
  // (profiles/gemm): an agent-scope release/acquire fence (writes back /
  // invalidates the XCD's whole L2 in every workgroup: 3-10x) and per-split
  // slabs written with write-through stores then summed by the last arriver.
  constexpr int C = NT * 32;
  constexpr int SLAB = MT * 32 * C;
  float* sc = scratch + (size_t)group * SLAB;
  for (int it = tid; it < SLAB; it += 64 * KS) {
    const int row = it / C, c = it % C;
    if (row < M) atomicAdd(sc + it, red[red_index<NT>(row, c >> 5, c & 31)]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) last = (atomicAdd(tickets + group, 1) == S - 1);
  __syncthreads();
  if (!last) return;
  epilogue<MT, NT, KS, EPI>(
      [&](int row, int t, int col) {
        return __hip_atomic_load(sc + row * C + t * 32 + col, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      },
      y, M, ldy, tile0, group);
  __syncthreads();
  for (int it = tid; it < SLAB; it += 64 * KS) sc[it] = 0.f;
  if (tid == 0) tickets[group] = 0;
}

// ============================================================================
// Wide workgroups: WV waves own different n-tiles over the SAME k-range, so the
// workgroup needs each X k-block once.  X is loaded cooperatively with fully
// coalesced 16-byte loads (row-major, 8 cache lines per KiB instead of 32)
// into a padded, double-buffered LDS tile, and each wave reads its MFMA
// A-operands with ds_read_b128.  Measured at 64 CUs, the per-wave X loads of
// the kernel above (each instruction touches 32 rows x 32 B) are what limits
// it: with X taken out of the loop the same W stream runs 1.5-1.6x faster
// (profiles/gemm_cu64_nox.json).  W stays double-buffered in registers (the
// next group's loads issued before the current group's MFMAs); one barrier per
// group hands the next X tile over.  No LDS reduction: every wave finishes its
// own tiles from its accumulators; inter-workgroup split S as above.
constexpr int unroll_wide(int nt) { return nt >= 4 ? 1 : (nt == 2 ? 2 : 4); }

template <int NT>
struct WFrag {
  u32x4_t b[NT][4];
};

template <int NT, int U>
__device__ __forceinline__ void wide_load_w(WFrag<NT> (&f)[U], const u32x4_t* __restrict__ wp, WStride ws, int kb,
                                            int lane) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const u32x4_t* src = wp + t * ws.tile + (size_t)(kb + u) * ws.kb + lane;
#pragma unroll
      for (int j = 0; j < 4; ++j) f[u].b[t][j] = __builtin_nontemporal_load(src + j * 64);
    }
}

// Hand-offs inside one launch (decode_chain_kernel): bytes a workgroup of the
// same grid produced are stored write-through (sc1, 4 or 16 bytes) and loaded
// with sc1 buffer loads -- coherent across the XCDs' L2s with no L2
// write-back or invalidate (MI355X_MICROARCH.md, hand-offs with sc1 loads).
constexpr int AUX_SC1 = 16;   // cache-policy bit sc1

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)0xffffffff, 0x00020000);
}

__device__ __forceinline__ u32x4_t load16_sc1(const void* base, size_t byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(base), (int)byte_off, 0, AUX_SC1);
}

__device__ __forceinline__ void store4_sc1(void* p, uint32_t v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// X[MT*32 rows][U*64 k] of k-blocks kb.. as MT*U*256 16-byte chunks, row-major,
// XC per thread (rows >= M re-read row M-1: never stored, no masks).  SC1: X
// was produced earlier in the same launch.
template <int MT, int U, int XC, bool SC1 = false>
__device__ __forceinline__ void wide_load_x(u32x4_t (&xr)[XC], const bf16_t* __restrict__ x, int M, int ldx, int kb,
                                            int tid, int nthreads) {
#pragma unroll
  for (int i = 0; i < XC; ++i) {
    const int c = tid + i * nthreads;
    const int row = c / (U * 8), c8 = c % (U * 8);
    const size_t off = (size_t)min(row, M - 1) * ldx + kb * 64 + c8 * 8;
    if constexpr (SC1)
      xr[i] = load16_sc1(x, off * 2);
    else
      xr[i] = *(const u32x4_t*)(x + off);
  }
}

template <int MT, int U, int XC, int PITCH>
__device__ __forceinline__ void wide_store_x(bf16_t* xs, const u32x4_t (&xr)[XC], int tid, int nthreads) {
#pragma unroll
  for (int i = 0; i < XC; ++i) {
    const int c = tid + i * nthreads;
    const int row = c / (U * 8), c8 = c % (U * 8);
    *(u32x4_t*)(xs + row * PITCH + c8 * 8) = xr[i];
  }
}

// The K-split kernel's X tile by LDS-DMA (MIVGPU_WIDEK_DMAX=1, A/B): with 8
// k-blocks per group a row of the group's X is 1 KB, one 64-lane 16-byte
// global_load_lds straight into its padded LDS row -- no VGPR staging, no
// ds_write; the wave's loads complete in issue order, so waiting for all but
// the W loads issued after it (vmcnt) covers the tile.  Measured slower
// (decode step 4.654-4.678 vs 4.573-4.575 ms, batch 32): the compiler cannot
// tell the DMA's LDS buffer from the one the MFMAs read and waits for every
// load in flight (vmcnt(0)) before those reads in every other group, so the
// next group's W no longer streams across the MFMAs.  Kept as an A/B option.
template <int MT, int GK, int PITCH, int WAVES>
__device__ __forceinline__ void widek_dma_x(bf16_t* xs, const bf16_t* __restrict__ x, int M, int ldx, int kb, int wave,
                                            int lane) {
  static_assert(GK * 64 * 2 == 64 * 16, "one row of the group's X is one 64-lane 16-byte DMA");
#pragma unroll
  for (int i = 0; i < MT * 32 / WAVES; ++i) {
    const int r = wave + i * WAVES;   // wave-uniform
    const bf16_t* g = x + (size_t)min(r, M - 1) * ldx + kb * 64 + lane * 8;
    __builtin_amdgcn_global_load_lds(g, xs + r * PITCH, 16, 0, 0);
  }
}

// X from decode-attention split partials instead of a bf16 matrix (batch 1):
// the K-split kernel builds the whole combined row in LDS once, before its W
// loop, computed as decode_attn_combine_kernel does (csrc/ops/model_ops.hip:
// online merge in split order, fp32, one bf16 rounding), so the GEMM sees
// bit-identical X and the combine launch goes.
struct XComb {
  const float* o;        // [B][Hq][nsplit][128]
  const float* ml;       // [B][Hq][nsplit][2]: max (natural-log units) and sum
  const int* seqlens;    // [B]
  int nsplit, split_keys, max_ctx, hq;
};
constexpr int XC_MAXS = 8;   // splits (<= 2048 keys of context)
constexpr int XC_NCH = 2;    // 8-column chunks per thread: K <= 16 * threads

__device__ __forceinline__ uint32_t pack_bf2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

// Row 0's combined X into xrow[0..K) (every load of the thread's chunks issued
// before the merge: one memory round trip).
__device__ __forceinline__ void xcomb_row(bf16_t* xrow, const XComb& xc, int K, int tid, int nthreads) {
  const int L = min(xc.seqlens[0], xc.max_ctx);
  const int active = min(xc.nsplit, L > 0 ? (L + xc.split_keys - 1) / xc.split_keys : 0);
  float mv[XC_NCH][XC_MAXS], lv[XC_NCH][XC_MAXS];
  float4 oa[XC_NCH][XC_MAXS], ob[XC_NCH][XC_MAXS];
#pragma unroll
  for (int c = 0; c < XC_NCH; ++c) {
    const int col = min((tid + c * nthreads) * 8, K - 8), h = col >> 7, d = col & 127;
    const size_t base = (size_t)h * xc.nsplit;
#pragma unroll
    for (int sp = 0; sp < XC_MAXS; ++sp) {
      const int q = sp < active ? sp : 0;
      mv[c][sp] = xc.ml[(base + q) * 2];
      lv[c][sp] = xc.ml[(base + q) * 2 + 1];
      oa[c][sp] = *reinterpret_cast<const float4*>(xc.o + (base + q) * 128 + d);
      ob[c][sp] = *reinterpret_cast<const float4*>(xc.o + (base + q) * 128 + d + 4);
    }
  }
#pragma unroll
  for (int c = 0; c < XC_NCH; ++c) {
    const int col = (tid + c * nthreads) * 8;
    float Mx = -INFINITY, den = 0.f, num[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) num[e] = 0.f;
#pragma unroll
    for (int sp = 0; sp < XC_MAXS; ++sp) {
      if (sp >= active || mv[c][sp] == -INFINITY) continue;
      const float nm = fmaxf(Mx, mv[c][sp]);
      const float a = Mx == -INFINITY ? 0.f : __expf(Mx - nm), w = __expf(mv[c][sp] - nm);
      const float ov[8] = {oa[c][sp].x, oa[c][sp].y, oa[c][sp].z, oa[c][sp].w,
                           ob[c][sp].x, ob[c][sp].y, ob[c][sp].z, ob[c][sp].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) num[e] = num[e] * a + w * ov[e];
      den = den * a + w * lv[c][sp];
      Mx = nm;
    }
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = den > 0.f ? num[e] / den : 0.f;
    if (col < K)
      *reinterpret_cast<u32x4_t*>(xrow + col) =
          u32x4_t{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7])};
  }
}

// MFMAs of one group with the A operand from ONE LDS row (batch 1: rows >= 1
// of the 32x32 product are never stored, so every lane reads row 0 -- an LDS
// broadcast).
template <int NT, int U>
__device__ __forceinline__ void wide_mma_row(const WFrag<NT> (&f)[U], const bf16_t* xr, f32x16_t (&acc)[1][NT], int h) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32x4_t a = *(const u32x4_t*)(xr + u * 64 + 32 * h + 8 * j);
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                            __builtin_bit_cast(bf16x8_t, f[u].b[t][j]), acc[0][t], 0, 0, 0);
    }
}

template <int MT, int NT, int U, int PITCH>
__device__ __forceinline__ void wide_mma(const WFrag<NT> (&f)[U], const bf16_t* xs, f32x16_t (&acc)[MT][NT], int r,
                                         int h) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const u32x4_t a = *(const u32x4_t*)(xs + (m * 32 + r) * PITCH + u * 64 + 32 * h + 8 * j);
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[m][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                              __builtin_bit_cast(bf16x8_t, f[u].b[t][j]), acc[m][t],
                                                              0, 0, 0);
      }
}

// One group: (prefetch the next group's X then W,) MFMAs of this group from
// `cur` + LDS buffer `xc`, (then stage the prefetched X into `xn` and hand it
// over with the barrier).  X is issued before W: vmcnt retires in issue
// order, so staging X never waits for the W prefetch.
template <int MT, int NT, int U, int XC, int PITCH, bool PREFETCH, bool SC1 = false>
__device__ __forceinline__ void wide_step(const WFrag<NT> (&cur)[U], WFrag<NT> (&nxt)[U], const bf16_t* xc,
                                          bf16_t* xn, f32x16_t (&acc)[MT][NT], const u32x4_t* __restrict__ wbase,
                                          WStride ws, const bf16_t* __restrict__ x, int M, int ldx, int kb, int tid,
                                          int nthreads, int lane, int r, int h) {
  u32x4_t xr[XC];
  if constexpr (PREFETCH) {
    wide_load_x<MT, U, XC, SC1>(xr, x, M, ldx, kb + U, tid, nthreads);
    wide_load_w<NT, U>(nxt, wbase, ws, kb + U, lane);
  }
  DB_FENCE();
  wide_mma<MT, NT, U, PITCH>(cur, xc, acc, r, h);
  DB_FENCE();
  if constexpr (PREFETCH) {
    wide_store_x<MT, U, XC, PITCH>(xn, xr, tid, nthreads);
    __syncthreads();
  }
}

// 32x32x16 accumulator element e of lane (r, h): row (e&3) + 8*(e>>2) + 4h, column r.
__device__ __forceinline__ int acc_row(int e, int h) { return (e & 3) + 8 * (e >> 2) + 4 * h; }

// Per-wave LDS tile of the residual epilogue's squares: [MT*32 rows][SQ_PITCH].
constexpr int SQ_PITCH = 40;   // 16-byte aligned rows; rows r and r+4 (the two lane halves) 32 banks apart

// SC1 (the output is handed to a later projection of the same launch): the
// bf16 results go out as 4-byte write-through stores of column pairs -- lanes
// r and r^1 hold columns r, r^1 of the same rows; one shuffle per row pair
// gives the even lane (col r, r+1) of row e and the odd lane (col r-1, r) of
// row e+1.
__device__ __forceinline__ void store_pair_sc1(bf16_t* __restrict__ y, int M, int ldy, int col0, int row0, int r,
                                               float v0, float v1) {
  // v0, v1: this lane's values of rows row0 (e even) and row0 + 1 (e odd), column col0 + r
  const bool odd = r & 1;
  const float recv = __shfl_xor(odd ? v0 : v1, 1, 64);
  const int row = odd ? row0 + 1 : row0;
  const uint32_t pk = odd ? pack_bf2(recv, v1) : pack_bf2(v0, recv);
  if (row < M) store4_sc1(y + (size_t)row * ldy + col0 + (r & ~1), pk);
}

template <int MT, int NT, int EPI, bool SC1 = false, class Get>
__device__ __forceinline__ void wide_epilogue(Get get, bf16_t* __restrict__ y, int M, int ldy, int tile0,
                                              int vgroup, int r, int h, const float* rs, float* __restrict__ ss_out,
                                              const bf16_t* res_lds, float* sq_lds = nullptr) {
  if constexpr (SC1 && EPI == EPI_RESID) {
    // as below, the new values kept for the paired write-through stores
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float vv[NT][16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m * 32 + acc_row(e, h);
        float sq = 0.f;
        const float sc = (row < M && rs) ? rs[row] : 1.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const bf16_t old = res_lds[((m * NT + t) * 32 + (row - m * 32)) * 32 + r];
          const float v = round_bf(__uint_as_float((uint32_t)old << 16) + get(m, t, e) * sc);
          vv[t][e] = v;
          sq += row < M ? v * v : 0.f;
        }
        sq_lds[row * SQ_PITCH + r] = sq;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 8; ++i)
          store_pair_sc1(y, M, ldy, (tile0 + t) * 32, m * 32 + acc_row(2 * i, h), r, vv[t][2 * i], vv[t][2 * i + 1]);
    }
    const int lane = r + 32 * h, half = lane & 1;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int row = m * 32 + (lane >> 1);
      const float4* p = reinterpret_cast<const float4*>(sq_lds + row * SQ_PITCH + 16 * half);
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 q = p[j];
        sum += (q.x + q.y) + (q.z + q.w);
      }
      sum += __shfl_xor(sum, 1, 64);
      if (half == 0) __hip_atomic_store(&ss_out[(size_t)vgroup * SS_ROWS + row], sum, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if constexpr (SC1 && EPI == EPI_SILU_MUL) {
    static_assert(NT == 2, "SiLU*up: a gate/up tile pair");
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float v[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int e = 2 * i + k, row = m * 32 + acc_row(e, h);
          const float sc = (row < M && rs) ? rs[row] : 1.f;
          const float g = round_bf(get(m, 0, e) * sc), u = round_bf(get(m, 1, e) * sc);
          v[k] = g / (1.f + __expf(-g)) * u;
        }
        store_pair_sc1(y, M, ldy, vgroup * 32, m * 32 + acc_row(2 * i, h), r, v[0], v[1]);
      }
    return;
  }
  if constexpr (EPI == EPI_RESID) {
    // update; each lane's squares (one column r of 16 rows) go to the wave's
    // LDS tile, then lane l sums half of row l/2 with four 16-byte reads
    // (was 5 dependent cross-lane shuffles per row: 80 per lane, ~3 us)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m * 32 + acc_row(e, h);
        float sq = 0.f;
        if (row < M) {
          const float sc = rs ? rs[row] : 1.f;
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            // the old residual was prefetched into this wave's LDS tile (row, 32t + r)
            const bf16_t old = res_lds[((m * NT + t) * 32 + (row - m * 32)) * 32 + r];
            const float v = round_bf(__uint_as_float((uint32_t)old << 16) + get(m, t, e) * sc);
            y[(size_t)row * ldy + (size_t)(tile0 + t) * 32 + r] = f2bf(v);
            sq += v * v;
          }
        }
        sq_lds[row * SQ_PITCH + r] = sq;
      }
    const int lane = r + 32 * h, half = lane & 1;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int row = m * 32 + (lane >> 1);
      const float4* p = reinterpret_cast<const float4*>(sq_lds + row * SQ_PITCH + 16 * half);
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 q = p[j];
        sum += (q.x + q.y) + (q.z + q.w);
      }
      sum += __shfl_xor(sum, 1, 64);
      if (half == 0) ss_out[(size_t)vgroup * SS_ROWS + row] = sum;
    }
    return;
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = m * 32 + acc_row(e, h);
      if (row >= M) continue;
      const float sc = rs ? rs[row] : 1.f;
      if constexpr (EPI == EPI_STORE) {
#pragma unroll
        for (int t = 0; t < NT; ++t) y[(size_t)row * ldy + (size_t)(tile0 + t) * 32 + r] = f2bf(get(m, t, e) * sc);
      } else if constexpr (NT == 2) {  // SiLU(gate)*up: tile pair (gate, up) of channel block `vgroup`
        const float g = round_bf(get(m, 0, e) * sc), u = round_bf(get(m, 1, e) * sc);
        y[(size_t)row * ldy + (size_t)vgroup * 32 + r] = f2bf(g / (1.f + __expf(-g)) * u);
      }
    }
}

// Row scales of the workgroup's MT*32 rows from the producer's per-wave-group
// sum-of-squares slots, in two halves so the loads overlap the W stream:
// rs_issue() issues one 16-byte load per (slot, 4 rows) -- RS_LMAX per thread
// -- before the first X/W loads; rs_finish() (after them, from every thread)
// reduces in registers, across lanes and through LDS (its internal barrier
// publishes s_rs).  vmcnt retires in issue order, so the reduction waits for
// the slot loads only.
constexpr int RS_LMAX = 8;

template <int MT, int NTHREADS, bool SC1 = false>
__device__ __forceinline__ void rs_issue(float4 (&v)[RS_LMAX], const float* __restrict__ part, int nparts, int tid) {
  constexpr int RC = MT * 8;                 // float4 chunks per slot (MT*32 rows)
  constexpr int PER = NTHREADS / RC;         // slots read in parallel
  static_assert(NTHREADS % RC == 0, "row chunks must tile the workgroup");
  const int rc = tid % RC, p0 = tid / RC;
#pragma unroll
  for (int i = 0; i < RS_LMAX; ++i) {
    const int pp = p0 + i * PER;
    if constexpr (SC1) {
      // a clamped slot address (always loaded: no branch around the load), zeroed when unused
      const u32x4_t q = load16_sc1(part, ((size_t)min(pp, nparts - 1) * SS_ROWS + 4 * rc) * 4);
      v[i] = pp < nparts ? __builtin_bit_cast(float4, q) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      v[i] = pp < nparts ? *(const float4*)(part + (size_t)pp * SS_ROWS + 4 * rc) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

template <int MT, int NTHREADS>
__device__ __forceinline__ void rs_finish(const float4 (&v)[RS_LMAX], float inv_dim, float eps, float* s_rs,
                                          float* s_tmp, int tid) {
  constexpr int RC = MT * 8;
  constexpr int WV = NTHREADS / 64;
  const int rc = tid % RC;
  float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < RS_LMAX; ++i) {
    sum.x += v[i].x; sum.y += v[i].y; sum.z += v[i].z; sum.w += v[i].w;
  }
  // threads with the same rc: lanes rc + RC*j of each wave, then across waves
#pragma unroll
  for (int o = RC; o < 64; o <<= 1) {
    sum.x += __shfl_xor(sum.x, o, 64);
    sum.y += __shfl_xor(sum.y, o, 64);
    sum.z += __shfl_xor(sum.z, o, 64);
    sum.w += __shfl_xor(sum.w, o, 64);
  }
  if ((tid & 63) < RC) {
    const int w = tid >> 6;
    s_tmp[(w * RC + rc) * 4 + 0] = sum.x;
    s_tmp[(w * RC + rc) * 4 + 1] = sum.y;
    s_tmp[(w * RC + rc) * 4 + 2] = sum.z;
    s_tmp[(w * RC + rc) * 4 + 3] = sum.w;
  }
  __syncthreads();
  if (tid < MT * 32) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < WV; ++w) t += s_tmp[w * RC * 4 + tid];
    s_rs[tid] = rsqrtf(t * inv_dim + eps);
  }
}

// Arguments of one projection (the wide and K-split bodies below).
struct GemmP {
  const u32x4_t* wp;
  const bf16_t* x;
  bf16_t* y;
  int M, K, N, ldx, ldy, S;
  float* scratch;
  int* tickets;
  int kmajor;
  const float* rs_part;
  int rs_nparts;
  float rs_inv_dim, rs_eps;
  float* ss_out;
};

// Dependency hook of a projection body.  The standalone kernels take NoDeps
// (every input is complete at launch).  In the chained decode launch
// (decode_chain_kernel below) a body waits for its producers after the
// workgroup's first W group is in flight -- the weights do not depend on the
// previous projection, only X does -- and publishes every finished
// wave-group's output to its consumers.
struct NoDeps {
  static constexpr bool chained = false;
  static constexpr bool sc1_loads = false;
  __device__ void wait(int, int) const {}
  __device__ void publish(int) const {}
};

// LDS of the wide body (one struct: the chained launch overlays the bodies of
// several projections in one buffer).
template <int MT, int NT, int WV, int EPI>
struct WideLds {
  static constexpr int U = unroll_wide(NT);
  static constexpr int PITCH = U * 64 + 8;   // +16 B per row: conflict-free ds_read_b128
  static constexpr int XBUF = MT * 32 * PITCH;
  static constexpr bool RS = EPI != EPI_RESID;   // row scales (the residual epilogue produces the sums)
  alignas(16) bf16_t xs[2 * XBUF];
  alignas(16) float s_rs[MT * 32];
  alignas(16) float s_rtmp[RS ? WV * MT * 32 : 4];
  // EPI_RESID: each wave's residual tile [m][t][32 rows][32 cols], prefetched by LDS-DMA
  alignas(16) bf16_t s_res[EPI == EPI_RESID ? WV * MT * NT * 32 * 32 : 8];
  // EPI_RESID: each wave's squares tile for the row sums (wide_epilogue)
  alignas(16) float s_sq[EPI == EPI_RESID ? WV * MT * 32 * SQ_PITCH : 4];
};

template <int MT, int NT, int WV, int EPI, class Deps>
__device__ __forceinline__ void wide_body(const GemmP& p, int block, WideLds<MT, NT, WV, EPI>& L, const Deps& deps) {
  static_assert(EPI != EPI_SILU_MUL || NT == 2, "SiLU*up pairs a gate tile with an up tile");
  using LD = WideLds<MT, NT, WV, EPI>;
  constexpr int U = LD::U;
  constexpr int PITCH = LD::PITCH;
  constexpr int XBUF = LD::XBUF;
  constexpr int NTHREADS = 64 * WV;
  constexpr int XC = MT * U * 256 / NTHREADS;       // X chunks per thread per group
  static_assert(XC * NTHREADS == MT * U * 256, "X tile must split evenly over the workgroup");
  constexpr bool RS = LD::RS;
  // chained: X, slots and the residual tile come from this launch -- sc1
  // loads, or plain ones after the waiting wave's acquire (ChainDeps ACQ)
  constexpr bool SC1 = Deps::sc1_loads;
  constexpr bool WT = Deps::chained;                // write-through stores of the handed-off output
  const u32x4_t* __restrict__ wp = p.wp;
  const bf16_t* __restrict__ x = p.x;
  bf16_t* __restrict__ y = p.y;
  const int M = p.M, ldx = p.ldx, ldy = p.ldy, S = p.S;
  bf16_t* xs = L.xs;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int KB = p.K >> 6;
  const int wg = block / S, split = block % S;
  const int vgroup = wg * WV + wave;
  const int tile0 = vgroup * NT;
  const WStride ws = p.kmajor ? WStride{256, (size_t)(p.N >> 5) * 256} : WStride{(size_t)KB * 256, 256};
  const u32x4_t* wbase = wp + (size_t)tile0 * ws.tile;
  const int kb0 = (int)((long long)KB * split / S), kb1 = (int)((long long)KB * (split + 1) / S);
  const int G = (kb1 - kb0) / U;                    // the plan makes (kb1 - kb0) a multiple of U, >= U

  f32x16_t acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[m][t][e] = 0.f;

  WFrag<NT> fa[U], fb[U];
  // Row-scale slot loads are issued first and reduced after the first X/W
  // loads are in flight (vmcnt retires in order: the reduction waits only for
  // them); the barrier below publishes s_rs.
  const float* rs = (RS && p.rs_part) ? L.s_rs : nullptr;
  bf16_t* res_lds = L.s_res + (EPI == EPI_RESID ? wave * (MT * NT * 32 * 32) : 0);
  if constexpr (Deps::chained) {
    // chained: this wave-group's first W group goes out before the wait on
    // the producers (the polling wave issues its own after the wait: the
    // acquire drains its loads)
    if (wave != WV - 1) wide_load_w<NT, U>(fa, wbase, ws, kb0, lane);
    deps.wait(WV - 1, split);
    if (wave == WV - 1) wide_load_w<NT, U>(fa, wbase, ws, kb0, lane);
  }
  // chained residual update: the old residual tile was written earlier in the
  // same launch, so it comes in by sc1 loads to registers (written to the
  // wave's LDS tile before the epilogue) instead of LDS-DMA
  constexpr int RCH = (EPI == EPI_RESID && SC1) ? MT * NT * 2 : 1;
  u32x4_t resr[RCH];
  {
    // row-scale slot loads and the residual tile's LDS-DMA first: older than
    // the X loads, so the X wait below covers them as well
    float4 rsv[RS ? RS_LMAX : 1];
    if constexpr (RS) {
      if (p.rs_part) rs_issue<MT, NTHREADS, SC1>(rsv, p.rs_part, p.rs_nparts, tid);
    }
    if constexpr (EPI == EPI_RESID && SC1) {
      // tile (m, t): 32 rows x 32 columns = 128 16-byte chunks, 2 per lane
#pragma unroll
      for (int q = 0; q < RCH; ++q) {
        const int mt = q >> 1, c = lane + 64 * (q & 1), row = (mt / NT) * 32 + (c >> 2);
        resr[q] = load16_sc1(y, ((size_t)min(row, M - 1) * ldy + (size_t)(tile0 + mt % NT) * 32 + (c & 3) * 8) * 2);
      }
    } else if constexpr (EPI == EPI_RESID) {
      // tile (m, t): 32 rows x 64 B, 4 rows per instruction, lane = (row, 4-byte column pair)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int row = m * 32 + 4 * i + (lane >> 4);
            const bf16_t* g = y + (size_t)min(row, M - 1) * ldy + (size_t)(tile0 + t) * 32 + 2 * (lane & 15);
            __builtin_amdgcn_global_load_lds(g, res_lds + ((m * NT + t) * 32 + 4 * i) * 32, 4, 0, 0);
          }
    }
    u32x4_t xr[XC];
    wide_load_x<MT, U, XC, SC1>(xr, x, M, ldx, kb0, tid, NTHREADS);
    if constexpr (!Deps::chained) wide_load_w<NT, U>(fa, wbase, ws, kb0, lane);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (RS) {
      if (p.rs_part) rs_finish<MT, NTHREADS>(rsv, p.rs_inv_dim, p.rs_eps, L.s_rs, L.s_rtmp, tid);
    }
    wide_store_x<MT, U, XC, PITCH>(xs, xr, tid, NTHREADS);
    __syncthreads();
  }
  int g = 0, kb = kb0;
  for (; g + 3 <= G; g += 2, kb += 2 * U) {
    wide_step<MT, NT, U, XC, PITCH, true, SC1>(fa, fb, xs, xs + XBUF, acc, wbase, ws, x, M, ldx, kb, tid, NTHREADS, lane,
                                          r, h);
    wide_step<MT, NT, U, XC, PITCH, true, SC1>(fb, fa, xs + XBUF, xs, acc, wbase, ws, x, M, ldx, kb + U, tid, NTHREADS,
                                          lane, r, h);
  }
  if (G - g == 2) {
    wide_step<MT, NT, U, XC, PITCH, true, SC1>(fa, fb, xs, xs + XBUF, acc, wbase, ws, x, M, ldx, kb, tid, NTHREADS, lane,
                                          r, h);
    wide_step<MT, NT, U, XC, PITCH, false, SC1>(fb, fa, xs + XBUF, xs, acc, wbase, ws, x, M, ldx, kb + U, tid, NTHREADS,
                                           lane, r, h);
  } else {
    wide_step<MT, NT, U, XC, PITCH, false, SC1>(fa, fb, xs, xs + XBUF, acc, wbase, ws, x, M, ldx, kb, tid, NTHREADS, lane,
                                           r, h);
  }

  float* sq = L.s_sq + wave * (EPI == EPI_RESID ? MT * 32 * SQ_PITCH : 0);
  if constexpr (EPI == EPI_RESID && SC1) {
    // this wave's own LDS tile (read back by this wave only: no barrier)
#pragma unroll
    for (int q = 0; q < RCH; ++q) {
      const int mt = q >> 1, c = lane + 64 * (q & 1);
      *reinterpret_cast<u32x4_t*>(res_lds + (mt * 32 + (c >> 2)) * 32 + (c & 3) * 8) = resr[q];
    }
  } else if constexpr (EPI == EPI_RESID) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // residual tile landed
  }
  if (S == 1) {
    wide_epilogue<MT, NT, EPI, WT>([&](int m, int t, int e) { return acc[m][t][e]; }, y, M, ldy, tile0, vgroup, r, h,
                               rs, p.ss_out, res_lds, sq);
    deps.publish(vgroup);
    return;
  }
  // Inter-workgroup split, per wave: add the tile into this wave-group's fp32
  // slab (lane-major, so the adds and the final reads are coalesced), drain,
  // take a ticket; the last of the S arrivals finishes and re-zeroes.
  constexpr int SLAB = MT * NT * 16 * 64;
  float* sc = p.scratch + (size_t)vgroup * SLAB;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) atomicAdd(sc + ((m * NT + t) * 16 + e) * 64 + lane, acc[m][t][e]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int ticket = 0;
  if (lane == 0) ticket = atomicAdd(p.tickets + vgroup, 1);
  ticket = __shfl(ticket, 0, 64);
  if (ticket != S - 1) return;
  wide_epilogue<MT, NT, EPI, WT>(
      [&](int m, int t, int e) {
        return __hip_atomic_load(sc + ((m * NT + t) * 16 + e) * 64 + lane, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      },
      y, M, ldy, tile0, vgroup, r, h, rs, p.ss_out, res_lds, sq);
#pragma unroll
  for (int i = 0; i < SLAB / 64; ++i) sc[i * 64 + lane] = 0.f;
  if (lane == 0) p.tickets[vgroup] = 0;
  deps.publish(vgroup);
}

template <int MT, int NT, int WV, int EPI>
__global__ void __launch_bounds__(64 * WV) skinny_wide_kernel(GemmP p) {
  __shared__ WideLds<MT, NT, WV, EPI> lds;
  wide_body<MT, NT, WV, EPI>(p, blockIdx.x, lds, NoDeps{});
}

// ============================================================================
// K-split wide workgroups ("widek", variant 3) for the small projections of a
// decode step on the whole chip (qkv 50 MB, o_proj 34 MB, down 101 MB: 128-192
// n-tiles for 256 CUs).  The wide kernel above gives each wave its own n-tile
// over the workgroup's whole k-range, so these shapes ran 96-256 workgroups of
// 1-2 waves -- few bytes in flight per CU -- or split K across workgroups with
// device-scope atomics and a last-arriver epilogue on the critical path.
// Here KW waves share ONE n-tile and interleave its k-blocks (wave kw takes
// k-blocks kw*U.. of every group of KW*U), all fed from one LDS X tile of the
// group's KW*U k-blocks; the KW partial accumulators are summed through LDS at
// the end, so K is split KW ways inside the workgroup with no global traffic.
// An inter-workgroup split S (as above) can still be added to fill the chip.
//
// Row-norm fusion as in the wide kernel: EPI_RESID updates the residual Y in
// place and writes one sum-of-squares slot per n-tile (the old residual tile
// is fetched by LDS-DMA at the start, off the critical path); rs_part != null
// scales the rows of a store by the producer's slots (rs_issue / rs_finish).
// NT = 2 with EPI_SILU_MUL: a gate tile and its up tile (gate_up), both
// carried by every k-wave, SiLU(gate)*up by the reducing wave.
template <int MT, int NT, int KW, int EPI, int UU = 2>
struct WidekLds {
  static constexpr int U = UU;                       // k-blocks per wave per group
  static constexpr int GK = KW * U;                  // k-blocks per group (the X tile)
  static constexpr int PITCH = GK * 64 + 8;          // +16 B per row: conflict-free ds_read_b128
  static constexpr int XBUF = MT * 32 * PITCH;
  static constexpr bool RS = EPI != EPI_RESID;
  alignas(16) bf16_t xs[2 * XBUF];
  alignas(16) float s_rs[MT * 32];
  alignas(16) float s_rtmp[RS ? KW * MT * 32 : 4];
  // EPI_RESID: the old residual tile [m][32 rows][32 cols], prefetched by wave 0
  alignas(16) bf16_t s_res[EPI == EPI_RESID ? MT * 32 * 32 : 8];
};

template <int MT, int NT, int KW, int EPI, bool COMB, class Deps, bool DMAX = false, int UU = 2>
__device__ __forceinline__ void widek_body(const GemmP& p, int block, WidekLds<MT, NT, KW, EPI, UU>& L,
                                           const XComb& xcomb, const Deps& deps) {
  static_assert((EPI == EPI_SILU_MUL) == (NT == 2) && NT <= 2, "widek: one tile, or a gate/up pair for SiLU*up");
  static_assert(!(COMB && Deps::chained), "the X-combine variant runs standalone");
  static_assert(!DMAX || (!COMB && !Deps::chained && KW == 4 && UU == 2), "LDS-DMA X: standalone, 4 k-waves");
  using LD = WidekLds<MT, NT, KW, EPI, UU>;
  constexpr int U = LD::U;
  constexpr int GK = LD::GK;
  constexpr int PITCH = LD::PITCH;
  constexpr int XBUF = LD::XBUF;
  constexpr int NTHREADS = 64 * KW;
  constexpr int XC = MT * GK * 256 / NTHREADS;       // X chunks per thread per group
  static_assert(XC * NTHREADS == MT * GK * 256, "X tile must split evenly over the workgroup");
  static_assert(KW * MT * NT * 16 * 64 * 4 <= 2 * XBUF * 2, "the k-wave reduction reuses the X buffers");
  static_assert((KW * MT * NT * 16 * 64 + MT * 32 * SQ_PITCH) * 4 <= 2 * XBUF * 2,
                "the residual epilogue's squares tile follows the reduction in the X buffers");
  constexpr bool RS = LD::RS;
  // X and slots produced earlier in the same launch (the chained qkv): sc1
  // loads, or plain ones after the acquire; the residual tile of a chained
  // residual update (o_proj, the chain's first projection) comes from the
  // previous launch: LDS-DMA as standalone
  constexpr bool SC1 = Deps::sc1_loads;
  constexpr bool WT = Deps::chained;
  const u32x4_t* __restrict__ wp = p.wp;
  const bf16_t* __restrict__ x = p.x;
  bf16_t* __restrict__ y = p.y;
  const int M = p.M, ldx = p.ldx, ldy = p.ldy, S = p.S;
  bf16_t* xs = L.xs;
  const int tid = threadIdx.x;
  const int kw = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int KB = p.K >> 6;
  const int vgroup = block / S, split = block % S;
  const int tile0 = vgroup * NT;
  const float* rs = (RS && p.rs_part) ? L.s_rs : nullptr;
  const WStride ws = p.kmajor ? WStride{256, (size_t)(p.N >> 5) * 256} : WStride{(size_t)KB * 256, 256};
  const u32x4_t* wbase = wp + (size_t)tile0 * ws.tile;
  const int kb0 = (int)((long long)KB * split / S), kb1 = (int)((long long)KB * (split + 1) / S);
  const int G = (kb1 - kb0) / GK;                    // the plan makes (kb1 - kb0) a multiple of GK, >= GK

  f32x16_t acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[m][t][e] = 0.f;

  WFrag<NT> fa[U], fb[U];
  if constexpr (Deps::chained) {
    // chained: the first W group before the wait on the producers (the
    // polling wave issues its own after it)
    if (kw != KW - 1) wide_load_w<NT, U>(fa, wbase, ws, kb0 + kw * U, lane);
    deps.wait(KW - 1, split);
    if (kw == KW - 1) wide_load_w<NT, U>(fa, wbase, ws, kb0 + kw * U, lane);
  }
  {
    // row-scale slot loads and the residual tile's LDS-DMA first: older than
    // the X loads, so the X wait below covers them as well
    float4 rsv[RS ? RS_LMAX : 1];
    if constexpr (RS) {
      if (p.rs_part) rs_issue<MT, NTHREADS, SC1>(rsv, p.rs_part, p.rs_nparts, tid);
    }
    if constexpr (EPI == EPI_RESID) {
      if (kw == 0) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int row = m * 32 + 4 * i + (lane >> 4);
            const bf16_t* g = y + (size_t)min(row, M - 1) * ldy + (size_t)tile0 * 32 + 2 * (lane & 15);
            __builtin_amdgcn_global_load_lds(g, L.s_res + (m * 32 + 4 * i) * 32, 4, 0, 0);
          }
      }
    }
    if constexpr (COMB) {
      // batch 1, X from attention partials: the whole combined row into LDS
      // once (W loads of the first group already in flight), then a W loop
      // with no X hand-overs
      wide_load_w<NT, U>(fa, wbase, ws, kb0 + kw * U, lane);
      __builtin_amdgcn_sched_barrier(0);
      xcomb_row(xs, xcomb, p.K, tid, NTHREADS);
      if constexpr (RS) {
        if (p.rs_part) rs_finish<MT, NTHREADS>(rsv, p.rs_inv_dim, p.rs_eps, L.s_rs, L.s_rtmp, tid);
      }
      __syncthreads();
      auto stepc = [&](const WFrag<NT>(&cur)[U], WFrag<NT>(&nxt)[U], int kb, bool prefetch) {
        if (prefetch) wide_load_w<NT, U>(nxt, wbase, ws, kb + GK + kw * U, lane);
        DB_FENCE();
        wide_mma_row<NT, U>(cur, xs + (kb + kw * U) * 64, acc, h);
        DB_FENCE();
      };
      int g = 0, kb = kb0;
      for (; g + 3 <= G; g += 2, kb += 2 * GK) {
        stepc(fa, fb, kb, true);
        stepc(fb, fa, kb + GK, true);
      }
      if (G - g == 2) {
        stepc(fa, fb, kb, true);
        stepc(fb, fa, kb + GK, false);
      } else {
        stepc(fa, fb, kb, false);
      }
    } else {
      u32x4_t xr[DMAX ? 1 : XC];
      if constexpr (DMAX) {
        widek_dma_x<MT, GK, PITCH, KW>(xs, x, M, ldx, kb0, kw, lane);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        wide_load_x<MT, GK, XC, SC1>(xr, x, M, ldx, kb0, tid, NTHREADS);
      }
      if constexpr (!Deps::chained) wide_load_w<NT, U>(fa, wbase, ws, kb0 + kw * U, lane);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (RS) {
        if (p.rs_part) rs_finish<MT, NTHREADS>(rsv, p.rs_inv_dim, p.rs_eps, L.s_rs, L.s_rtmp, tid);
      }
      if constexpr (DMAX)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U * NT * 4) : "memory");   // all but this wave's W loads
      else
        wide_store_x<MT, GK, XC, PITCH>(xs, xr, tid, NTHREADS);
      __syncthreads();
    }
  }
  if constexpr (!COMB) {
  // one group: prefetch the next group's X then this wave's W, MFMAs of this
  // group from registers + this wave's columns of the LDS tile, stage X
  auto step = [&](const WFrag<NT>(&cur)[U], WFrag<NT>(&nxt)[U], const bf16_t* xc, bf16_t* xn, int kb,
                  bool prefetch) {
    u32x4_t xr[DMAX ? 1 : XC];
    if (prefetch) {
      if constexpr (DMAX) {
        widek_dma_x<MT, GK, PITCH, KW>(xn, x, M, ldx, kb + GK, kw, lane);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        wide_load_x<MT, GK, XC, SC1>(xr, x, M, ldx, kb + GK, tid, NTHREADS);
      }
      wide_load_w<NT, U>(nxt, wbase, ws, kb + GK + kw * U, lane);
    }
    DB_FENCE();
    wide_mma<MT, NT, U, PITCH>(cur, xc + kw * U * 64, acc, r, h);
    DB_FENCE();
    if (prefetch) {
      if constexpr (DMAX) {
        // the X tile landed (this wave's DMA); a bare barrier: __syncthreads'
        // fence would also wait for the W loads still in flight
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U * NT * 4) : "memory");
        __builtin_amdgcn_s_barrier();
      } else {
        wide_store_x<MT, GK, XC, PITCH>(xn, xr, tid, NTHREADS);
        __syncthreads();
      }
    }
  };
  int g = 0, kb = kb0;
  for (; g + 3 <= G; g += 2, kb += 2 * GK) {
    step(fa, fb, xs, xs + XBUF, kb, true);
    step(fb, fa, xs + XBUF, xs, kb + GK, true);
  }
  if (G - g == 2) {
    step(fa, fb, xs, xs + XBUF, kb, true);
    step(fb, fa, xs + XBUF, xs, kb + GK, false);
  } else {
    step(fa, fb, xs, xs + XBUF, kb, false);
  }
  }   // !COMB
  // sum the KW waves' partial tiles through LDS (the X buffers are free now)
  __syncthreads();
  float* red = reinterpret_cast<float*>(xs);
  if (kw > 0) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) red[((((kw - 1) * MT + m) * NT + t) * 16 + e) * 64 + lane] = acc[m][t][e];
  }
  __syncthreads();
  if (kw > 0) return;
#pragma unroll
  for (int w = 1; w < KW; ++w)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[m][t][e] += red[((((w - 1) * MT + m) * NT + t) * 16 + e) * 64 + lane];
  if constexpr (EPI == EPI_RESID) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // residual tile landed
  if (S == 1) {
    wide_epilogue<MT, NT, EPI, WT>([&](int m, int t, int e) { return acc[m][t][e]; }, y, M, ldy, tile0, vgroup, r, h,
                               rs, p.ss_out, L.s_res, red + KW * MT * NT * 16 * 64);
    deps.publish(vgroup);
    return;
  }
  constexpr int SLAB = MT * NT * 16 * 64;
  float* sc = p.scratch + (size_t)vgroup * SLAB;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) atomicAdd(sc + ((m * NT + t) * 16 + e) * 64 + lane, acc[m][t][e]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int ticket = 0;
  if (lane == 0) ticket = atomicAdd(p.tickets + vgroup, 1);
  ticket = __shfl(ticket, 0, 64);
  if (ticket != S - 1) return;
  wide_epilogue<MT, NT, EPI, WT>(
      [&](int m, int t, int e) {
        return __hip_atomic_load(sc + ((m * NT + t) * 16 + e) * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      },
      y, M, ldy, tile0, vgroup, r, h, rs, p.ss_out, L.s_res, red + KW * MT * NT * 16 * 64);
#pragma unroll
  for (int i = 0; i < SLAB / 64; ++i) sc[i * 64 + lane] = 0.f;
  if (lane == 0) p.tickets[vgroup] = 0;
  deps.publish(vgroup);
}

template <int MT, int NT, int KW, int EPI, bool COMB = false, bool DMAX = false, int UU = 2>
__global__ void __launch_bounds__(64 * KW) skinny_widek_kernel(GemmP p, XComb xcomb) {
  __shared__ WidekLds<MT, NT, KW, EPI, UU> lds;
  widek_body<MT, NT, KW, EPI, COMB, NoDeps, DMAX, UU>(p, blockIdx.x, lds, xcomb, NoDeps{});
}

// ============================================================================
// Chained decode projections: o_proj (+ residual) -> gate_up (+ SiLU*up) ->
// down (+ residual) -> the next layer's qkv in ONE launch.  Separately, each of
// these kernels pays its own ramp and drain: the first W bytes arrive ~2 us
// after the launch and the last workgroups finish alone, ~4-5 us per launch
// (profiles/README.md section 35).  Here the four bodies run as consecutive
// block ranges of one grid.  A workgroup of a later projection is dispatched
// as soon as a CU frees up in the previous one's tail, issues its first W
// group (the weights do not depend on the previous projection), and only then
// waits for the inputs it reads:
//   * gate_up waits for every o_proj tile (its X is the whole residual row and
//     its row scales are o_proj's sum-of-squares slots);
//   * down split s waits only for the gate_up channel blocks of its k-range;
//   * qkv waits for every down tile.
// Hand-off (MI355X_MICROARCH.md, hand-offs with sc1 loads, row 1): handed-off
// bytes (residual stream, SiLU output, sum-of-squares slots) are stored
// write-through (sc1, 4-byte column pairs) and read with sc1 loads; each
// storing wave drains its stores, and after the workgroup's last barrier one
// lane per counter adds the workgroup's published units (agent-scope atomic).
// One lane of a consumer polls with sc1 loads and s_sleep; its workgroup's
// barrier releases the rest.  No L2 write-back or invalidate anywhere: the
// first version released and acquired at agent scope in every wave and ran
// the decode step 1.65x slower (profiles/README.md section 37).
// Deadlock freedom: the grid is one workgroup per CU (the kernel fits two),
// so every worker is resident -- or becomes so as other tenants' workgroups
// drain -- and each one's tiles of a projection only wait on tiles of earlier
// projections.  (A first version ran each projection as its own block range
// of the grid: consumers dispatched into whatever slots the producer left,
// two to a CU on half the chip.)  Spins are bounded
// (CHAIN_SPIN_TICKS of the 100 MHz real-time counter): a give-up sets the
// error word and the launch completes (wrong output, reported, never a hang).
// The last workgroup to finish re-zeroes the counters for the next launch.
constexpr int CHAIN_PROJ = 4;
constexpr int CHAIN_MAX_SPLITS = 8;
// counters, each on a 128-byte line of its own (a polled line next to
// another counter's adds would bounce between them)
constexpr int CTR_STRIDE = 32;
enum { CTR_O = 0, CTR_D = 1, CTR_FIN = 2, CTR_ERR = 3, CTR_GU = 4, CTR_N = CTR_GU + CHAIN_MAX_SPLITS };
constexpr int CTR_WORDS = CTR_N * CTR_STRIDE;
constexpr unsigned long long CHAIN_SPIN_TICKS = 5000000ull;   // 50 ms

template <bool ACQ>
struct ChainDeps {
  static constexpr bool chained = true;
  // ACQ: the polling wave acquires at agent scope once the count is reached
  // (invalidating its XCD's L2) and the workgroup reads the handed-off bytes
  // with plain, L2-cached loads; !ACQ: every such load is an sc1 load
  static constexpr bool sc1_loads = !ACQ;
  int* wait_ctr;     // counter(s) to wait on (nullptr: none)
  int wait_target;   // units published per counter
  int wait_split;    // one counter per split of this projection's k-range
  int* pub_lds;      // this workgroup's published units per counter (LDS; nullptr: publishes nothing)
  int pub_div;       // units per counter (0: all units to one counter)
  int* err;

  // One lane of the polling wave spins on an sc1 load of the counter; the
  // other waves join it at the barrier (their loads of the handed-off bytes,
  // all sc1, come after it).
  __device__ void wait(int poll_wave, int split) const {
    if (wait_ctr == nullptr) return;
    if ((int)(threadIdx.x >> 6) == poll_wave && (threadIdx.x & 63) == 0) {
      const int* c = wait_ctr + (wait_split ? split * CTR_STRIDE : 0);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < wait_target) {
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > CHAIN_SPIN_TICKS) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    if constexpr (ACQ) {
      if ((int)(threadIdx.x >> 6) == poll_wave) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the invalidate done before the barrier
      }
    }
    __syncthreads();
  }

  // A wave's write-through stores of `unit` are drained; the workgroup's
  // count goes out after the kernel's final barrier (one add per counter).
  __device__ void publish(int unit) const {
    if (pub_lds == nullptr) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) atomicAdd(pub_lds + (pub_div ? unit / pub_div : 0), 1);
  }
};

struct ChainArgs {
  GemmP g[CHAIN_PROJ];          // o_proj, gate_up, down, qkv
  int nblk[CHAIN_PROJ];         // workgroups of each (0: absent)
  int wait_target[CHAIN_PROJ];  // producer units each one waits for (0: no wait)
  int gu_div;                   // gate_up units per down split
  int* ctr;                     // CTR_WORDS ints, zero before the first launch (left zero)
};

template <int a, int b>
constexpr int cmax() { return a > b ? a : b; }

template <int W, bool ACQ>
__global__ void __launch_bounds__(64 * W) decode_chain_kernel(ChainArgs a) {
  using Deps = ChainDeps<ACQ>;
  using L0 = WidekLds<1, 1, W, EPI_RESID>;
  using L1 = WideLds<1, 2, W, EPI_SILU_MUL>;
  using L2 = WideLds<1, 1, W, EPI_RESID>;
  using L3 = WidekLds<1, 1, W, EPI_STORE>;
  constexpr int LB = cmax<cmax<(int)sizeof(L0), (int)sizeof(L1)>(), cmax<(int)sizeof(L2), (int)sizeof(L3)>()>();
  __shared__ __attribute__((aligned(16))) char lds[LB];
  __shared__ int pub[CHAIN_MAX_SPLITS];
  int* c = a.ctr;
  int* err = c + CTR_ERR * CTR_STRIDE;
  const int G = gridDim.x, me = blockIdx.x;
  // one item of projection `role`: its body, then (behind the workgroup
  // barrier every storing wave's drained stores precede) one add per counter
  auto item = [&](int role, int it, auto&& body) {
    if (threadIdx.x < CHAIN_MAX_SPLITS) pub[threadIdx.x] = 0;
    __syncthreads();   // the previous item's LDS reads are done; pub zeroed
    body(it);
    __syncthreads();
    int* pc = nullptr;
    if (role == 0 && a.nblk[1]) pc = c + CTR_O * CTR_STRIDE;
    if (role == 1 && a.nblk[2]) pc = c + CTR_GU * CTR_STRIDE;
    if (role == 2 && a.nblk[3]) pc = c + CTR_D * CTR_STRIDE;
    if (pc != nullptr && threadIdx.x < CHAIN_MAX_SPLITS && pub[threadIdx.x] > 0)
      __hip_atomic_fetch_add(pc + threadIdx.x * CTR_STRIDE, pub[threadIdx.x], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  };
  for (int it = me; it < a.nblk[0]; it += G)
    item(0, it, [&](int i) {
      widek_body<1, 1, W, EPI_RESID, false>(a.g[0], i, *reinterpret_cast<L0*>(lds), XComb{},
                                           Deps{nullptr, 0, 0, a.nblk[1] ? pub : nullptr, 0, err});
    });
  for (int it = me; it < a.nblk[1]; it += G)
    item(1, it, [&](int i) {
      wide_body<1, 2, W, EPI_SILU_MUL>(a.g[1], i, *reinterpret_cast<L1*>(lds),
                                       Deps{a.wait_target[1] ? c + CTR_O * CTR_STRIDE : nullptr,
                                                 a.wait_target[1], 0, a.nblk[2] ? pub : nullptr, a.gu_div, err});
    });
  for (int it = me; it < a.nblk[2]; it += G)
    item(2, it, [&](int i) {
      wide_body<1, 1, W, EPI_RESID>(a.g[2], i, *reinterpret_cast<L2*>(lds),
                                    Deps{a.wait_target[2] ? c + CTR_GU * CTR_STRIDE : nullptr, a.wait_target[2],
                                              1, a.nblk[3] ? pub : nullptr, 0, err});
    });
  for (int it = me; it < a.nblk[3]; it += G)
    item(3, it, [&](int i) {
      widek_body<1, 1, W, EPI_STORE, false>(a.g[3], i, *reinterpret_cast<L3*>(lds), XComb{},
                                           Deps{a.wait_target[3] ? c + CTR_D * CTR_STRIDE : nullptr,
                                                     a.wait_target[3], 0, nullptr, 0, err});
    });
  // the last worker out re-zeroes the counters (every wait is behind it)
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(c + CTR_FIN * CTR_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
      for (int i = 0; i < CTR_N; ++i)
        if (i != CTR_ERR) __hip_atomic_store(c + i * CTR_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Pack W[N][K] (row-major bf16) into the fragment order above.
__global__ void pack_weight_kernel(const bf16_t* __restrict__ w, u32x4_t* __restrict__ wp, int N, int K,
                                   int kmajor) {
  const size_t KB = K >> 6, NTL = N >> 5;
  const size_t total = NTL * KB * 256;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (size_t)gridDim.x * blockDim.x) {
    const int l = q & 63;
    const int j = (q >> 6) & 3;
    const size_t tk = q >> 8;  // t*KB + kb (tile-major) or kb*NTL + t (k-block-major)
    const size_t t = kmajor ? tk % NTL : tk / KB, kb = kmajor ? tk / NTL : tk % KB;
    const size_t row = t * 32 + (l & 31);
    const size_t col = kb * 64 + 32 * (l >> 5) + 8 * j;
    wp[q] = *(const u32x4_t*)(w + row * K + col);
  }
}

// The inverse: packed -> W[N][K] row-major, for prompt-sized GEMMs on the
// library path (a slice keeps only the packed copy; re-streaming it once per
// 128-row chunk of an 8k prompt read the weights 64 times).  deinterleave:
// the packed rows are gate/up interleaved per 32-row block (interleave_gate_up
// in ops/__init__.py); write them back as [gate rows; up rows].
__global__ void unpack_weight_kernel(const u32x4_t* __restrict__ wp, bf16_t* __restrict__ w, int N, int K,
                                     int kmajor, int deinterleave) {
  const size_t KB = K >> 6, NTL = N >> 5;
  const size_t total = NTL * KB * 256;
  const size_t half = (size_t)N >> 1;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (size_t)gridDim.x * blockDim.x) {
    const int l = q & 63;
    const int j = (q >> 6) & 3;
    const size_t tk = q >> 8;
    const size_t t = kmajor ? tk % NTL : tk / KB, kb = kmajor ? tk / NTL : tk % KB;
    size_t row = t * 32 + (l & 31);
    if (deinterleave) {
      const size_t c = row >> 6, within = row & 63;
      row = within < 32 ? c * 32 + within : half + c * 32 + (within - 32);
    }
    const size_t col = kb * 64 + 32 * (l >> 5) + 8 * j;
    *(u32x4_t*)(w + row * K + col) = __builtin_nontemporal_load(wp + q);
  }
}

struct Args {
  const void* wp;
  const void* x;
  void* y;
  int M, K, N, ldx, ldy, S;
  float* scratch;
  int* tickets;
  bool db;
  int kmajor;
  const float* rs_part = nullptr;   // row-norm fusion (wide kernel only)
  int rs_nparts = 0;
  float rs_inv_dim = 0.f;
  float rs_eps = 0.f;
  float* ss_out = nullptr;
  XComb xcomb{};                    // K-split kernel: X from attention split partials (xcomb.o != null)
};

GemmP gemm_p(const Args& a) {
  return GemmP{(const u32x4_t*)a.wp, (const bf16_t*)a.x, (bf16_t*)a.y, a.M, a.K, a.N, a.ldx, a.ldy, a.S, a.scratch,
               a.tickets, a.kmajor, a.rs_part, a.rs_nparts, a.rs_inv_dim, a.rs_eps, a.ss_out};
}

template <int MT, int NT, int KS, int EPI>
hipError_t launch(const Args& a, hipStream_t s) {
  const int groups = (a.N / 32) / NT;
  if (a.db)
    hipLaunchKernelGGL((skinny_gemm_kernel<MT, NT, KS, EPI, true>), dim3(groups * a.S), dim3(64 * KS), 0, s,
                       (const u32x4_t*)a.wp, (const bf16_t*)a.x, (bf16_t*)a.y, a.M, a.K, a.N, a.ldx, a.ldy, a.S,
                       a.scratch, a.tickets, a.kmajor);
  else
    hipLaunchKernelGGL((skinny_gemm_kernel<MT, NT, KS, EPI, false>), dim3(groups * a.S), dim3(64 * KS), 0, s,
                       (const u32x4_t*)a.wp, (const bf16_t*)a.x, (bf16_t*)a.y, a.M, a.K, a.N, a.ldx, a.ldy, a.S,
                       a.scratch, a.tickets, a.kmajor);
  return hipGetLastError();
}

// Largest KS (waves per workgroup) whose register budget (512 / waves per
// SIMD) holds the tile without spilling (-Rpass-analysis=kernel-resource-usage:
// MT,NT = 1,1: ~140 VGPR+AGPR with U=4 groups; 1,2 and 2,1: ~140-160; 2,2:
// ~200; 4,1: ~260; 4,2: >256 -> KS <= 4).
constexpr int ks_max(int mt, int nt) { return (mt == 4 && nt == 2) ? 4 : 8; }

template <int MT, int NT, int EPI>
hipError_t launch_ks(int ks, const Args& a, hipStream_t s) {
  constexpr int KSM = ks_max(MT, NT);
  if (ks > KSM) ks = KSM;
  if (a.db && ks > 4) ks = 4;   // two register buffers: 8 waves per workgroup would spill
  switch (ks) {
    case 1: return launch<MT, NT, 1, EPI>(a, s);
    case 2: return launch<MT, NT, 2, EPI>(a, s);
    case 4: return launch<MT, NT, 4, EPI>(a, s);
    case 8:
      if constexpr (KSM >= 8) return launch<MT, NT, 8, EPI>(a, s);
      break;
  }
  return hipErrorInvalidValue;
}

template <int NT, int EPI>
hipError_t launch_mt(int mt, int ks, const Args& a, hipStream_t s) {
  switch (mt) {
    case 1: return launch_ks<1, NT, EPI>(ks, a, s);
    case 2: return launch_ks<2, NT, EPI>(ks, a, s);
    case 4: return launch_ks<4, NT, EPI>(ks, a, s);
  }
  return hipErrorInvalidValue;
}

template <int MT, int NT, int EPI>
hipError_t launch_wide(int wv, const Args& a, hipStream_t s) {
  const int blocks = (a.N / 32) / NT / wv * a.S;
#define MIVGPU_LAUNCH_WIDE(WV)                                                                                \
  hipLaunchKernelGGL((skinny_wide_kernel<MT, NT, WV, EPI>), dim3(blocks), dim3(64 * WV), 0, s, gemm_p(a))
  switch (wv) {
    case 1: MIVGPU_LAUNCH_WIDE(1); break;
    case 2: MIVGPU_LAUNCH_WIDE(2); break;
    case 4: MIVGPU_LAUNCH_WIDE(4); break;
    default: return hipErrorInvalidValue;
  }
#undef MIVGPU_LAUNCH_WIDE
  return hipGetLastError();
}

template <int NT, int EPI>
hipError_t launch_wide_mt(int mt, int wv, const Args& a, hipStream_t s) {
  switch (mt) {
    case 1: return launch_wide<1, NT, EPI>(wv, a, s);
    case 2: return launch_wide<2, NT, EPI>(wv, a, s);
    case 4: return launch_wide<4, NT, EPI>(wv, a, s);
  }
  return hipErrorInvalidValue;
}

template <int NT>
hipError_t launch_wide_resid(int mt, int wv, const Args& a, hipStream_t s) {
  switch (mt) {
    case 1: return launch_wide<1, NT, EPI_RESID>(wv, a, s);
    case 2: return launch_wide<2, NT, EPI_RESID>(wv, a, s);
  }
  return hipErrorInvalidValue;
}

// k-blocks per wave per group of the K-split kernel (MIVGPU_WIDEK_U, A/B): 2 or 4
int widek_u() {
  static const int u = [] {
    const char* e = getenv("MIVGPU_WIDEK_U");
    return e && atoi(e) == 4 ? 4 : 2;
  }();
  return u;
}

template <int MT, int NT, int EPI>
hipError_t launch_widek(int kw, const Args& a, hipStream_t s) {
  const int blocks = (a.N / 32) / NT * a.S;
#define MIVGPU_LAUNCH_WIDEK(KW, CC)                                                                                \
  hipLaunchKernelGGL((skinny_widek_kernel<MT, NT, KW, EPI, CC>), dim3(blocks), dim3(64 * KW), 0, s, gemm_p(a), a.xcomb)
  const bool comb = a.xcomb.o != nullptr;
  if constexpr (MT == 1 && NT == 1) {
    if (comb) {
      switch (kw) {
        case 2: MIVGPU_LAUNCH_WIDEK(2, true); break;
        case 4: MIVGPU_LAUNCH_WIDEK(4, true); break;
        case 8: MIVGPU_LAUNCH_WIDEK(8, true); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
  } else if (comb) {
    return hipErrorInvalidValue;
  }
  static const bool dmax = [] {
    const char* e = getenv("MIVGPU_WIDEK_DMAX");
    return e && *e == '1';
  }();
  if (dmax && kw == 4) {
    hipLaunchKernelGGL((skinny_widek_kernel<MT, NT, 4, EPI, false, true>), dim3(blocks), dim3(256), 0, s, gemm_p(a),
                       a.xcomb);
    return hipGetLastError();
  }
  // MIVGPU_WIDEK_U=4 (A/B): four k-blocks per wave per group instead of two --
  // twice the weight bytes in flight per workgroup (16 KB per wave), one X
  // tile of 16 k-blocks per group (two 66 KB buffers: one M-tile, 4 k-waves)
  if constexpr (MT == 1 && NT == 1) {
    if (kw == 4 && widek_u() == 4) {
      hipLaunchKernelGGL((skinny_widek_kernel<1, 1, 4, EPI, false, false, 4>), dim3(blocks), dim3(256), 0, s,
                         gemm_p(a), a.xcomb);
      return hipGetLastError();
    }
  }
  switch (kw) {
    case 2: MIVGPU_LAUNCH_WIDEK(2, false); break;
    case 4: MIVGPU_LAUNCH_WIDEK(4, false); break;
    case 8:
      // 8 k-waves: two 66 KB X buffers, one M-tile only (LDS)
      if constexpr (MT == 1) {
        MIVGPU_LAUNCH_WIDEK(8, false);
        break;
      }
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
#undef MIVGPU_LAUNCH_WIDEK
  return hipGetLastError();
}

int mt_of(int M) { return M <= 32 ? 1 : (M <= 64 ? 2 : 4); }

// Partition-size plan switch: the "slice" plans (no inter-workgroup split,
// fatter workgroups) apply at <= MIVGPU_SLICE_PLAN_CUS visible CUs (default 96).
bool slice_plan(int cus) {
  static const int limit = [] {
    const char* e = getenv("MIVGPU_SLICE_PLAN_CUS");
    return e && *e ? atoi(e) : 96;
  }();
  return cus <= limit;
}

// Half-GPU partitions (97-160 CUs) get their own wide-kernel wave counts
// (MIVGPU_WIDE_MID_PLAN=0 restores the whole-chip ones for A/B runs).
bool mid_plan(int cus, bool slice) {
  static const int on = [] {
    const char* e = getenv("MIVGPU_WIDE_MID_PLAN");
    return e && *e ? atoi(e) : 1;
  }();
  return on && !slice && cus <= 160;
}

}  // namespace
extern "C" int mivgpu_ops_visible_cus();   // model_ops.hip
namespace {

// Default plan, from bench/gemm.py --sweep on MI355X (profiles/gemm):
//  * nt = 2 (X fragments reused twice) once there are >= 384 tile pairs;
//  * many groups (gate_up, lm_head): single-wave workgroups, no split (12
//    independent waves per CU hide each other's prologue/epilogue);
//  * few groups (qkv 192, o/down 128): 2 waves per workgroup, and S = 2 when
//    <= 128 groups so that more CUs stream.
//  * a CU partition of <= 96 CUs (a vGPU slice): nt = 2, 2 waves per
//    workgroup, no inter-workgroup split (down 68 -> 57 us, o_proj 27 -> 25 us
//    at 64 CUs vs hipBLASLt; splitting only adds combine traffic there).
void plan(int M, int K, int N, int epi, int* nt, int* ks, int* S) {
  static const int cus = mivgpu_ops_visible_cus();
  const int mt = mt_of(M);
  const bool slice = slice_plan(cus);
  if (epi == EPI_SILU_MUL) *nt = 2;
  if (*nt != 1 && *nt != 2) *nt = (mt < 4 && ((N / 64) >= 384 || (slice && (N / 64) >= 32))) ? 2 : 1;
  const int groups = (N / 32) / *nt, KB = K / 64;
  if (*ks <= 0) *ks = slice ? 2 : (groups >= 384 ? 1 : 2);
  if (*S <= 0) *S = (!slice && groups <= 128 && KB >= 4 * *ks) ? 2 : 1;
}

// Double-buffered schedule: MIVGPU_SKINNY_DB=0/1 forces it (A/B runs);
// default off until measured per partition size.
bool use_db() {
  static const int v = [] {
    const char* e = getenv("MIVGPU_SKINNY_DB");
    return e && *e ? atoi(e) : -1;
  }();
  return v > 0;
}

// Packed-W layout: MIVGPU_SKINNY_KMAJOR=0/1 (read once per process; packing
// and the GEMM must agree, so both read it here).
bool use_kmajor() {
  static const int v = [] {
    const char* e = getenv("MIVGPU_SKINNY_KMAJOR");
    return e && *e ? atoi(e) : -1;
  }();
  return v > 0;
}

constexpr int unroll_wide_host(int nt) { return nt >= 4 ? 1 : (nt == 2 ? 2 : 4); }

// Wide plan (bench/gemm.py --sweep at 64 and 256 CUs, profiles/gemm_wide_*):
//  * one tile per wave (X shared by the workgroup's waves, not by a wave's
//    tiles), except SiLU*up, which pairs a gate with an up tile;
//  * a CU partition (<= 96 CUs): no split, 4 waves per workgroup when there
//    are >= 16 wave-groups per CU (lm_head: 422 vs 491 us at 64 CUs) or more
//    than 32 rows (2-wave workgroups of 2-4 M-tiles spill), otherwise 2 or 4
//    by CU balance (below);
//  * the whole chip: S = 4 with 2 waves when <= 128 wave-groups (o_proj,
//    down), else no split with 2 waves.
// Values > 0 are requests; false when the wide kernel cannot run them (the
// caller falls back to the classic kernel).
bool plan_wide(int M, int K, int N, int epi, int* nt, int* wv, int* S) {
  static const int cus = mivgpu_ops_visible_cus();
  const bool slice = slice_plan(cus);
  const int ntiles = N / 32, KB = K / 64;
  if (epi == EPI_SILU_MUL) {
    if (*nt > 0 && *nt != 2) return false;
    *nt = 2;
  }
  if (*nt <= 0) *nt = 1;
  if (*nt != 1 && *nt != 2) return false;
  const int vgroups = ntiles / *nt;
  const bool auto_s = *S <= 0;
  if (auto_s) *S = (!slice && vgroups <= 128) ? 4 : 1;
  if (M > 64) {
    // Prompt rows (serving prefill chunks of up to 128), swept by
    // scripts/probe/wide_m128_sweep.py (profiles/round2/gemm_prefill_rows/):
    //  * gate_up + SiLU: 2 waves, no split -- 64 CUs 158 vs 177 us at 128
    //    rows, 256 CUs 77.5 vs 91.5;
    //  * stores split K: inside a partition S = 2 for N <= 4096 (down 105 vs
    //    162 us, o_proj 54 vs 59), on the chip S = 4 up to 192 wave-groups
    //    (qkv 49.9 vs 59.2; down / o_proj already split 4).
    if (auto_s) {
      if (epi == EPI_SILU_MUL) *S = 1;
      else if (slice) *S = ntiles <= 128 ? 2 : 1;
      else if (cus > 160) *S = vgroups <= 192 ? 4 : 1;
      // 97-160 CUs keep the split chosen above (measured: the chip's rule cost
      // the 128-CU prefill 0.8 ms)
    }
    if (*wv <= 0) *wv = epi == EPI_SILU_MUL ? 2 : 4;
  }
  if (*wv <= 0) {
    // > 32 rows: 4 waves (2-wave workgroups of 2-4 M-tiles spill registers)
    *wv = (M > 32 || (slice && vgroups >= 16 * cus)) ? 4 : 2;
    if (M <= 32 && slice && vgroups < 16 * cus) {
      // Slice partitions, bench/gemm.py --sweep (profiles/sweeps/): keep the
      // workgroup count a multiple of the CU count where that is possible.
      //  * <= 48 CUs (8 slices): 4 waves when vgroups/4 fills every CU equally
      //    (o_proj 25.3 vs 28.0 us, gate_up 121 vs 132, down 69 vs 79 at 32
      //    CUs), else 2 (qkv: 48 workgroups on 32 CUs lose to 96);
      //  * 49-96 CUs (4 slices): 2 waves when vgroups/2 fills the CUs equally
      //    (o_proj, gate_up, down at 64 CUs), else 4 (qkv 25.9 vs 29.4 us).
      if (cus <= 48) *wv = (vgroups % 4 == 0 && (vgroups / 4) % cus == 0) ? 4 : 2;
      else *wv = (vgroups % 2 == 0 && (vgroups / 2) % cus == 0) ? 2 : 4;
    }
    if (M <= 32 && mid_plan(cus, slice)) {
      // 97-160 CUs (a half-GPU slice), bench/gemm.py --sweep at 128 CUs
      // (profiles/cu128/sweep_cu128.json): lm_head 4 waves 255 vs 287 us,
      // down (S = 4) 4 waves 29.4 vs 32.5, gate_up+SiLU 1 wave 47.7 vs 53.0.
      if (vgroups >= 16 * cus || (vgroups <= 128 && *S > 1)) *wv = 4;
      else if (epi == EPI_SILU_MUL) *wv = 1;
    }
    while (*wv > 1 && ntiles % (*nt * *wv)) *wv /= 2;
  }
  if ((*wv != 1 && *wv != 2 && *wv != 4) || ntiles % (*nt * *wv)) return false;
  const int U = unroll_wide_host(*nt);
  if (auto_s && *S > 1 && (KB % (*S * U) || KB / *S < U)) *S = 1;   // auto split that does not fit: none
  return *S >= 1 && KB % (*S * U) == 0 && KB / *S >= U;
}

// K-split wide plan (variant 3): nt = 1 (nt = 2 for SiLU*up: a gate/up tile
// pair), ks = k-waves per workgroup (2 or 4, default 4), S = inter-workgroup
// split (default 1).  Stores (optionally row scaled), SiLU*up, or the residual
// update (planned as stores), M <= 64.
// False when it cannot run these values.
bool plan_widek(int M, int K, int N, int epi, int* nt, int* kw, int* S) {
  static const int cus = mivgpu_ops_visible_cus();
  if ((epi != EPI_STORE && epi != EPI_SILU_MUL) || M > 64) return false;
  const int want = epi == EPI_SILU_MUL ? 2 : 1;   // SiLU*up: a gate/up tile pair per workgroup
  if (*nt > 0 && *nt != want) return false;
  *nt = want;
  if ((N / 32) % want) return false;
  if (*kw <= 0) {
    // MIVGPU_WIDEK_KW: k-waves per workgroup for A/B runs (8: one M-tile only;
    // measured whole GPU, qkv + o_proj: batch 32 4.583 vs 4.563 ms, batch 1
    // 3.415 vs 3.346 -- twice the waves per CU do not stream faster)
    static const int env = [] {
      const char* e = getenv("MIVGPU_WIDEK_KW");
      return e && *e ? atoi(e) : 0;
    }();
    *kw = (env == 8 && M <= 32) || env == 2 || env == 4 ? env : 4;
  }
  if (*kw != 2 && *kw != 4 && !(*kw == 8 && M <= 32)) return false;
  const int KB = K / 64, GK = *kw * ((*kw == 4 && M <= 32 && epi == EPI_STORE) ? widek_u() : 2);
  // no inter-workgroup split by default: measured on the whole chip (bench/gemm.py,
  // profiles/round3/widek_gemm.json) S = 2 costs qkv 13.6 -> 19.1 us and o_proj
  // 12.2 -> 15.6 us at 32 rows (the atomics + last-arriver tail)
  (void)cus;
  if (*S <= 0) *S = 1;
  return *S >= 1 && KB % (*S * GK) == 0 && KB / *S >= GK;
}

// Kernel choice: 1 = classic, 2 = wide; 0 = auto = wide where it can run
// (MIVGPU_SKINNY_WIDE=0/1 forces one for A/B runs).  An infeasible wide request
// falls back to classic.  Resolves nt/ks/S for the kernel chosen.
int resolve(int M, int K, int N, int epi, int* nt, int* ks, int* S, int variant) {
  if (variant == 0) {
    static const int env = [] {
      const char* e = getenv("MIVGPU_SKINNY_WIDE");
      return e && *e ? atoi(e) : -1;
    }();
    // wide unless forced off.  Prefill row counts (96-128, 4 M-tiles) too
    // (profiles/round2/gemm_prefill_rows/): at 64 CUs wide vs classic is
    // gate_up 178 vs 355 us, down 162 vs 226, qkv 60 vs 119, o_proj 59 vs 85;
    // on the whole chip gate_up 93 vs 126 and down 72 vs 74 (qkv / o_proj,
    // where classic is ahead, run on hipBLASLt there)
    variant = env >= 0 ? (env ? 2 : 1) : 2;
  }
  if (variant == 3) {
    int a = *nt, b = *ks, c = *S;
    if (plan_widek(M, K, N, epi, &a, &b, &c)) {
      *nt = a, *ks = b, *S = c;
      return 3;
    }
    variant = 2;   // infeasible: the wide kernel's plan
  }
  if (variant == 2) {
    int a = *nt, b = *ks, c = *S;
    if (plan_wide(M, K, N, epi, &a, &b, &c)) {
      *nt = a, *ks = b, *S = c;
      return 2;
    }
  }
  plan(M, K, N, epi, nt, ks, S);
  return 1;
}

}  // namespace

extern "C" {

// Largest M handled in one pass (4 M-tiles of 32 rows per wave).
int mivgpu_skinny_max_m() { return 128; }

// Resolve the launch plan (0 = auto for nt/ks/S) and the scratch it needs:
// *scratch_floats fp32 elements and *tickets ints, both zero-initialised by the
// caller once (the kernel leaves them zeroed).
int mivgpu_skinny_plan(int M, int K, int N, int epi, int* nt, int* ks, int* S, long long* scratch_floats,
                       int* tickets, int* variant) {
  if (M <= 0 || M > 128 || K <= 0 || (K & 63) || N <= 0 || (N & 31)) return (int)hipErrorInvalidValue;
  *variant = resolve(M, K, N, epi, nt, ks, S, *variant);
  const int groups = (N / 32) / *nt;
  *scratch_floats = *S > 1 ? (long long)groups * (mt_of(M) * 32) * (*nt * 32) : 0;
  *tickets = *S > 1 ? groups : 0;
  return 0;
}

// Packed buffer size in bytes for W[N][K] (same as the unpacked size).
long long mivgpu_packed_weight_bytes(int N, int K) { return (long long)N * K * 2; }

int mivgpu_pack_weight(const void* w, void* wp, int N, int K, hipStream_t s) {
  if (N <= 0 || K <= 0 || (N & 31) || (K & 63)) return (int)hipErrorInvalidValue;
  const size_t total = (size_t)(N >> 5) * (K >> 6) * 256;
  const int blocks = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(pack_weight_kernel, dim3(blocks), dim3(256), 0, s, (const bf16_t*)w, (u32x4_t*)wp, N, K,
                     use_kmajor() ? 1 : 0);
  return (int)hipGetLastError();
}

int mivgpu_unpack_weight(const void* wp, void* w, int N, int K, int deinterleave, hipStream_t s) {
  if (N <= 0 || K <= 0 || (N & 31) || (K & 63) || (deinterleave && (N & 63))) return (int)hipErrorInvalidValue;
  const size_t total = (size_t)(N >> 5) * (K >> 6) * 256;
  const int blocks = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(unpack_weight_kernel, dim3(blocks), dim3(256), 0, s, (const u32x4_t*)wp, (bf16_t*)w, N, K,
                     use_kmajor() ? 1 : 0, deinterleave);
  return (int)hipGetLastError();
}

int mivgpu_skinny_gemm_norm(const void* wp, const void* x, void* y, int M, int K, int N, int ldx, int ldy, int epi,
                            int nt, int ks, int S, int variant, float* scratch, int* tickets, const float* rs_part,
                            int rs_nparts, float rs_inv_dim, float rs_eps, float* ss_out, hipStream_t s);

// epi: 0 = store Y[M][N] (ldy >= N);  1 = SiLU(gate)*up -> Y[M][N/2] for an
// interleaved gate/up weight.  variant: 0 auto, 1 classic, 2 wide workgroups
// (ks = waves per workgroup there).  nt/ks/S: 0 = auto (see mivgpu_skinny_plan);
// scratch/tickets must hold what mivgpu_skinny_plan reports for the same
// arguments when S > 1.
int mivgpu_skinny_gemm(const void* wp, const void* x, void* y, int M, int K, int N, int ldx, int ldy, int epi,
                       int nt, int ks, int S, int variant, float* scratch, int* tickets, hipStream_t s) {
  if (M <= 0 || M > 128 || K <= 0 || (K & 63) || N <= 0 || (N & 31) || ldx < K || (ldx & 7) || (ldy & 7))
    return (int)hipErrorInvalidValue;
  if (epi != EPI_STORE && epi != EPI_SILU_MUL) return (int)hipErrorInvalidValue;
  return mivgpu_skinny_gemm_norm(wp, x, y, M, K, N, ldx, ldy, epi, nt, ks, S, variant, scratch, tickets, nullptr, 0,
                                 0.f, 0.f, nullptr, s);
}

// mivgpu_skinny_gemm plus the row-norm fusion of the wide kernel (see
// EPI_RESID / SS_ROWS above): epi 2 = residual update with sum-of-squares
// slots ss_out[(N/32/nt) * 128]; rs_part != nullptr = row scales from rs_nparts
// such slots (rs_inv_dim = 1/normalised dim).  Either requires the wide kernel
// (hipErrorInvalidValue when the plan resolves to the classic one).
static int skinny_gemm_norm_impl(const void* wp, const void* x, void* y, int M, int K, int N, int ldx, int ldy,
                                 int epi, int nt, int ks, int S, int variant, float* scratch, int* tickets,
                                 const float* rs_part, int rs_nparts, float rs_inv_dim, float rs_eps, float* ss_out,
                                 const XComb& xcomb, hipStream_t s);

int mivgpu_skinny_gemm_norm(const void* wp, const void* x, void* y, int M, int K, int N, int ldx, int ldy, int epi,
                            int nt, int ks, int S, int variant, float* scratch, int* tickets, const float* rs_part,
                            int rs_nparts, float rs_inv_dim, float rs_eps, float* ss_out, hipStream_t s) {
  return skinny_gemm_norm_impl(wp, x, y, M, K, N, ldx, ldy, epi, nt, ks, S, variant, scratch, tickets, rs_part,
                               rs_nparts, rs_inv_dim, rs_eps, ss_out, XComb{}, s);
}

// mivgpu_skinny_gemm_norm on the K-split kernel with X taken from decode
// attention split partials (o_part [B][Hq][nsplit][128], ml_part
// [B][Hq][nsplit][2], as mivgpu_decode_attention_fused leaves them with
// defer_combine): X[0][h*128 + d] is the split combine.  K = Hq * 128, M = 1,
// nsplit <= 8; hipErrorInvalidValue when the plan is not the K-split kernel.
int mivgpu_skinny_gemm_norm_xcomb(const void* wp, const float* o_part, const float* ml_part, const int* seqlens,
                                  int nsplit, int split_keys, int max_ctx, int hq, void* y, int M, int K, int N,
                                  int ldy, int epi, int ks, int S, float* scratch, int* tickets,
                                  const float* rs_part, int rs_nparts, float rs_inv_dim, float rs_eps, float* ss_out,
                                  hipStream_t s) {
  if (!o_part || !ml_part || !seqlens || nsplit < 1 || nsplit > XC_MAXS || split_keys <= 0 || max_ctx <= 0 ||
      hq <= 0 || K != hq * 128 || M != 1)
    return (int)hipErrorInvalidValue;
  int a = 0, b = ks, c = S;
  if (!plan_widek(M, K, N, epi == EPI_RESID ? EPI_STORE : epi, &a, &b, &c) || a != 1) return (int)hipErrorInvalidValue;
  // the combined row: XC_NCH 8-column chunks per thread, in the X buffers
  // (2 * 32 * (GK * 64 + 8) bf16 >= K + 8)
  if (K > XC_NCH * 8 * 64 * b || K + 8 > 2 * 32 * (b * 2 * 64 + 8)) return (int)hipErrorInvalidValue;
  const XComb xc{o_part, ml_part, seqlens, nsplit, split_keys, max_ctx, hq};
  return skinny_gemm_norm_impl(wp, o_part, y, M, K, N, K, ldy, epi, 1, b, c, 3, scratch, tickets, rs_part, rs_nparts,
                               rs_inv_dim, rs_eps, ss_out, xc, s);
}

static int skinny_gemm_norm_impl(const void* wp, const void* x, void* y, int M, int K, int N, int ldx, int ldy,
                                 int epi, int nt, int ks, int S, int variant, float* scratch, int* tickets,
                                 const float* rs_part, int rs_nparts, float rs_inv_dim, float rs_eps, float* ss_out,
                                 const XComb& xcomb, hipStream_t s) {
  if (M <= 0 || M > 128 || K <= 0 || (K & 63) || N <= 0 || (N & 31) || ldx < K || (ldx & 7) || (ldy & 7))
    return (int)hipErrorInvalidValue;
  if (epi != EPI_STORE && epi != EPI_SILU_MUL && epi != EPI_RESID) return (int)hipErrorInvalidValue;
  const bool fused = rs_part != nullptr || epi == EPI_RESID;
  if (epi == EPI_RESID && ss_out == nullptr) return (int)hipErrorInvalidValue;
  if (rs_part != nullptr && rs_nparts <= 0) return (int)hipErrorInvalidValue;
  // the row-norm fusion runs on the wide kernel or, when asked for, the K-split one
  const int v = resolve(M, K, N, epi == EPI_RESID ? EPI_STORE : epi, &nt, &ks, &S,
                        fused ? (variant == 3 ? 3 : 2) : variant);
  if (v == 3) {
    if ((epi == EPI_SILU_MUL ? ldy < N / 2 : ldy < N) || (S > 1 && (scratch == nullptr || tickets == nullptr)))
      return (int)hipErrorInvalidValue;
    Args a{wp, x, y, M, K, N, ldx, ldy, S, scratch, tickets, false, use_kmajor() ? 1 : 0};
    a.rs_part = rs_part;
    a.rs_nparts = rs_nparts;
    a.rs_inv_dim = rs_inv_dim;
    a.rs_eps = rs_eps;
    a.ss_out = ss_out;
    a.xcomb = xcomb;
    const int mt = mt_of(M);
    if (rs_part != nullptr && (epi == EPI_RESID || rs_nparts > 64 * ks * RS_LMAX / (mt * 8)))
      return (int)hipErrorInvalidValue;
    if (xcomb.o != nullptr && (mt != 1 || nt != 1)) return (int)hipErrorInvalidValue;
    if (epi == EPI_RESID)
      return (int)(mt == 1 ? launch_widek<1, 1, EPI_RESID>(ks, a, s) : launch_widek<2, 1, EPI_RESID>(ks, a, s));
    if (epi == EPI_SILU_MUL)
      return (int)(mt == 1 ? launch_widek<1, 2, EPI_SILU_MUL>(ks, a, s) : launch_widek<2, 2, EPI_SILU_MUL>(ks, a, s));
    return (int)(mt == 1 ? launch_widek<1, 1, EPI_STORE>(ks, a, s) : launch_widek<2, 1, EPI_STORE>(ks, a, s));
  }
  if (xcomb.o != nullptr) return (int)hipErrorInvalidValue;   // X from partials: the K-split kernel only
  if (v == 2) {
    if (epi == EPI_SILU_MUL && ldy < N / 2) return (int)hipErrorInvalidValue;
    if (epi != EPI_SILU_MUL && ldy < N) return (int)hipErrorInvalidValue;
    if (S > 1 && (scratch == nullptr || tickets == nullptr)) return (int)hipErrorInvalidValue;
    Args a{wp, x, y, M, K, N, ldx, ldy, S, scratch, tickets, false, use_kmajor() ? 1 : 0};
    a.rs_part = rs_part;
    a.rs_nparts = rs_nparts;
    a.rs_inv_dim = rs_inv_dim;
    a.rs_eps = rs_eps;
    a.ss_out = ss_out;
    const int mt = mt_of(M);
    // rs_issue reads RS_LMAX slots per thread in one batch: a plan with too few
    // waves for the producer's slot count (the 97-160-CU gate_up plan has one
    // wave, 64 slots, after a 128-slot down projection) gets more waves
    while (rs_part != nullptr && rs_nparts > 64 * ks * RS_LMAX / (mt * 8) && ks < 4 &&
           (N / 32) % (nt * ks * 2) == 0)
      ks *= 2;
    // the residual epilogue takes no row scale
    if (rs_part != nullptr && (epi == EPI_RESID || rs_nparts > 64 * ks * RS_LMAX / (mt * 8)))
      return (int)hipErrorInvalidValue;
    if (epi == EPI_RESID && mt > 2) return (int)hipErrorInvalidValue;   // LDS: residual tiles of <= 64 rows
    hipError_t e;
    if (epi == EPI_SILU_MUL)
      e = launch_wide_mt<2, EPI_SILU_MUL>(mt, ks, a, s);
    else if (epi == EPI_RESID)
      e = nt == 2 ? launch_wide_resid<2>(mt, ks, a, s) : launch_wide_resid<1>(mt, ks, a, s);
    else if (nt == 2)
      e = launch_wide_mt<2, EPI_STORE>(mt, ks, a, s);
    else
      e = launch_wide_mt<1, EPI_STORE>(mt, ks, a, s);
    return (int)e;
  }
  if (fused) return (int)hipErrorInvalidValue;   // the classic kernel has no row-norm fusion
  if ((N / 32) % nt || S < 1 || S > K / 64) return (int)hipErrorInvalidValue;
  if (epi == EPI_STORE && ldy < N) return (int)hipErrorInvalidValue;
  if (epi == EPI_SILU_MUL && ldy < N / 2) return (int)hipErrorInvalidValue;
  if (S > 1 && (scratch == nullptr || tickets == nullptr)) return (int)hipErrorInvalidValue;
  if (ks != 1 && ks != 2 && ks != 4 && ks != 8) return (int)hipErrorInvalidValue;
  const Args a{wp, x, y, M, K, N, ldx, ldy, S, scratch, tickets, use_db(), use_kmajor() ? 1 : 0};
  const int mt = mt_of(M);
  hipError_t e;
  if (epi == EPI_SILU_MUL)
    e = launch_mt<2, EPI_SILU_MUL>(mt, ks, a, s);
  else if (nt == 2)
    e = launch_mt<2, EPI_STORE>(mt, ks, a, s);
  else
    e = launch_mt<1, EPI_STORE>(mt, ks, a, s);
  return (int)e;
}


// ---------------------------------------------------------------- chain --
// One projection of mivgpu_decode_chain (layout shared with ops/__init__.py).
struct MivgpuChainGemm {
  const void* wp;
  const void* x;
  void* y;
  int M, K, N, ldx, ldy, S;
  float* scratch;
  int* tickets;
  const float* rs_part;
  int rs_nparts;
  float rs_inv_dim, rs_eps;
  float* ss_out;
};

int mivgpu_chain_counter_words() { return CTR_WORDS; }
int mivgpu_chain_err_word() { return CTR_ERR * CTR_STRIDE; }

// sizeof and field offsets of MivgpuChainGemm (the ctypes mirror is checked
// against them): size, wp, x, y, M, S, scratch, tickets, rs_part, rs_nparts,
// rs_eps, ss_out.
void mivgpu_chain_gemm_layout(long long* out) {
  const long long v[] = {(long long)sizeof(MivgpuChainGemm), (long long)offsetof(MivgpuChainGemm, wp),
                         (long long)offsetof(MivgpuChainGemm, x), (long long)offsetof(MivgpuChainGemm, y),
                         (long long)offsetof(MivgpuChainGemm, M), (long long)offsetof(MivgpuChainGemm, S),
                         (long long)offsetof(MivgpuChainGemm, scratch), (long long)offsetof(MivgpuChainGemm, tickets),
                         (long long)offsetof(MivgpuChainGemm, rs_part), (long long)offsetof(MivgpuChainGemm, rs_nparts),
                         (long long)offsetof(MivgpuChainGemm, rs_eps), (long long)offsetof(MivgpuChainGemm, ss_out)};
  for (int i = 0; i < (int)(sizeof(v) / sizeof(v[0])); ++i) out[i] = v[i];
}

// Plan check of one chained projection; blocks of its range, or -1.
static int chain_blocks(int role, int W, const MivgpuChainGemm& g) {
  if (g.wp == nullptr) return 0;
  if (g.M <= 0 || g.M > 32 || g.K <= 0 || (g.K & 63) || g.N <= 0 || (g.N & 31) || g.ldx < g.K || (g.ldx & 7) ||
      (g.ldy & 7) || g.x == nullptr || g.y == nullptr)
    return -1;
  const int rs_max = 64 * W * RS_LMAX / 8;   // rs_issue's slots per batch at MT = 1
  int nt = 0, w = W, S = g.S;
  switch (role) {
    case 0:   // o_proj: K-split kernel, residual update + slots
      if (g.ss_out == nullptr || g.rs_part != nullptr || g.ldy < g.N || S != 1) return -1;
      return plan_widek(g.M, g.K, g.N, EPI_STORE, &nt, &w, &S) && w == W ? g.N / 32 : -1;
    case 1:   // gate_up: wide kernel, SiLU*up, row scales
      if (g.ss_out != nullptr || S != 1 || g.ldy < g.N / 2 || (g.rs_part && g.rs_nparts > rs_max)) return -1;
      nt = 2;
      return plan_wide(g.M, g.K, g.N, EPI_SILU_MUL, &nt, &w, &S) && w == W && nt == 2 ? g.N / 32 / 2 / W : -1;
    case 2:   // down: wide kernel, residual update + slots, split S
      if (g.ss_out == nullptr || g.rs_part != nullptr || g.ldy < g.N || S < 1 || S > CHAIN_MAX_SPLITS) return -1;
      if (S > 1 && (g.scratch == nullptr || g.tickets == nullptr)) return -1;
      nt = 1;
      return plan_wide(g.M, g.K, g.N, EPI_STORE, &nt, &w, &S) && w == W && nt == 1 ? g.N / 32 / W * S : -1;
    case 3:   // qkv: K-split kernel, stores, row scales
      if (g.ss_out != nullptr || S != 1 || g.ldy < g.N || (g.rs_part && g.rs_nparts > rs_max)) return -1;
      return plan_widek(g.M, g.K, g.N, EPI_STORE, &nt, &w, &S) && w == W ? g.N / 32 : -1;
  }
  return -1;
}

// One launch of up to four decode projections (o_proj, gate_up, down, qkv;
// wp == nullptr: absent) on W-wave workgroups (2 or 4).  ctr:
// mivgpu_chain_counter_words() ints, zero before the first launch and left
// zero by every launch except word mivgpu_chain_err_word(), the give-up flag
// (nonzero: a wait timed out and the output is wrong).  Consecutive projections must chain: gate_up
// reads o_proj's output and slots, down gate_up's, qkv down's.
int mivgpu_decode_chain(const MivgpuChainGemm* g, int W, int* ctr, hipStream_t s) {
  if (g == nullptr || ctr == nullptr || (W != 2 && W != 4)) return (int)hipErrorInvalidValue;
  ChainArgs a{};
  for (int r = 0; r < CHAIN_PROJ; ++r) {
    const int nb = chain_blocks(r, W, g[r]);
    if (nb < 0) return (int)hipErrorInvalidValue;
    a.nblk[r] = nb;
    const MivgpuChainGemm& q = g[r];
    a.g[r] = GemmP{(const u32x4_t*)q.wp, (const bf16_t*)q.x, (bf16_t*)q.y, q.M, q.K, q.N, q.ldx, q.ldy,
                   q.S > 0 ? q.S : 1, q.scratch, q.tickets, use_kmajor() ? 1 : 0, q.rs_part, q.rs_nparts,
                   q.rs_inv_dim, q.rs_eps, q.ss_out};
  }
  // producer -> consumer: each must read what the previous one wrote
  if (a.nblk[0] && a.nblk[1] && (g[1].x != g[0].y || g[1].rs_part != g[0].ss_out || g[1].K != g[0].N)) return (int)hipErrorInvalidValue;
  if (a.nblk[1] && a.nblk[2] && (g[2].x != g[1].y || g[2].K != g[1].N / 2)) return (int)hipErrorInvalidValue;
  if (a.nblk[2] && a.nblk[3] && (g[3].x != g[2].y || g[3].rs_part != g[2].ss_out || g[3].K != g[2].N)) return (int)hipErrorInvalidValue;
  if (a.nblk[1] && !a.nblk[0] && a.nblk[2] + a.nblk[3] == 0) return (int)hipErrorInvalidValue;   // use the plain launch
  a.wait_target[1] = a.nblk[0] && a.nblk[1] ? g[0].N / 32 : 0;
  if (a.nblk[1] && a.nblk[2]) {
    // gate_up vgroup v writes act channels [32v, 32v + 32) = down k-block v / 2
    const int kb_per_split = (g[2].K / 64) / a.g[2].S;
    a.gu_div = 2 * kb_per_split;
    a.wait_target[2] = a.gu_div;
  }
  a.wait_target[3] = a.nblk[2] && a.nblk[3] ? g[2].N / 32 : 0;
  a.ctr = ctr;
  if (a.nblk[0] + a.nblk[1] + a.nblk[2] + a.nblk[3] == 0) return 0;
  // one worker per visible CU (each CU fits two of these workgroups: every
  // worker is resident at once, which the in-kernel waits need)
  const int workers = mivgpu_ops_visible_cus();
  if (workers <= 0) return (int)hipErrorInvalidValue;
  // hand-off reads: acquire + L2-cached loads (default) or sc1 loads
  // (MIVGPU_CHAIN_SC1=1, A/B)
  const char* e = getenv("MIVGPU_CHAIN_SC1");   // per call: tests switch it in one process
  const bool sc1 = e && *e && atoi(e) != 0;
  if (W == 2) {
    if (sc1) hipLaunchKernelGGL((decode_chain_kernel<2, false>), dim3(workers), dim3(128), 0, s, a);
    else hipLaunchKernelGGL((decode_chain_kernel<2, true>), dim3(workers), dim3(128), 0, s, a);
  } else {
    if (sc1) hipLaunchKernelGGL((decode_chain_kernel<4, false>), dim3(workers), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((decode_chain_kernel<4, true>), dim3(workers), dim3(256), 0, s, a);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
