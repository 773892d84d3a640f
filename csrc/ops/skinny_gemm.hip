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
#include <stdint.h>

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

enum { EPI_STORE = 0, EPI_SILU_MUL = 1 };

// k-blocks per load group: ~128 VGPRs of fragments in flight per wave
// (16 VGPRs per M- or N-tile per k-block).
constexpr int unroll_of(int mt, int nt) {
  return 128 / (16 * (mt + nt)) >= 4 ? 4 : (128 / (16 * (mt + nt)) >= 2 ? 2 : 1);
}

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
__device__ __forceinline__ void load_kblock(Frag<MT, NT>& f, const u32x4_t* __restrict__ wp, size_t wstride_tile,
                                            const bf16_t* const* xrow, int kb, int lane) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const u32x4_t* src = wp + t * wstride_tile + (size_t)kb * 256 + lane;
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

template <int MT, int NT, int KS, int EPI>
__global__ void __launch_bounds__(64 * KS)
skinny_gemm_kernel(const u32x4_t* __restrict__ wp, const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int M,
                   int K, int N, int ldx, int ldy, int S, float* __restrict__ scratch, int* __restrict__ tickets) {
  __shared__ float red[MT * NT * 16 * 64];
  __shared__ int last;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int KB = K >> 6;
  const int group = blockIdx.x / S, split = blockIdx.x % S;
  const int tile0 = group * NT;
  const size_t wstride_tile = (size_t)KB * 256;  // 16-byte chunks per n-tile
  const u32x4_t* wbase = wp + (size_t)tile0 * wstride_tile;

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

  // Groups of U k-blocks: every load of the group is issued before the first
  // MFMA, which then consume them in order behind decreasing vmcnt waits.
  // (A rotated one-ahead pipeline gets re-serialised by the compiler.)
  constexpr int U = unroll_of(MT, NT);
  int kb = kb0;
  for (; kb + U <= kb1; kb += U) {
    Frag<MT, NT> f[U];
#pragma unroll
    for (int u = 0; u < U; ++u) load_kblock<MT, NT>(f[u], wbase, wstride_tile, xrow, kb + u, lane);
    // keep the whole group in flight: the occupancy-driven scheduler would
    // otherwise sink loads behind MFMAs (≈2 loads in flight per wave)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) mma_kblock<MT, NT>(f[u], acc);
  }
  for (; kb < kb1; ++kb) {
    Frag<MT, NT> f;
    load_kblock<MT, NT>(f, wbase, wstride_tile, xrow, kb, lane);
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

// Pack W[N][K] (row-major bf16) into the fragment order above.
__global__ void pack_weight_kernel(const bf16_t* __restrict__ w, u32x4_t* __restrict__ wp, int N, int K) {
  const size_t KB = K >> 6;
  const size_t total = (size_t)(N >> 5) * KB * 256;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (size_t)gridDim.x * blockDim.x) {
    const int l = q & 63;
    const int j = (q >> 6) & 3;
    const size_t tk = q >> 8;  // t*KB + kb
    const size_t t = tk / KB, kb = tk % KB;
    const size_t row = t * 32 + (l & 31);
    const size_t col = kb * 64 + 32 * (l >> 5) + 8 * j;
    wp[q] = *(const u32x4_t*)(w + row * K + col);
  }
}

struct Args {
  const void* wp;
  const void* x;
  void* y;
  int M, K, N, ldx, ldy, S;
  float* scratch;
  int* tickets;
};

template <int MT, int NT, int KS, int EPI>
hipError_t launch(const Args& a, hipStream_t s) {
  const int groups = (a.N / 32) / NT;
  hipLaunchKernelGGL((skinny_gemm_kernel<MT, NT, KS, EPI>), dim3(groups * a.S), dim3(64 * KS), 0, s,
                     (const u32x4_t*)a.wp, (const bf16_t*)a.x, (bf16_t*)a.y, a.M, a.K, a.N, a.ldx, a.ldy, a.S,
                     a.scratch, a.tickets);
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

int mt_of(int M) { return M <= 32 ? 1 : (M <= 64 ? 2 : 4); }

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
  const bool slice = cus <= 96;
  if (epi == EPI_SILU_MUL) *nt = 2;
  if (*nt != 1 && *nt != 2) *nt = (mt < 4 && ((N / 64) >= 384 || (slice && (N / 64) >= 32))) ? 2 : 1;
  const int groups = (N / 32) / *nt, KB = K / 64;
  if (*ks <= 0) *ks = slice ? 2 : (groups >= 384 ? 1 : 2);
  if (*S <= 0) *S = (!slice && groups <= 128 && KB >= 4 * *ks) ? 2 : 1;
}

}  // namespace

extern "C" {

// Largest M handled in one pass (4 M-tiles of 32 rows per wave).
int mivgpu_skinny_max_m() { return 128; }

// Resolve the launch plan (0 = auto for nt/ks/S) and the scratch it needs:
// *scratch_floats fp32 elements and *tickets ints, both zero-initialised by the
// caller once (the kernel leaves them zeroed).
int mivgpu_skinny_plan(int M, int K, int N, int epi, int* nt, int* ks, int* S, long long* scratch_floats,
                       int* tickets) {
  if (M <= 0 || M > 128 || K <= 0 || (K & 63) || N <= 0 || (N & 31)) return (int)hipErrorInvalidValue;
  plan(M, K, N, epi, nt, ks, S);
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
  hipLaunchKernelGGL(pack_weight_kernel, dim3(blocks), dim3(256), 0, s, (const bf16_t*)w, (u32x4_t*)wp, N, K);
  return (int)hipGetLastError();
}

// epi: 0 = store Y[M][N] (ldy >= N);  1 = SiLU(gate)*up -> Y[M][N/2] for an
// interleaved gate/up weight.  nt/ks/S: 0 = auto (see mivgpu_skinny_plan);
// scratch/tickets must hold what mivgpu_skinny_plan reports for the same
// arguments when S > 1.
int mivgpu_skinny_gemm(const void* wp, const void* x, void* y, int M, int K, int N, int ldx, int ldy, int epi,
                       int nt, int ks, int S, float* scratch, int* tickets, hipStream_t s) {
  if (M <= 0 || M > 128 || K <= 0 || (K & 63) || N <= 0 || (N & 31) || ldx < K || (ldx & 7) || (ldy & 7))
    return (int)hipErrorInvalidValue;
  if (epi != EPI_STORE && epi != EPI_SILU_MUL) return (int)hipErrorInvalidValue;
  plan(M, K, N, epi, &nt, &ks, &S);
  if ((N / 32) % nt || S < 1 || S > K / 64) return (int)hipErrorInvalidValue;
  if (epi == EPI_STORE && ldy < N) return (int)hipErrorInvalidValue;
  if (epi == EPI_SILU_MUL && ldy < N / 2) return (int)hipErrorInvalidValue;
  if (S > 1 && (scratch == nullptr || tickets == nullptr)) return (int)hipErrorInvalidValue;
  if (ks != 1 && ks != 2 && ks != 4 && ks != 8) return (int)hipErrorInvalidValue;
  const Args a{wp, x, y, M, K, N, ldx, ldy, S, scratch, tickets};
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

}  // extern "C"
