// Hand-written gfx950 kernels for the benchmark workload (Qwen3-style decode).
//
// The reference has no kernels; its benchmark drives vLLM
// Qwen3-8B decode (benchmarks/ai-benchmark/benchmark.py:72-75).  These are the
// non-GEMM hot ops of that decode step, written for CDNA4 (64-wide waves,
// 16-byte vector memory ops, wave-shuffle reductions, LDS staging), exported
// with a C ABI so Python calls them through ctypes with raw device pointers and
// the caller's HIP stream (and so they are captured by hipGraphs).
//
//   mivgpu_rmsnorm          out = rmsnorm(x) * w
//   mivgpu_add_rmsnorm      res += x ; out = rmsnorm(res) * w      (fused)
//   mivgpu_qk_norm_rope_kv  per-head RMSNorm(q,k) + NeoX RoPE + KV-cache append
//   mivgpu_prefill_qk_norm_rope_kv  the same over a prompt's tokens into one cache row
//   mivgpu_decode_attention GQA split-K flash-decoding (partials + combine)
//   mivgpu_silu_mul         out = silu(gate) * up
//   mivgpu_embed_rmsnorm    decode head: res = embed[tokens], out = rmsnorm(res) * w
//   mivgpu_decode_tail      decode tail: tokens = argmax(logits), pos += 1, seqlens += 1
//
// All tensors bf16 (raw uint16 bits) unless noted; fp32 accumulation.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint16_t bf16_t;

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (bf16_t)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
  u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even
  return (bf16_t)(u >> 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Unpack 8 bf16 held in a uint4 into floats.
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = (uint32_t)f2bf(f[0]) | ((uint32_t)f2bf(f[1]) << 16);
  v.y = (uint32_t)f2bf(f[2]) | ((uint32_t)f2bf(f[3]) << 16);
  v.z = (uint32_t)f2bf(f[4]) | ((uint32_t)f2bf(f[5]) << 16);
  v.w = (uint32_t)f2bf(f[6]) | ((uint32_t)f2bf(f[7]) << 16);
  return v;
}

// ----------------------------------------------------------------- RMSNorm --
// One 256-thread workgroup per row; thread t owns the 16-byte vectors t,
// t+256, ... (dim % 8 == 0, dim <= 8192).  Every load of the row (x, the
// residual, the norm weight) is issued up front from clamped addresses, so a
// row costs one memory round trip before the reduction instead of one per
// vector (a tiny kernel like this is pure latency: 5.1 -> see profiles).
template <bool ADD>
__global__ void __launch_bounds__(256)
rmsnorm_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ res, const bf16_t* __restrict__ w,
               bf16_t* __restrict__ out, int dim, float eps) {
  const int row = blockIdx.x;
  const int t = threadIdx.x;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * dim);
  uint4* rr = reinterpret_cast<uint4*>(res + (size_t)row * dim);
  uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * dim);
  const uint4* wv = reinterpret_cast<const uint4*>(w);
  __shared__ float red[4];
  constexpr int MAXV = 4;  // up to 4 x 8 elements per thread (dim <= 8192)
  const int nvec = dim / 8;
  uint4 xa[MAXV], xb[MAXV], wa[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = min(t + k * 256, nvec - 1);
    xa[k] = xr[vi];
    if (ADD) xb[k] = rr[vi];
    wa[k] = wv[vi];
  }
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = t + k * 256;
    float a[8];
    unpack8(xa[k], a);
    if (ADD) {
      float c[8];
      unpack8(xb[k], c);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += c[e];
      const uint4 packed = pack8(a);
      if (vi < nvec) rr[vi] = packed;
      unpack8(packed, a);   // normalise the bf16-rounded residual, exactly what is stored
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[k][e] = a[e];
      if (vi < nvec) ss += a[e] * a[e];
    }
  }
  ss = wave_sum(ss);
  if ((t & 63) == 0) red[t >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float inv = rsqrtf(tot / (float)dim + eps);
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = t + k * 256;
    if (vi < nvec) {
      float wf[8], o[8];
      unpack8(wa[k], wf);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = v[k][e] * inv * wf[e];
      orow[vi] = pack8(o);
    }
  }
}

// ------------------------------------------ decode step head and tail ----
// Head: res[b] = embed[tokens[b]], h[b] = rmsnorm(res[b]) * w in one launch
// (was index_select + rmsnorm).  One 256-thread workgroup per row, the
// embedding row loaded up front as in rmsnorm_kernel.
__global__ void __launch_bounds__(256)
embed_rmsnorm_kernel(const bf16_t* __restrict__ embed, const int64_t* __restrict__ tokens,
                     const bf16_t* __restrict__ w, bf16_t* __restrict__ res, bf16_t* __restrict__ out, int dim,
                     long long vocab, float eps, float* __restrict__ ss_out) {
  const int row = blockIdx.x;
  const int t = threadIdx.x;
  long long tok = tokens[row];
  tok = tok < 0 ? 0 : (tok >= vocab ? vocab - 1 : tok);   // a bad id reads a valid row, never out of bounds
  const uint4* xr = reinterpret_cast<const uint4*>(embed + (size_t)tok * dim);
  uint4* rr = reinterpret_cast<uint4*>(res + (size_t)row * dim);
  uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * dim);
  // w may be null when only the sums of squares are wanted (out == nullptr):
  // then the norm weight is never read
  const uint4* wv = reinterpret_cast<const uint4*>(out != nullptr ? w : embed);
  __shared__ float red[4];
  constexpr int MAXV = 4;
  const int nvec = dim / 8;
  uint4 xa[MAXV], wa[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = min(t + k * 256, nvec - 1);
    xa[k] = xr[vi];
    wa[k] = wv[vi];
  }
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = t + k * 256;
    if (vi < nvec) {
      rr[vi] = xa[k];
      float a[8];
      unpack8(xa[k], a);
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += a[e] * a[e];
    }
  }
  ss = wave_sum(ss);
  if ((t & 63) == 0) red[t >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  if (ss_out != nullptr && t == 0) ss_out[row] = tot;   // the norm-fused decoder's first row-scale slot
  if (out == nullptr) return;
  const float inv = rsqrtf(tot / (float)dim + eps);
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = t + k * 256;
    if (vi < nvec) {
      float a[8], wf[8], o[8];
      unpack8(xa[k], a);
      unpack8(wa[k], wf);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = a[e] * inv * wf[e];
      orow[vi] = pack8(o);
    }
  }
}

// Tail: tokens[b] = argmax(logits[b]) (first index of the maximum, NaN
// counts as the maximum, as torch.argmax), pos[b] += 1, seqlens[b] += 1 in
// one launch (was argmax + two adds: 48 + 9 us of a 4.9 ms step on the whole
// GPU).  TAIL_SPLIT workgroups per row, each over a contiguous slice with
// every 16-byte load issued before the compare (one memory round trip); each
// publishes its best as one 64-bit key (order-preserving value bits above the
// complemented index, so the larger key is the larger value, then the smaller
// index) with a device-scope atomicMax into the row's slot, then takes a
// ticket; the last arriver writes the token, advances pos / seqlens and
// resets slot and ticket for the next launch.
constexpr int TAIL_THREADS = 256;
constexpr int TAIL_SPLIT = 8;
constexpr int TAIL_MAXV = 10;   // 16-byte vectors per thread: vocab <= 10 * 8 * 256 * 8 = 163840

__device__ __forceinline__ unsigned long long argmax_key(float v, int i) {
  uint32_t u = __float_as_uint(v);
  u = (v != v) ? 0xffffffffu : ((u & 0x80000000u) ? ~u : (u | 0x80000000u));
  return ((unsigned long long)u << 32) | (uint32_t)(~(uint32_t)i);
}

__global__ void __launch_bounds__(TAIL_THREADS)
decode_tail_kernel(const bf16_t* __restrict__ logits, int ld, int vocab, int64_t* __restrict__ tokens,
                   int* __restrict__ pos, int* __restrict__ seqlens, unsigned long long* __restrict__ slots,
                   int* __restrict__ tickets) {
  const int row = blockIdx.y, part = blockIdx.x;
  const int t = threadIdx.x;
  const int nvec = vocab / 8;
  const int v0 = (int)((long long)nvec * part / TAIL_SPLIT), v1 = (int)((long long)nvec * (part + 1) / TAIL_SPLIT);
  const uint4* lr = reinterpret_cast<const uint4*>(logits + (size_t)row * ld);
  uint4 va[TAIL_MAXV];
#pragma unroll
  for (int k = 0; k < TAIL_MAXV; ++k) va[k] = lr[min(v0 + t + k * TAIL_THREADS, nvec - 1)];
  unsigned long long best = 0;
#pragma unroll
  for (int k = 0; k < TAIL_MAXV; ++k) {
    const int vi = v0 + t + k * TAIL_THREADS;
    if (vi < v1) {
      float a[8];
      unpack8(va[k], a);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const unsigned long long key = argmax_key(a[e], vi * 8 + e);
        best = key > best ? key : best;
      }
    }
  }
  if (part == TAIL_SPLIT - 1)
    for (int i = nvec * 8 + t; i < vocab; i += TAIL_THREADS) {   // vocab % 8 tail
      const unsigned long long key = argmax_key(bf2f(logits[(size_t)row * ld + i]), i);
      best = key > best ? key : best;
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long other = __shfl_xor(best, o, 64);
    best = other > best ? other : best;
  }
  __shared__ unsigned long long s_b[TAIL_THREADS / 64];
  if ((t & 63) == 0) s_b[t >> 6] = best;
  __syncthreads();
  if (t != 0) return;
#pragma unroll
  for (int w = 1; w < TAIL_THREADS / 64; ++w) best = s_b[w] > best ? s_b[w] : best;
  // device-scope atomics only (no cache-flushing fences): the max is drained
  // (vmcnt) before the ticket is taken, as the split-K GEMM's slab adds
  __hip_atomic_fetch_max(slots + row, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int ticket = __hip_atomic_fetch_add(tickets + row, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (ticket != TAIL_SPLIT - 1) return;
  const unsigned long long key = __hip_atomic_exchange(slots + row, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(tickets + row, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  tokens[row] = (int64_t)(~(uint32_t)(key & 0xffffffffu));
  pos[row] += 1;
  seqlens[row] += 1;
}

// ------------------------------------------- QK-norm + RoPE + KV append ----
// grid = (B, Hq + 2*Hkv); one wave per (token, head).  D = 128: lane l owns
// elements l and l+64, which is exactly a NeoX rotate-half pair.
// Decode: row b is sequence b (cache row b), q out [B][Hq][D].
// Prefill (cache_b >= 0): the rows are the prompt tokens of ONE sequence, all
// appended to cache row cache_b at their own positions; q is written
// head-grouped [Hkv][G][rows][D] (the G query heads sharing a KV head are one
// contiguous block of rows for the attention GEMMs), and K/V also go to
// k_plain / v_plain [Hkv][rows][D] when given (the prompt's own attention).
// Prefill runs TPW tokens per wave (qk_norm_rope_kv_kernel<PACKED, 8>): a
// one-token wave has 256 B in flight, and with the CU's workgroup slots full
// that capped an 8192-token prompt at ~1.7 TB/s (135 us per layer); eight
// tokens' loads are issued before the first token is processed.
template <bool PACKED>
__device__ __forceinline__ void qk_one(const bf16_t* __restrict__ qkv_row, float x0, float x1, int b, int h,
                                       int l, int p, int rows, const bf16_t* __restrict__ qw,
                                       const bf16_t* __restrict__ kw, bf16_t* __restrict__ q_out,
                                       bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache, int Hq,
                                       int Hkv, int max_ctx, float eps, float inv_freq, int cache_b,
                                       bf16_t* __restrict__ k_plain, bf16_t* __restrict__ v_plain) {
  constexpr int D = 128;
  const int cb = cache_b >= 0 ? cache_b : b;
  const bool in_range = p >= 0 && p < max_ctx;  // never write past the cache
  if (h >= Hq + Hkv) {  // V head: plain copy into the cache
    const int hv = h - Hq - Hkv;
    if (v_plain) {
      bf16_t* dst = v_plain + ((size_t)hv * rows + b) * D;
      dst[l] = qkv_row[l];
      dst[l + 64] = qkv_row[l + 64];
    }
    if (!in_range) return;
    if (PACKED) {  // V group [dt 8][q 4][r 16][e 8]: key = 8q + e, dim = 16dt + r
      bf16_t* grp = v_cache + ((size_t)cb * Hkv + hv) * (size_t)max_ctx * D + (size_t)(p >> 5) * (32 * D);
      const int kq = (p & 31) >> 3, ke = p & 7;
      grp[(((l >> 4) * 4 + kq) * 16 + (l & 15)) * 8 + ke] = f2bf(x0);
      grp[((((l + 64) >> 4) * 4 + kq) * 16 + (l & 15)) * 8 + ke] = f2bf(x1);
    } else {
      bf16_t* dst = v_cache + (((size_t)cb * Hkv + hv) * max_ctx + p) * D;
      dst[l] = f2bf(x0);
      dst[l + 64] = f2bf(x1);
    }
    return;
  }
  const bool is_q = h < Hq;
  const bf16_t* nw = is_q ? qw : kw;
  const float ss = wave_sum(x0 * x0 + x1 * x1);
  const float inv = rsqrtf(ss / (float)D + eps);
  x0 = x0 * inv * bf2f(nw[l]);
  x1 = x1 * inv * bf2f(nw[l + 64]);
  float s, c;
  sincosf((float)p * inv_freq, &s, &c);
  const float o0 = x0 * c - x1 * s;
  const float o1 = x1 * c + x0 * s;
  bf16_t* dst;
  if (is_q) {
    if (cache_b >= 0) {
      const int G = Hq / Hkv;
      dst = q_out + (((size_t)(h / G) * G + h % G) * rows + b) * D;
    } else {
      dst = q_out + ((size_t)b * Hq + h) * D;
    }
  } else {
    const int hk = h - Hq;
    if (k_plain) {
      bf16_t* kp = k_plain + ((size_t)hk * rows + b) * D;
      kp[l] = f2bf(o0);
      kp[l + 64] = f2bf(o1);
    }
    if (!in_range) return;
    if (PACKED) {  // K group [t 2][s 4][q 4][r 16][e 8]: key = 8(r/4) + 4t + r%4, dim = 32s + 8q + e
      bf16_t* grp = k_cache + ((size_t)cb * Hkv + hk) * (size_t)max_ctx * D + (size_t)(p >> 5) * (32 * D);
      const int k = p & 31;
      const int kt = (k >> 2) & 1, kr = 4 * (k >> 3) + (k & 3);
      grp[(((kt * 4 + (l >> 5)) * 4 + ((l >> 3) & 3)) * 16 + kr) * 8 + (l & 7)] = f2bf(o0);
      grp[(((kt * 4 + ((l + 64) >> 5)) * 4 + (((l + 64) >> 3) & 3)) * 16 + kr) * 8 + (l & 7)] = f2bf(o1);
      return;
    }
    dst = k_cache + (((size_t)cb * Hkv + hk) * max_ctx + p) * D;
  }
  dst[l] = f2bf(o0);
  dst[l + 64] = f2bf(o1);
}

// grid = (ceil(rows / TPW), Hq + 2*Hkv), one wave of 64 lanes.  (Four
// head-waves per workgroup measured the same: 99.3 vs 99.6 us at 8192 rows.)
template <bool PACKED, int TPW>
__global__ void __launch_bounds__(64)
qk_norm_rope_kv_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ qw,
                       const bf16_t* __restrict__ kw, const int* __restrict__ pos,
                       bf16_t* __restrict__ q_out, bf16_t* __restrict__ k_cache,
                       bf16_t* __restrict__ v_cache, int Hq, int Hkv, int max_ctx, float eps,
                       float theta, int cache_b, bf16_t* __restrict__ k_plain,
                       bf16_t* __restrict__ v_plain, int rows) {
  constexpr int D = 128;
  const int b0 = blockIdx.x * TPW;
  const int h = blockIdx.y;
  const int l = threadIdx.x;
  const int row_stride = (Hq + 2 * Hkv) * D;
  float x0[TPW], x1[TPW];
  int p[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {  // every token's loads in flight first
    const int b = min(b0 + t, rows - 1);
    const bf16_t* src = qkv + (size_t)b * row_stride + (size_t)h * D;
    x0[t] = bf2f(src[l]);
    x1[t] = bf2f(src[l + 64]);
    p[t] = pos[b];
  }
  if constexpr (PACKED && TPW == 8) {
    // V head, eight consecutive positions from a multiple of 8 (a prompt):
    // they are the eight keys of one 16-byte run per dim of the packed group,
    // so each lane stores its two dims' runs whole (2 stores, not 16 2-byte)
    bool run = h >= Hq + Hkv && cache_b >= 0 && b0 + TPW <= rows && (p[0] & 7) == 0 && p[0] >= 0 &&
               p[0] + TPW <= max_ctx;
#pragma unroll
    for (int t = 1; t < TPW; ++t) run = run && p[t] == p[0] + t;
    if (run) {
      const int hv = h - Hq - Hkv;
      if (v_plain) {
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          bf16_t* dst = v_plain + ((size_t)hv * rows + b0 + t) * D;
          dst[l] = f2bf(x0[t]);  // bf16 -> fp32 -> bf16 is exact
          dst[l + 64] = f2bf(x1[t]);
        }
      }
      bf16_t* grp = v_cache + ((size_t)cache_b * Hkv + hv) * (size_t)max_ctx * D + (size_t)(p[0] >> 5) * (32 * D);
      const int kq = (p[0] & 31) >> 3;
      uint4 r0, r1;
      r0.x = (uint32_t)f2bf(x0[0]) | ((uint32_t)f2bf(x0[1]) << 16);
      r0.y = (uint32_t)f2bf(x0[2]) | ((uint32_t)f2bf(x0[3]) << 16);
      r0.z = (uint32_t)f2bf(x0[4]) | ((uint32_t)f2bf(x0[5]) << 16);
      r0.w = (uint32_t)f2bf(x0[6]) | ((uint32_t)f2bf(x0[7]) << 16);
      r1.x = (uint32_t)f2bf(x1[0]) | ((uint32_t)f2bf(x1[1]) << 16);
      r1.y = (uint32_t)f2bf(x1[2]) | ((uint32_t)f2bf(x1[3]) << 16);
      r1.z = (uint32_t)f2bf(x1[4]) | ((uint32_t)f2bf(x1[5]) << 16);
      r1.w = (uint32_t)f2bf(x1[6]) | ((uint32_t)f2bf(x1[7]) << 16);
      *(uint4*)(grp + (((l >> 4) * 4 + kq) * 16 + (l & 15)) * 8) = r0;
      *(uint4*)(grp + ((((l + 64) >> 4) * 4 + kq) * 16 + (l & 15)) * 8) = r1;
      return;
    }
  }
  // inv_freq = theta^(-2l/D)
  const float inv_freq = exp2f(-(2.0f * (float)l / (float)D) * log2f(theta));
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int b = b0 + t;
    if (b >= rows) break;  // wave-uniform
    qk_one<PACKED>(qkv + (size_t)b * row_stride + (size_t)h * D, x0[t], x1[t], b, h, l, p[t], rows, qw, kw,
                   q_out, k_cache, v_cache, Hq, Hkv, max_ctx, eps, inv_freq, cache_b, k_plain, v_plain);
  }
}

// Prefill QK-norm + RoPE + KV append, vectorised (round 6).  The per-token
// kernel above gives each lane two bf16 elements (l, l + 64): 2-byte loads
// and stores, 128 B per memory instruction, and measured ~2.3 TB/s on an
// 8192-token prompt (99.6 us per layer; four head-waves per workgroup made no
// difference, so it is not the workgroup slots).  Here 16 lanes own one
// token (lane j: dims 4j..4j+3 and their NeoX partners 64+4j..64+4j+3, one
// 8-byte load each), a wave covers four tokens per instruction and loops
// over QP_TPW tokens with every load issued first; the RMS reduction is four
// xor-shuffles inside the 16-lane group.  Stores: q / k_plain / v_plain and
// the packed K run (4 dims = 8 contiguous bytes of a 16-byte e-run) as
// 8-byte stores; V heads are transposed through LDS so that each packed-V
// run (eight consecutive keys of one dim) is one 16-byte store.
constexpr int QP_TPW = 16;
template <bool PACKED>
__global__ void __launch_bounds__(64)
qk_prefill_vec_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ qw, const bf16_t* __restrict__ kw,
                      const int* __restrict__ pos, bf16_t* __restrict__ q_out, bf16_t* __restrict__ k_cache,
                      bf16_t* __restrict__ v_cache, int Hq, int Hkv, int max_ctx, float eps, float log2_theta,
                      int cache_b, bf16_t* __restrict__ k_plain, bf16_t* __restrict__ v_plain, int rows) {
  constexpr int D = 128, NG = QP_TPW / 4;
  const int b0 = blockIdx.x * QP_TPW;
  const int h = blockIdx.y;
  const int lane = threadIdx.x;
  const int sub = lane >> 4;   // token within a group of four
  const int j = lane & 15;     // dims 4j..4j+3 and 64+4j..64+4j+3
  const size_t row_stride = (size_t)(Hq + 2 * Hkv) * D;
  uint2 lo[NG], hi[NG];
  int p[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {  // every token's loads in flight first
    const int b = min(b0 + 4 * g + sub, rows - 1);
    const bf16_t* src = qkv + (size_t)b * row_stride + (size_t)h * D;
    lo[g] = *reinterpret_cast<const uint2*>(src + 4 * j);
    hi[g] = *reinterpret_cast<const uint2*>(src + 64 + 4 * j);
    p[g] = pos[b];
  }
  auto unpack = [](uint2 u, float* f) {
    f[0] = __uint_as_float(u.x << 16);
    f[1] = __uint_as_float(u.x & 0xffff0000u);
    f[2] = __uint_as_float(u.y << 16);
    f[3] = __uint_as_float(u.y & 0xffff0000u);
  };
  auto pack = [](const float* f) {
    uint2 u;
    u.x = (uint32_t)f2bf(f[0]) | ((uint32_t)f2bf(f[1]) << 16);
    u.y = (uint32_t)f2bf(f[2]) | ((uint32_t)f2bf(f[3]) << 16);
    return u;
  };
  if (h >= Hq + Hkv) {  // ---- V head: plain copy, cache append
    const int hv = h - Hq - Hkv;
    __shared__ uint2 s_v[QP_TPW][32];   // [token][16 lo + 16 hi quads]: 4 KB
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int b = b0 + 4 * g + sub;
      if (v_plain && b < rows) {
        bf16_t* dst = v_plain + ((size_t)hv * rows + b) * D;
        *reinterpret_cast<uint2*>(dst + 4 * j) = lo[g];
        *reinterpret_cast<uint2*>(dst + 64 + 4 * j) = hi[g];
      }
      s_v[4 * g + sub][j] = lo[g];
      s_v[4 * g + sub][16 + j] = hi[g];
    }
    const int pb = pos[min(b0, rows - 1)];
    bool run = PACKED && b0 + QP_TPW <= rows && (pb & 7) == 0 && pb >= 0 && pb + QP_TPW <= max_ctx;
    // every token of the tile at consecutive positions (a prompt): wave-uniform
#pragma unroll
    for (int g = 0; g < NG; ++g) run = run && p[g] == pb + 4 * g + sub;
    run = __all(run);
    __syncthreads();
    const int cb = cache_b;
    if (run) {
      // 2 runs of 8 keys x 128 dims = 256 16-byte stores, four per lane
      bf16_t* base = v_cache + ((size_t)cb * Hkv + hv) * (size_t)max_ctx * D;
      const bf16_t* sv = reinterpret_cast<const bf16_t*>(&s_v[0][0]);   // [token][lo 64 | hi 64] dims
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int idx = k * 64 + lane;
        const int r = idx >> 7;          // key run: tokens 8r..8r+7
        const int d = idx & 127;         // dim
        // s_v row layout: quads 0..15 = dims 0..63 (4j..4j+3), quads 16..31 = dims 64..127
        const int col = d;               // dims are laid out in order in the row
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t a = sv[(8 * r + 2 * e) * D + col];
          const uint32_t c = sv[(8 * r + 2 * e + 1) * D + col];
          w[e] = a | (c << 16);
        }
        const int pr = pb + 8 * r;
        bf16_t* grp = base + (size_t)(pr >> 5) * (32 * D);
        const int kq = (pr & 31) >> 3;
        *reinterpret_cast<uint4*>(grp + (((d >> 4) * 4 + kq) * 16 + (d & 15)) * 8) = make_uint4(w[0], w[1], w[2], w[3]);
      }
      return;
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {   // ragged tail or scattered positions: element stores
      const int b = b0 + 4 * g + sub;
      const int pp = p[g];
      if (b >= rows || pp < 0 || pp >= max_ctx) continue;
      float f[8];
      unpack(lo[g], f);
      unpack(hi[g], f + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int d = (e < 4 ? 0 : 64) + 4 * j + (e & 3);
        if (PACKED) {
          bf16_t* grp = v_cache + ((size_t)cb * Hkv + hv) * (size_t)max_ctx * D + (size_t)(pp >> 5) * (32 * D);
          grp[(((d >> 4) * 4 + ((pp & 31) >> 3)) * 16 + (d & 15)) * 8 + (pp & 7)] = f2bf(f[e]);
        } else {
          v_cache[(((size_t)cb * Hkv + hv) * max_ctx + pp) * D + d] = f2bf(f[e]);
        }
      }
    }
    return;
  }
  // ---- Q / K head: RMSNorm over the head, NeoX RoPE
  const bool is_q = h < Hq;
  const bf16_t* nw = is_q ? qw : kw;
  float w[8], invf[4];
  unpack(*reinterpret_cast<const uint2*>(nw + 4 * j), w);
  unpack(*reinterpret_cast<const uint2*>(nw + 64 + 4 * j), w + 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) invf[e] = exp2f(-(2.0f * (float)(4 * j + e) / (float)D) * log2_theta);
  const int G = Hq / Hkv;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int b = b0 + 4 * g + sub;
    float x[8];
    unpack(lo[g], x);
    unpack(hi[g], x + 4);
    float ss = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) ss += x[e] * x[e];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);   // inside the 16-lane group
    const float inv = rsqrtf(ss / (float)D + eps);
    float o[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x0 = x[e] * inv * w[e], x1 = x[e + 4] * inv * w[e + 4];
      float sn, cs;
      sincosf((float)p[g] * invf[e], &sn, &cs);
      o[e] = x0 * cs - x1 * sn;
      o[e + 4] = x1 * cs + x0 * sn;
    }
    if (b >= rows) continue;
    const uint2 olo = pack(o), ohi = pack(o + 4);
    if (is_q) {
      bf16_t* dst = q_out + (((size_t)(h / G) * G + h % G) * rows + b) * D;
      *reinterpret_cast<uint2*>(dst + 4 * j) = olo;
      *reinterpret_cast<uint2*>(dst + 64 + 4 * j) = ohi;
      continue;
    }
    const int hk = h - Hq;
    if (k_plain) {
      bf16_t* kp = k_plain + ((size_t)hk * rows + b) * D;
      *reinterpret_cast<uint2*>(kp + 4 * j) = olo;
      *reinterpret_cast<uint2*>(kp + 64 + 4 * j) = ohi;
    }
    const int pp = p[g];
    if (pp < 0 || pp >= max_ctx) continue;
    if (PACKED) {  // K group [t 2][s 4][q 4][r 16][e 8]: key = 8(r/4) + 4t + r%4, dim = 32s + 8q + e
      bf16_t* grp = k_cache + ((size_t)cache_b * Hkv + hk) * (size_t)max_ctx * D + (size_t)(pp >> 5) * (32 * D);
      const int k = pp & 31;
      const int kt = (k >> 2) & 1, kr = 4 * (k >> 3) + (k & 3);
      const int d0 = 4 * j, d1 = 64 + 4 * j;   // 4-aligned: inside one 8-dim e-run
      *reinterpret_cast<uint2*>(grp + (((kt * 4 + (d0 >> 5)) * 4 + ((d0 >> 3) & 3)) * 16 + kr) * 8 + (d0 & 7)) = olo;
      *reinterpret_cast<uint2*>(grp + (((kt * 4 + (d1 >> 5)) * 4 + ((d1 >> 3) & 3)) * 16 + kr) * 8 + (d1 & 7)) = ohi;
    } else {
      bf16_t* dst = k_cache + (((size_t)cache_b * Hkv + hk) * max_ctx + pp) * D;
      *reinterpret_cast<uint2*>(dst + 4 * j) = olo;
      *reinterpret_cast<uint2*>(dst + 64 + 4 * j) = ohi;
    }
  }
}

// ---------------------------------------------- GQA split-K decode attention --
// grid = (nsplit, Hkv, B), 256 threads.  Each workgroup scores SPLIT keys of
// one (batch, kv-head) against the G = Hq/Hkv query heads that share it, so
// every K/V byte is read once per group instead of once per query head.
//   scores: 8 lanes per key (16 dims each), 8 keys per wave-iteration
//   P.V   : 16 lanes per key row (8 dims each, one 16-B load), 16 rows at once
// Partials (unnormalised O, running max m, sum l) go to fp32 workspace; the
// combine kernel merges splits.  G <= 8 supported (Qwen3-8B: G = 4).
#ifndef MIVGPU_ATT_SPLIT
#define MIVGPU_ATT_SPLIT 256
#endif
constexpr int ATT_SPLIT = MIVGPU_ATT_SPLIT;   // keys per partial workgroup
constexpr int ATT_D = 128;

// PF (load scheduling): 0 = one dependent K / V load per loop trip (lowest
// VGPRs, highest occupancy); 1 = every K and V load of the thread issued up
// front; 2 = K up front, V issued right after the scores (before the softmax
// barrier).  Chosen per launch by mivgpu_decode_attention (measured).  A
// streaming flash-decoding variant (one workgroup walking 64/128-key blocks
// with an online softmax and double-buffered K/V) measured 2x slower in a
// 64-CU slice: profiles/attention_streaming_negative.json.
template <int G, int PF>
__global__ void __launch_bounds__(256)
decode_attn_partial_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k_cache,
                           const bf16_t* __restrict__ v_cache, const int* __restrict__ seqlens,
                           float* __restrict__ o_part, float* __restrict__ ml_part, int Hq, int Hkv,
                           int max_ctx, int nsplit, float scale) {
  const int split = blockIdx.x;
  const int hk = blockIdx.y;
  const int b = blockIdx.z;
  const int t = threadIdx.x;
  const int L = min(seqlens[b], max_ctx);
  const int j0 = split * ATT_SPLIT;
  const int n = min(ATT_SPLIT, L - j0);
  __shared__ float s_p[G][ATT_SPLIT];
  __shared__ float s_red[8][G];
  __shared__ float s_acc[16][G][ATT_D / 2];  // reduced in two halves of D
  const size_t part_base = ((size_t)b * Hq + (size_t)hk * G);
  if (n <= 0) {  // empty split (short sequence): neutral partial
    if (t < G) {
      ml_part[((part_base + t) * nsplit + split) * 2 + 0] = -INFINITY;
      ml_part[((part_base + t) * nsplit + split) * 2 + 1] = 0.f;
    }
    return;
  }
  const bf16_t* kb = k_cache + ((size_t)b * Hkv + hk) * (size_t)max_ctx * ATT_D;
  const bf16_t* vb = v_cache + ((size_t)b * Hkv + hk) * (size_t)max_ctx * ATT_D;

  const int lane = t & 63, wave = t >> 6;
  const int sub = lane & 7;       // 16-dim chunk of a key row (scores)
  const int krow = lane >> 3;     // key within a wave-iteration (scores)
  const int r = t >> 4, c = t & 15;  // P.V: row group, 8-dim column chunk
  constexpr int KIT = ATT_SPLIT / 32;   // score iterations per wave
  constexpr int VIT = ATT_SPLIT / 16;   // P.V rows per thread
  // Out-of-range rows are clamped to row j0 and their results discarded (no
  // branches around loads).  q is loaded first: vmcnt retires in order.
  uint4 qreg[G][2];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint4* qp = reinterpret_cast<const uint4*>(q + (part_base + g) * ATT_D + sub * 16);
    qreg[g][0] = qp[0];
    qreg[g][1] = qp[1];
  }
  uint4 kreg[PF ? KIT : 1][2];
  uint4 vreg[PF ? VIT : 1];
  auto load_k = [&](int i, uint4* dst) {
    const int jj = wave * 8 + krow + 32 * i;
    const uint4* kp = reinterpret_cast<const uint4*>(kb + (size_t)(j0 + (jj < n ? jj : 0)) * ATT_D + sub * 16);
    dst[0] = kp[0];
    dst[1] = kp[1];
  };
  auto load_v = [&](int i) {
    const int jj = r + 16 * i;
    return *reinterpret_cast<const uint4*>(vb + (size_t)(j0 + (jj < n ? jj : 0)) * ATT_D + c * 8);
  };
  if constexpr (PF >= 1) {
#pragma unroll
    for (int i = 0; i < KIT; ++i) load_k(i, kreg[i]);
  }
  if constexpr (PF == 1) {
#pragma unroll
    for (int i = 0; i < VIT; ++i) vreg[i] = load_v(i);
  }
  if constexpr (PF >= 1) __builtin_amdgcn_sched_barrier(0);   // keep the batch ahead of its uses

  // ---- scores
  {
    float qf[G][16];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      unpack8(qreg[g][0], &qf[g][0]);
      unpack8(qreg[g][1], &qf[g][8]);
    }
#pragma unroll
    for (int i = 0; i < KIT; ++i) {
      const int jj = wave * 8 + krow + 32 * i;
      uint4 kk[2];
      if constexpr (PF >= 1) {
        kk[0] = kreg[i][0];
        kk[1] = kreg[i][1];
      } else {
        load_k(i, kk);
      }
      float kf[16];
      unpack8(kk[0], &kf[0]);
      unpack8(kk[1], &kf[8]);
      float acc[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float a = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) a = fmaf(qf[g][e], kf[e], a);
        a += __shfl_xor(a, 1, 64);
        a += __shfl_xor(a, 2, 64);
        a += __shfl_xor(a, 4, 64);
        acc[g] = a;
      }
      if (sub == 0 && jj < n) {
#pragma unroll
        for (int g = 0; g < G; ++g) s_p[g][jj] = acc[g] * scale;
      }
    }
  }
  if constexpr (PF == 2) {
#pragma unroll
    for (int i = 0; i < VIT; ++i) vreg[i] = load_v(i);   // in flight across the softmax
  }
  __syncthreads();

  // ---- softmax statistics per query head (t indexes keys)
  float m[G], lsum[G];
  {
    float mv[G];
#pragma unroll
    for (int g = 0; g < G; ++g) mv[g] = t < n ? s_p[g][t] : -INFINITY;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float w = wave_max(mv[g]);
      if ((t & 63) == 0) s_red[t >> 6][g] = w;
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < G; ++g) m[g] = fmaxf(fmaxf(s_red[0][g], s_red[1][g]), fmaxf(s_red[2][g], s_red[3][g]));
    __syncthreads();
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float e = t < n ? __expf(mv[g] - m[g]) : 0.f;
      if (t < n) s_p[g][t] = e;
      float w = wave_sum(e);
      if ((t & 63) == 0) s_red[4 + (t >> 6)][g] = w;
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < G; ++g) lsum[g] = s_red[4][g] + s_red[5][g] + s_red[6][g] + s_red[7][g];
  }

  // ---- P.V: group r = t>>4 owns rows r, r+16, ...; column chunk c = t&15
  float acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[g][e] = 0.f;
#pragma unroll
  for (int i = 0; i < VIT; ++i) {
    const int jj = r + 16 * i;
    if (jj < n) {
      float vf[8];
      if constexpr (PF >= 1)
        unpack8(vreg[i], vf);
      else
        unpack8(load_v(i), vf);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float p = s_p[g][jj];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[g][e] = fmaf(p, vf[e], acc[g][e]);
      }
    }
  }
  // Cross-group reduction through LDS, one half of D at a time (16 KB for G=4).
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const bool mine = (c >> 3) == half;
    if (mine) {
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 8; ++e) s_acc[r][g][(c & 7) * 8 + e] = acc[g][e];
    }
    __syncthreads();
    for (int idx = t; idx < G * (ATT_D / 2); idx += 256) {
      const int g = idx / (ATT_D / 2), d = idx % (ATT_D / 2);
      float s = 0.f;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) s += s_acc[rr][g][d];
      o_part[((part_base + g) * nsplit + split) * ATT_D + half * (ATT_D / 2) + d] = s;
    }
    __syncthreads();
  }
  if (t < G) {
    ml_part[((part_base + t) * nsplit + split) * 2 + 0] = m[t];
    ml_part[((part_base + t) * nsplit + split) * 2 + 1] = lsum[t];
  }
}

// ------------------------------------------- MFMA decode attention (default) --
// Same partial/combine contract as above, but QK^T and P.V run on
// v_mfma_f32_16x16x32_bf16, and K and V live in a FRAGMENT-PACKED cache: each
// 32-key group of a (batch, kv-head) is 8 KB of K followed (in its own
// tensor) by 8 KB of V, laid out so that every load instruction of a wave is
// one linear 1 KB read that lands exactly in the MFMA operand registers:
//   K group: [t 2][s 4][q 4][r 16][e 8]   key = 8*(r/4) + 4t + r%4, dim = 32s + 8q + e
//   V group: [dt 8][q 4][r 16][e 8]       key = 8q + e,              dim = 16dt + r
// (lane l = 16q + r reads element block l of every 1 KB slab).  The VALU
// kernel spends ~1.7k vector instructions per wave per 64 keys on unpack +
// FMA + shuffles, 30-40 % of its time in a 64- or 32-CU slice; here a wave's
// 32 keys cost 16 MFMAs and ~60 VALU instructions.
//
// grid = (nsplit, Hkv, B), WAVES x 64 threads, 32 keys (one group) per wave:
//   scores S^T = K (32 keys x 128) . Q^T (128 x G): 2 key tiles x 4 k-steps;
//     the packing gives lane l the 8 contiguous keys 8*(l/16) .. +8 of query
//     l%16 in its two C tiles.
//   local softmax per wave (max/sum over its 32 keys, no barrier).
//   O^T = V^T (128 x 32 keys) . P^T (32 keys x G): 8 dim tiles; A operand =
//     the V slab, B operand = the lane's own 8 probabilities (bf16).
//   one LDS merge of the WAVES per-wave (m, l, O) triples -> partial.
// All 20 loads of a wave (Q, 8 K, 8 V slabs: 16 KB) are issued before the first
// MFMA; a wave past the sequence end reads the split's first group (valid
// memory) and masks everything.
constexpr int ATT_KPW = 32;            // keys per wave = one packed group
constexpr int ATT_GROUP = ATT_KPW * ATT_D;   // elements per packed group (K or V)

template <int G, int WAVES, bool NT>
__global__ void __launch_bounds__(WAVES * 64)
decode_attn_mfma_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k_pack,
                        const bf16_t* __restrict__ v_pack, const int* __restrict__ seqlens,
                        float* __restrict__ o_part, float* __restrict__ ml_part, int Hq, int Hkv,
                        int max_ctx, int nsplit, float scale_log2) {
  typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
  typedef __attribute__((ext_vector_type(4))) float f32x4_t;
  constexpr int SPLIT = WAVES * ATT_KPW;
  // padded LDS row: the P.V partial writes (lane (r16, q4) -> row r16,
  // column 16dt + 4q4 + i) fall on bank r16 * DP + 4q4: a pitch of 1 (mod 32)
  // spreads the G x 4 lanes of a write over distinct banks (D + 4 put them
  // 4-way on 4 banks: 491k conflict cycles per call, profiles/round3/pmc_final)
  constexpr int DP = ATT_D + 1;
  const int split = blockIdx.x;
  const int hk = blockIdx.y;
  const int b = blockIdx.z;
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int r16 = lane & 15, q4 = lane >> 4;
  const int L = min(seqlens[b], max_ctx);
  const int j0 = split * SPLIT;
  const int n = min(SPLIT, L - j0);
  const size_t part_base = ((size_t)b * Hq + (size_t)hk * G);
  if (n <= 0) {
    if (t < G) {
      ml_part[((part_base + t) * nsplit + split) * 2 + 0] = -INFINITY;
      ml_part[((part_base + t) * nsplit + split) * 2 + 1] = 0.f;
    }
    return;
  }
  __shared__ float s_o[WAVES][G][DP];
  __shared__ float s_m[WAVES][G];
  __shared__ float s_l[WAVES][G];

  const int wj0 = j0 + wave * ATT_KPW;   // first key of this wave
  const int wn = min(ATT_KPW, L - wj0);   // valid keys of this wave (may be <= 0)
  const int grp = (wn > 0 ? wj0 : j0) / ATT_KPW;
  const size_t gbase = ((size_t)b * Hkv + hk) * (size_t)max_ctx * ATT_D + (size_t)grp * ATT_GROUP;

  // Q as the B operand: lane -> query r16, dims 32*s + 8*q4 .. +8.  Columns
  // r16 >= G load a duplicate query: MFMA columns are independent, and only
  // columns < G are ever stored.
  uint4 qr[4];
  {
    const int g = r16 < G ? r16 : 0;
    const uint4* qp = reinterpret_cast<const uint4*>(q + (part_base + g) * ATT_D + 8 * q4);
#pragma unroll
    for (int s = 0; s < 4; ++s) qr[s] = qp[4 * s];
  }
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
  const u32x4_t* kp = reinterpret_cast<const u32x4_t*>(k_pack + gbase) + lane;
  const u32x4_t* vp = reinterpret_cast<const u32x4_t*>(v_pack + gbase) + lane;
  u32x4_t kr[2][4];
  u32x4_t vr[8];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int s = 0; s < 4; ++s) kr[tt][s] = NT ? __builtin_nontemporal_load(kp + 64 * (4 * tt + s)) : kp[64 * (4 * tt + s)];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) vr[dt] = NT ? __builtin_nontemporal_load(vp + 64 * dt) : vp[64 * dt];
  // keep all loads ahead of the first MFMA (the scheduler would otherwise
  // sink the V loads below the softmax to save registers: 16 KB in flight
  // per wave is the point of this kernel)
  __builtin_amdgcn_sched_barrier(0);

  // ---- scores (raw dot products; scale folded into the exp2)
  f32x4_t sc[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    sc[tt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s)
      sc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, kr[tt][s]),
                                                      __builtin_bit_cast(bf16x8_t, qr[s]), sc[tt], 0, 0, 0);
  }
  // ---- local softmax: lane holds keys 8*q4 + 4*tt + i of query r16
  float p[8];
  float m = -INFINITY;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool ok = (8 * q4 + 4 * tt + i) < wn;
      p[4 * tt + i] = ok ? sc[tt][i] : -INFINITY;
      m = fmaxf(m, p[4 * tt + i]);
    }
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float lsum = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    p[j] = m == -INFINITY ? 0.f : exp2f((p[j] - m) * scale_log2);
    lsum += p[j];
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  bf16x8_t pb;
#pragma unroll
  for (int j = 0; j < 8; ++j) pb[j] = (__bf16)p[j];

  // ---- P.V: C tile dt, lane l, reg i -> dim 16*dt + 4*q4 + i, query r16
  f32x4_t o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
    o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, vr[dt]), pb,
                                                    f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  if (r16 < G) {
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) s_o[wave][r16][16 * dt + 4 * q4 + i] = o[dt][i];
    if (q4 == 0) {
      s_m[wave][r16] = m;
      s_l[wave][r16] = lsum;
    }
  }
  __syncthreads();
  // ---- merge the waves: partial relative to the split max (base-2 scaled)
  for (int idx = t; idx < G * ATT_D; idx += WAVES * 64) {
    const int g = idx / ATT_D, d = idx % ATT_D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) M = fmaxf(M, s_m[w][g]);
    float num = 0.f, den = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < WAVES; ++w) {
        const float mw = s_m[w][g];
        const float f = mw == -INFINITY ? 0.f : exp2f((mw - M) * scale_log2);
        num += f * s_o[w][g][d];
        den += f * s_l[w][g];
      }
    }
    o_part[((part_base + g) * nsplit + split) * ATT_D + d] = num;
    if (d == 0) {
      // the combine kernel works in natural-log units of the scaled scores
      ml_part[((part_base + g) * nsplit + split) * 2 + 0] = M == -INFINITY ? -INFINITY : M * scale_log2 * 0.69314718f;
      ml_part[((part_base + g) * nsplit + split) * 2 + 1] = den;
    }
  }
}

// ------------------------------------ fused decode attention (one launch) --
// decode_attn_mfma_kernel with the neighbouring launches folded in (the
// combine only with COMBINE, see attn_fused_mode for the measured trade-off):
//   * QK-norm + RoPE + KV append (was qk_norm_rope_kv_kernel): waves 0..G-1
//     normalise + rotate the workgroup's G query heads straight from the qkv
//     GEMM output into LDS, wave G the new key, wave G+1 copies the new value
//     (one wave per head, lane l owns the rotate-half pair l, l+64).  Only the
//     workgroup whose split holds the new position writes K/V into the packed
//     cache, and the wave that owns that 32-key group patches its already
//     loaded K/V fragments from LDS (no other workgroup reads that key).
//   * the split combine (was decode_attn_combine_kernel): partials are
//     published with write-through (sc1) stores; after every storing wave's
//     vmcnt(0) and a workgroup barrier, one lane bumps the (b, kv-head)
//     arrival counter (agent-scope atomic); the workgroup whose add returns
//     active-1 is the last one: it resets the counter and merges the active
//     splits with sc1 loads (MI355X_MICROARCH.md, "Hand-offs measured with sc1
//     loads", row 1).  Only splits holding keys arrive (active = ceil(L /
//     SPLIT), the same in every workgroup of the row); empty ones leave.
// The qkv/weight loads are issued before the K/V loads so the prep math does
// not wait behind the 16 KB of K/V (vmcnt retires in order).
template <int G, int WAVES, bool NT, bool COMBINE, bool MULTI>
__global__ void __launch_bounds__(WAVES * 64)
decode_attn_fused_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ qnw,
                         const bf16_t* __restrict__ knw, const int* __restrict__ pos,
                         const int* __restrict__ seqlens, bf16_t* __restrict__ k_pack,
                         bf16_t* __restrict__ v_pack, bf16_t* __restrict__ out,
                         float* __restrict__ o_part, float* __restrict__ ml_part,
                         int* __restrict__ counters, int Hq, int Hkv, int max_ctx, int nsplit,
                         int iters, float scale_log2, float eps, float log2_theta) {
  typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
  typedef __attribute__((ext_vector_type(4))) float f32x4_t;
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
  constexpr int D = ATT_D;
  // keys per split: `iters` 32-key groups per wave (MULTI; 1 otherwise), group
  // i of wave w at position (i * WAVES + w) in the split (the waves read
  // adjacent groups at each step)
  const int SPLIT = WAVES * ATT_KPW * (MULTI ? iters : 1);
  constexpr int DP = D + 1;   // conflict-free partial writes (decode_attn_mfma_kernel)
  const int split = blockIdx.x;
  const int hk = blockIdx.y;
  const int b = blockIdx.z;
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int r16 = lane & 15, q4 = lane >> 4;
  const int L = min(seqlens[b], max_ctx);
  const int p = pos[b];
  const int j0 = split * SPLIT;
  const int n = min(SPLIT, L - j0);
  // splits holding keys: only these take part in the combine (a long cache
  // with a short sequence -- serving -- launches mostly empty splits; they
  // leave at once instead of arriving on the counter)
  const int active = L > 0 ? min(nsplit, (L + SPLIT - 1) / SPLIT) : 1;
  const size_t part_base = ((size_t)b * Hq + (size_t)hk * G);
  __shared__ float s_o[WAVES][G][DP];
  __shared__ float s_m[WAVES][G];
  __shared__ float s_l[WAVES][G];
  // +8 per row: the Q operand reads 16 B of rows 0..G-1 in the same columns
  // (ds_read_b128, bank = dword mod 64): 256-byte rows put them all on bank 0
  __shared__ __attribute__((aligned(16))) bf16_t s_q[G][D + 8];
  __shared__ __attribute__((aligned(16))) bf16_t s_kv[2][D];   // new key (normed, rotated), new value
  __shared__ int s_last;

  if (n > 0) {
    const bool owner = p >= j0 && p < j0 + SPLIT && p < max_ctx;   // this split appends the new key
    // ---- prep loads (issued first)
    // Unconditional loads from clamped, always-valid addresses, issued before
    // the K/V loads: their wait must not sit behind 16 KB of K/V.
    const int row = wave < G + 2 ? wave : -1;   // q heads 0..G-1, k, v
    const int rr = row < 0 ? 0 : row;
    const int hsrc = rr < G ? hk * G + rr : (rr == G ? Hq + hk : Hq + Hkv + hk);
    const bf16_t* src = qkv + (size_t)b * (Hq + 2 * Hkv) * D + (size_t)hsrc * D;
    const bf16_t* nw = rr < G ? qnw : knw;
    const bf16_t raw_x0 = src[lane], raw_x1 = src[lane + 64];
    const bf16_t raw_w0 = nw[lane], raw_w1 = nw[lane + 64];
    __builtin_amdgcn_sched_barrier(0);
    // ---- K/V loads of one 32-key group of this wave (as decode_attn_mfma_kernel);
    // a group past the keys re-reads the split's first group (valid address,
    // every score masked)
    const size_t head = ((size_t)b * Hkv + hk) * (size_t)max_ctx * D;
    // (always_inline: an outlined lambda keeps the fragment arrays in scratch)
    auto load_kv = [&](u32x4_t (&kr)[2][4], u32x4_t (&vr)[8], int it) __attribute__((always_inline)) {
      const int wj0 = j0 + (it * WAVES + wave) * ATT_KPW;
      const int grp = (wj0 < L ? wj0 : j0) / ATT_KPW;
      const u32x4_t* kp = reinterpret_cast<const u32x4_t*>(k_pack + head + (size_t)grp * ATT_GROUP) + lane;
      const u32x4_t* vp = reinterpret_cast<const u32x4_t*>(v_pack + head + (size_t)grp * ATT_GROUP) + lane;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int s = 0; s < 4; ++s)
          kr[tt][s] = NT ? __builtin_nontemporal_load(kp + 64 * (4 * tt + s)) : kp[64 * (4 * tt + s)];
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) vr[dt] = NT ? __builtin_nontemporal_load(vp + 64 * dt) : vp[64 * dt];
    };
    u32x4_t kra[2][4], vra[8], krb[2][4], vrb[8];
    load_kv(kra, vra, 0);
    __builtin_amdgcn_sched_barrier(0);

    // ---- prep math: RMSNorm + NeoX RoPE (q, k), copy (v).  Computed by every
    // wave, outside any branch: a use inside a branch lets LLVM sink the loads
    // into it, behind the K/V loads (then their wait drains all 16 KB).
    float x0 = bf2f(raw_x0), x1 = bf2f(raw_x1);
    {
      const float w0 = bf2f(raw_w0), w1 = bf2f(raw_w1);
      const float ss = wave_sum(x0 * x0 + x1 * x1);
      const float inv = rsqrtf(ss / (float)D + eps);
      const float n0 = x0 * inv * w0, n1 = x1 * inv * w1;
      const float inv_freq = exp2f(-(2.0f * (float)lane / (float)D) * log2_theta);
      float sn, cs;
      sincosf((float)p * inv_freq, &sn, &cs);
      if (rr <= G) {   // q heads and the key; the value is copied as is
        x0 = n0 * cs - n1 * sn;
        x1 = n1 * cs + n0 * sn;
      }
    }
    if (row >= 0 && (row < G || owner)) {
      const bf16_t h0 = f2bf(x0), h1 = f2bf(x1);
      if (row < G) {
        s_q[row][lane] = h0;
        s_q[row][lane + 64] = h1;
      } else {
        const int which = row - G;   // 0 = k, 1 = v
        s_kv[which][lane] = h0;
        s_kv[which][lane + 64] = h1;
        bf16_t* grpp = (which ? v_pack : k_pack) + head + (size_t)(p >> 5) * ATT_GROUP;
        const int k = p & 31;
        if (which == 0) {   // K group [t][s][q][r][e]
          const int kt = (k >> 2) & 1, kr_ = 4 * (k >> 3) + (k & 3);
          grpp[(((kt * 4 + (lane >> 5)) * 4 + ((lane >> 3) & 3)) * 16 + kr_) * 8 + (lane & 7)] = h0;
          grpp[(((kt * 4 + ((lane + 64) >> 5)) * 4 + (((lane + 64) >> 3) & 3)) * 16 + kr_) * 8 + (lane & 7)] = h1;
        } else {            // V group [dt][q][r][e]
          const int kq = k >> 3, ke = k & 7;
          grpp[(((lane >> 4) * 4 + kq) * 16 + (lane & 15)) * 8 + ke] = h0;
          grpp[((((lane + 64) >> 4) * 4 + kq) * 16 + (lane & 15)) * 8 + ke] = h1;
        }
      }
    }
    __syncthreads();

    // ---- Q operand from LDS

    u32x4_t qr[4];
    auto load_q = [&]() __attribute__((always_inline)) {
      const int g = r16 < G ? r16 : 0;
#pragma unroll
      for (int s = 0; s < 4; ++s) qr[s] = *reinterpret_cast<const u32x4_t*>(&s_q[g][32 * s + 8 * q4]);
    };
    load_q();

    // ---- per group: the wave owning the new key patches its fragments (its
    // loads may predate the append), scores, online softmax, P.V accumulated
    // into o[] with the running max and sum rescaled
    f32x4_t o[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, lsum = 0.f;
    auto group = [&](u32x4_t (&kr)[2][4], u32x4_t (&vr)[8], int it) __attribute__((always_inline)) {
      const int wj0 = j0 + (it * WAVES + wave) * ATT_KPW;
      const int wn = min(ATT_KPW, L - wj0);
      if (owner && p >= wj0 && p < wj0 + ATT_KPW) {   // uniform per wave
        // selects, not stores under a lane-dependent branch: those kept the
        // fragment arrays in scratch (112 bytes per lane)
        const bool patch = true;
        const int k = p & 31;
        const int kt = (k >> 2) & 1, kr_ = 4 * (k >> 3) + (k & 3);
        const bool pk = patch && r16 == kr_;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const u32x4_t nk = *reinterpret_cast<const u32x4_t*>(&s_kv[0][32 * s + 8 * q4]);
            kr[tt][s] = (pk && tt == kt) ? nk : kr[tt][s];
          }
        const bool pv = patch && q4 == (k >> 3);
        const int ke = k & 7;
        const unsigned sh = (ke & 1) * 16, keep = 0xffff0000u >> sh;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          const unsigned nv = (unsigned)s_kv[1][16 * dt + r16] << sh;
#pragma unroll
          for (int c = 0; c < 4; ++c) vr[dt][c] = (pv && c == (ke >> 1)) ? ((vr[dt][c] & keep) | nv) : vr[dt][c];
        }
      }
      f32x4_t sc[2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        sc[tt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s)
          sc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, kr[tt][s]),
                                                          __builtin_bit_cast(bf16x8_t, qr[s]), sc[tt], 0, 0, 0);
      }
      float pr[8];
      float mg = -INFINITY;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool ok = (8 * q4 + 4 * tt + i) < wn;
          pr[4 * tt + i] = ok ? sc[tt][i] : -INFINITY;
          mg = fmaxf(mg, pr[4 * tt + i]);
        }
      mg = fmaxf(mg, __shfl_xor(mg, 16, 64));
      mg = fmaxf(mg, __shfl_xor(mg, 32, 64));
      const float mn = fmaxf(m, mg);
      const float a = m == -INFINITY ? 0.f : exp2f((m - mn) * scale_log2);
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pr[j] = mn == -INFINITY ? 0.f : exp2f((pr[j] - mn) * scale_log2);
        ls += pr[j];
      }
      ls += __shfl_xor(ls, 16, 64);
      ls += __shfl_xor(ls, 32, 64);
      lsum = lsum * a + ls;
      m = mn;
      bf16x8_t pb;
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[j] = (__bf16)pr[j];
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, vr[dt]), pb, o[dt] * a, 0, 0,
                                                        0);
    };
    // groups of this wave holding keys: it < nit (later groups are past L)
    const int first = j0 + wave * ATT_KPW;
    const int nit = first < L ? min(iters, (L - first + WAVES * ATT_KPW - 1) / (WAVES * ATT_KPW)) : 0;
    // The first group is processed unconditionally (a wave past the keys sees
    // every score masked: a neutral partial): its loads were issued before the
    // prep math, and a use inside a branch lets LLVM sink them behind the
    // barrier (measured 42 vs 26 us per layer).
    if constexpr (MULTI && WAVES >= 12) {
      // twelve waves, one register buffer (a 768-thread workgroup leaves 168
      // registers per lane, two buffers take 226): the other eleven waves'
      // loads cover each one's round trip per group
#pragma clang loop unroll(disable)
      for (int it = 0; it < nit; ++it) {
        if (it > 0) load_kv(kra, vra, it);
        group(kra, vra, it);
      }
    } else if constexpr (MULTI) {
      // two register buffers: the next group's loads go out before this group's math
      int it = 0;
      while (true) {
        if (it + 1 < nit) load_kv(krb, vrb, it + 1);
        group(kra, vra, it);
        if (++it >= nit) break;
        if (it + 1 < nit) load_kv(kra, vra, it + 1);
        group(krb, vrb, it);
        if (++it >= nit) break;
      }
    } else {
      // one group per wave (iters == 1): one register buffer, ~100 fewer VGPRs,
      // so several workgroups share a CU and hide each other's load latency
      group(kra, vra, 0);
    }
    if (r16 < G) {
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) s_o[wave][r16][16 * dt + 4 * q4 + i] = o[dt][i];
      if (q4 == 0) {
        s_m[wave][r16] = m;
        s_l[wave][r16] = lsum;
      }
    }
    __syncthreads();
    // ---- this split's partial, published write-through (sc1)
    for (int idx = t; idx < G * D; idx += WAVES * 64) {
      const int g = idx / D, d = idx % D;
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) M = fmaxf(M, s_m[w][g]);
      float num = 0.f, den = 0.f;
      if (M != -INFINITY) {
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
          const float mw = s_m[w][g];
          const float f = mw == -INFINITY ? 0.f : exp2f((mw - M) * scale_log2);
          num += f * s_o[w][g][d];
          den += f * s_l[w][g];
        }
      }
      if (!COMBINE && nsplit == 1) {   // one split holds every key: the merged output, no combine
        out[(part_base + g) * D + d] = f2bf(den > 0.f ? num / den : 0.f);
        continue;
      }
      const float mn = M == -INFINITY ? -INFINITY : M * scale_log2 * 0.69314718f;
      float* op = &o_part[((part_base + g) * nsplit + split) * D + d];
      float* mp = &ml_part[((part_base + g) * nsplit + split) * 2];
      if constexpr (COMBINE) {   // write-through: read back by another CU in this launch
        __hip_atomic_store(op, num, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == 0) {
          __hip_atomic_store(mp, mn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(mp + 1, den, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        *op = num;
        if (d == 0) {
          mp[0] = mn;
          mp[1] = den;
        }
      }
    }
  } else if (t < G && split < active) {   // empty split below the combine's count: neutral partial
    float* mp = &ml_part[((part_base + t) * nsplit + split) * 2];
    if constexpr (COMBINE) {
      __hip_atomic_store(mp, -INFINITY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(mp + 1, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      mp[0] = -INFINITY;
      mp[1] = 0.f;
    }
  }
  if constexpr (!COMBINE) return;
  if (split >= active) return;     // uniform per workgroup: no barrier below is split

  // ---- arrival: every storing wave drained, then one add per workgroup
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* cnt = counters + (size_t)b * Hkv + hk;
  if (t == 0) {
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == active - 1;
  }
  __syncthreads();
  if (!s_last) return;
  if (t == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // ready for the next launch
  // ---- last workgroup of (b, kv-head): merge the nsplit partials (sc1
  // loads), 8 splits per batch so each batch is one memory round trip
  // (a loop of dependent loads here costs a round trip per split).
  constexpr int MS = 8;
  for (int idx = t; idx < G * D; idx += WAVES * 64) {
    const int g = idx / D, d = idx % D;
    const size_t base = part_base + g;
    float M = -INFINITY, num = 0.f, den = 0.f;
    for (int s0 = 0; s0 < active; s0 += MS) {
      float mv[MS], lv[MS], ov[MS];
#pragma unroll
      for (int i = 0; i < MS; ++i) {
        const int sp = s0 + i < active ? s0 + i : s0;
        mv[i] = __hip_atomic_load(&ml_part[(base * nsplit + sp) * 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lv[i] = __hip_atomic_load(&ml_part[(base * nsplit + sp) * 2 + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ov[i] = __hip_atomic_load(&o_part[(base * nsplit + sp) * D + d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int i = 0; i < MS; ++i) {
        if (s0 + i >= active || mv[i] == -INFINITY) continue;
        const float nm = fmaxf(M, mv[i]);
        const float a = M == -INFINITY ? 0.f : __expf(M - nm), w = __expf(mv[i] - nm);
        num = num * a + w * ov[i];
        den = den * a + w * lv[i];
        M = nm;
      }
    }
    out[base * D + d] = f2bf(den > 0.f ? num / den : 0.f);
  }
}

// grid = (Hq, B), 128 threads (one per output dim).
__global__ void __launch_bounds__(128)
decode_attn_combine_kernel(const float* __restrict__ o_part, const float* __restrict__ ml_part,
                           bf16_t* __restrict__ out, int Hq, int nsplit, int count,
                           const int* __restrict__ seqlens, int split_keys, int max_ctx) {
  // nsplit = workspace stride, count = splits written (<= nsplit); with
  // seqlens, only the splits holding keys of row b are merged (a cache sized
  // for a long context with a short sequence: most partials are empty)
  // Loads batched 8 splits at a time (one memory round trip per batch) with
  // an online merge; a max pass followed by a weighted pass costs a dependent
  // round trip per split.
  const int h = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const size_t base = (size_t)b * Hq + h;
  constexpr int MS = 8;
  // the first batch of partials is loaded together with seqlens[b] (the
  // workspace holds nsplit entries, so every index < nsplit is in bounds; the
  // count read from seqlens masks the stale ones): one round trip, not two
  float mv[MS], lv[MS], ov[MS];
#pragma unroll
  for (int i = 0; i < MS; ++i) {
    const int sp = i < nsplit ? i : 0;
    mv[i] = ml_part[(base * nsplit + sp) * 2];
    lv[i] = ml_part[(base * nsplit + sp) * 2 + 1];
    ov[i] = o_part[(base * nsplit + sp) * ATT_D + d];
  }
  if (seqlens) {
    const int L = min(seqlens[b], max_ctx);
    count = min(count, L > 0 ? (L + split_keys - 1) / split_keys : 0);
  }
  float M = -INFINITY, num = 0.f, den = 0.f;
  for (int s0 = 0; s0 < count; s0 += MS) {
    if (s0 > 0) {
#pragma unroll
      for (int i = 0; i < MS; ++i) {
        const int sp = s0 + i < count ? s0 + i : s0;
        mv[i] = ml_part[(base * nsplit + sp) * 2];
        lv[i] = ml_part[(base * nsplit + sp) * 2 + 1];
        ov[i] = o_part[(base * nsplit + sp) * ATT_D + d];
      }
    }
#pragma unroll
    for (int i = 0; i < MS; ++i) {
      if (s0 + i >= count || mv[i] == -INFINITY) continue;
      const float nm = fmaxf(M, mv[i]);
      const float a = M == -INFINITY ? 0.f : __expf(M - nm), w = __expf(mv[i] - nm);
      num = num * a + w * ov[i];
      den = den * a + w * lv[i];
      M = nm;
    }
  }
  out[base * ATT_D + d] = f2bf(den > 0.f ? num / den : 0.f);
}

// ---------------------------------------------------------------- SiLU*mul --
__global__ void __launch_bounds__(256)
silu_mul_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ out, int inter, int rows) {
  const int nvec = inter / 8;
  const size_t total = (size_t)rows * nvec;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < total; i += (size_t)gridDim.x * 256ull) {
    const size_t row = i / nvec, vi = i % nvec;
    float g[8], u[8], o[8];
    unpack8(reinterpret_cast<const uint4*>(gu + row * 2 * inter)[vi], g);
    unpack8(reinterpret_cast<const uint4*>(gu + row * 2 * inter + inter)[vi], u);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = g[e] / (1.f + __expf(-g[e])) * u[e];
    reinterpret_cast<uint4*>(out + row * inter)[vi] = pack8(o);
  }
}

// ================================================================ C ABI ====
extern "C" {

int mivgpu_rmsnorm(const void* x, const void* w, void* out, int rows, int dim, float eps,
                   hipStream_t s) {
  if (dim % 8 || dim > 8192 || rows <= 0) return -1;
  hipLaunchKernelGGL(rmsnorm_kernel<false>, dim3(rows), dim3(256), 0, s, (const bf16_t*)x,
                     (bf16_t*)nullptr, (const bf16_t*)w, (bf16_t*)out, dim, eps);
  return (int)hipGetLastError();
}

// out == nullptr: only res and the rows' sums of squares (ss_out[row]).
int mivgpu_embed_rmsnorm(const void* embed, const int64_t* tokens, const void* w, void* res, void* out, int rows,
                         int dim, long long vocab, float eps, float* ss_out, hipStream_t s) {
  if (dim % 8 || dim > 8192 || rows <= 0 || vocab <= 0 || (out == nullptr && ss_out == nullptr)) return -1;
  if (out != nullptr && w == nullptr) return -1;
  hipLaunchKernelGGL(embed_rmsnorm_kernel, dim3(rows), dim3(256), 0, s, (const bf16_t*)embed, tokens,
                     (const bf16_t*)w, (bf16_t*)res, (bf16_t*)out, dim, vocab, eps, ss_out);
  return (int)hipGetLastError();
}

// work: rows * 2 int64-sized words (slots, then tickets as ints), zeroed once;
// every launch leaves it zero.
int mivgpu_decode_tail(const void* logits, int ld, int vocab, int rows, int64_t* tokens, int* pos, int* seqlens,
                       void* work, hipStream_t s) {
  if (rows <= 0 || vocab < 8 * TAIL_SPLIT || ld < vocab || ld % 8 || vocab > TAIL_MAXV * 8 * TAIL_THREADS * TAIL_SPLIT ||
      work == nullptr)
    return -1;
  unsigned long long* slots = (unsigned long long*)work;
  hipLaunchKernelGGL(decode_tail_kernel, dim3(TAIL_SPLIT, rows), dim3(TAIL_THREADS), 0, s, (const bf16_t*)logits, ld,
                     vocab, tokens, pos, seqlens, slots, (int*)(slots + rows));
  return (int)hipGetLastError();
}

int mivgpu_add_rmsnorm(const void* x, void* res, const void* w, void* out, int rows, int dim,
                       float eps, hipStream_t s) {
  if (dim % 8 || dim > 8192 || rows <= 0) return -1;
  hipLaunchKernelGGL(rmsnorm_kernel<true>, dim3(rows), dim3(256), 0, s, (const bf16_t*)x,
                     (bf16_t*)res, (const bf16_t*)w, (bf16_t*)out, dim, eps);
  return (int)hipGetLastError();
}

// Decode-attention implementation, read once per process: 0 = the VALU
// split-K kernel (row-major K and V caches), 8 / 4 = the MFMA kernel with 8
// (default) or 4 waves per workgroup (fragment-packed caches).
// MIVGPU_ATTN_KERNEL=mfma|mfma4|valu; MIVGPU_ATTN_NT=1|0 picks the MFMA
// kernel's K/V load policy (nontemporal by default: every byte is read once).
// Measured (Qwen3-8B, B=32, ctx 1024, profiles/attention_mfma.json):
//   256 / 64 / 32 CUs: VALU 34.6 / 73.1 / 132 us, MFMA-8 nt 28.7 / 52.4 / 92.4 us.
static int attn_impl() {
  static const int impl = [] {
    const char* e = getenv("MIVGPU_ATTN_KERNEL");
    if (!e || !*e || !strcmp(e, "mfma")) return 8;
    if (!strcmp(e, "mfma4")) return 4;
    if (!strcmp(e, "valu")) return 0;
    return 8;
  }();
  return impl;
}

// MIVGPU_ATTN_FUSED (read by mivgpu_decode_attention_fused): 1 (default) =
// prep + attention in one launch, then the combine kernel; 2 = the combine
// folded in as well (last-arriving workgroup).  Measured decode step, batch
// 32 (profiles/README.md section 13): whole GPU 4.93 (unfused) / 4.86 (1) /
// 4.95 ms (2); 64-CU slice 8.88 / 8.87 / 9.65 ms -- the per-workgroup
// arrival atomic (a full memory round trip before the slot frees) and the
// last arriver's merge on the critical path cost more than the combine launch.
static int attn_fused_mode() {
  static const int m = [] {
    const char* e = getenv("MIVGPU_ATTN_FUSED");
    return e && *e ? atoi(e) : 1;
  }();
  return m;
}

static int attn_nt() {
  static const int nt = [] {
    const char* e = getenv("MIVGPU_ATTN_NT");
    return e ? atoi(e) : 1;
  }();
  return nt;
}

// 1 = fragment-packed K/V caches (32-key groups), 0 = row-major [B][Hkv][T][D]
int mivgpu_ops_kv_packed() { return attn_impl() != 0; }

int mivgpu_qk_norm_rope_kv(const void* qkv, const void* qw, const void* kw, const int* pos,
                           void* q_out, void* k_cache, void* v_cache, int B, int Hq, int Hkv,
                           int head_dim, int max_ctx, float eps, float theta, hipStream_t s) {
  if (head_dim != 128 || B <= 0) return -1;
  if (attn_impl()) {
    if (max_ctx % ATT_KPW) return -1;
    hipLaunchKernelGGL((qk_norm_rope_kv_kernel<true, 1>), dim3(B, Hq + 2 * Hkv), dim3(64), 0, s,
                       (const bf16_t*)qkv, (const bf16_t*)qw, (const bf16_t*)kw, pos,
                       (bf16_t*)q_out, (bf16_t*)k_cache, (bf16_t*)v_cache, Hq, Hkv, max_ctx, eps,
                       theta, -1, (bf16_t*)nullptr, (bf16_t*)nullptr, B);
  } else {
    hipLaunchKernelGGL((qk_norm_rope_kv_kernel<false, 1>), dim3(B, Hq + 2 * Hkv), dim3(64), 0, s,
                       (const bf16_t*)qkv, (const bf16_t*)qw, (const bf16_t*)kw, pos,
                       (bf16_t*)q_out, (bf16_t*)k_cache, (bf16_t*)v_cache, Hq, Hkv, max_ctx, eps,
                       theta, -1, (bf16_t*)nullptr, (bf16_t*)nullptr, B);
  }
  return (int)hipGetLastError();
}

// Prefill of one sequence: `rows` prompt tokens (positions pos[0..rows)) into
// cache row cache_b of a [B][Hkv][max_ctx][D] (or packed) cache; q out
// head-grouped [Hkv][G][rows][D], K/V also plain [Hkv][rows][D] (may be null).
int mivgpu_prefill_qk_norm_rope_kv(const void* qkv, const void* qw, const void* kw, const int* pos,
                                   void* q_out, void* k_plain, void* v_plain, void* k_cache, void* v_cache,
                                   int rows, int cache_b, int Hq, int Hkv, int head_dim, int max_ctx, float eps,
                                   float theta, hipStream_t s) {
  if (head_dim != 128 || rows <= 0 || cache_b < 0 || Hkv <= 0 || Hq % Hkv) return -1;
  static const bool vec = [] {
    const char* e = getenv("MIVGPU_PREFILL_QK");   // "8": the per-token kernel (A/B)
    return !(e && !strcmp(e, "8"));
  }();
  if (vec) {
    if (attn_impl() && max_ctx % ATT_KPW) return -1;
    const dim3 grid((rows + QP_TPW - 1) / QP_TPW, Hq + 2 * Hkv);
    const float l2t = log2f(theta);
    if (attn_impl())
      hipLaunchKernelGGL((qk_prefill_vec_kernel<true>), grid, dim3(64), 0, s, (const bf16_t*)qkv, (const bf16_t*)qw,
                         (const bf16_t*)kw, pos, (bf16_t*)q_out, (bf16_t*)k_cache, (bf16_t*)v_cache, Hq, Hkv,
                         max_ctx, eps, l2t, cache_b, (bf16_t*)k_plain, (bf16_t*)v_plain, rows);
    else
      hipLaunchKernelGGL((qk_prefill_vec_kernel<false>), grid, dim3(64), 0, s, (const bf16_t*)qkv,
                         (const bf16_t*)qw, (const bf16_t*)kw, pos, (bf16_t*)q_out, (bf16_t*)k_cache,
                         (bf16_t*)v_cache, Hq, Hkv, max_ctx, eps, l2t, cache_b, (bf16_t*)k_plain,
                         (bf16_t*)v_plain, rows);
    return (int)hipGetLastError();
  }
  constexpr int kPrefillTpw = 8;
  const int grid_x = (rows + kPrefillTpw - 1) / kPrefillTpw;
  if (attn_impl()) {
    if (max_ctx % ATT_KPW) return -1;
    hipLaunchKernelGGL((qk_norm_rope_kv_kernel<true, kPrefillTpw>), dim3(grid_x, Hq + 2 * Hkv), dim3(64), 0, s,
                       (const bf16_t*)qkv, (const bf16_t*)qw, (const bf16_t*)kw, pos, (bf16_t*)q_out,
                       (bf16_t*)k_cache, (bf16_t*)v_cache, Hq, Hkv, max_ctx, eps, theta, cache_b,
                       (bf16_t*)k_plain, (bf16_t*)v_plain, rows);
  } else {
    hipLaunchKernelGGL((qk_norm_rope_kv_kernel<false, kPrefillTpw>), dim3(grid_x, Hq + 2 * Hkv), dim3(64), 0, s,
                       (const bf16_t*)qkv, (const bf16_t*)qw, (const bf16_t*)kw, pos, (bf16_t*)q_out,
                       (bf16_t*)k_cache, (bf16_t*)v_cache, Hq, Hkv, max_ctx, eps, theta, cache_b,
                       (bf16_t*)k_plain, (bf16_t*)v_plain, rows);
  }
  return (int)hipGetLastError();
}

extern "C" int mivgpu_ops_visible_cus();

// Workspace: o_part = B*Hq*nsplit*128 floats, ml_part = B*Hq*nsplit*2 floats.
int mivgpu_decode_attention(const void* q, const void* k_cache, const void* v_cache,
                            const int* seqlens, void* out, void* o_part, void* ml_part, int B,
                            int Hq, int Hkv, int head_dim, int max_ctx, int nsplit, float scale,
                            hipStream_t s) {
  if (head_dim != ATT_D || Hq % Hkv || nsplit <= 0 || B <= 0) return -1;
  const int G = Hq / Hkv;
  dim3 grid(nsplit, Hkv, B);
  if (attn_impl()) {
    const int waves = attn_impl();
    // the workspace must cover every key: nsplit * split >= max_ctx
    if (max_ctx % ATT_KPW || (long long)nsplit * waves * ATT_KPW < max_ctx) return -1;
    const bool nt = attn_nt() != 0;
    const float scale_log2 = scale * 1.44269504f;
#define MIVGPU_ATTN_MFMA(GG, WW, NN)                                                                      \
  hipLaunchKernelGGL((decode_attn_mfma_kernel<GG, WW, NN>), grid, dim3(WW * 64), 0, s, (const bf16_t*)q, \
                     (const bf16_t*)k_cache, (const bf16_t*)v_cache, seqlens, (float*)o_part,             \
                     (float*)ml_part, Hq, Hkv, max_ctx, nsplit, scale_log2)
#define MIVGPU_ATTN_MFMA_G(GG)                                  \
  case GG:                                                      \
    if (waves == 8) {                                           \
      if (nt) MIVGPU_ATTN_MFMA(GG, 8, true);                    \
      else MIVGPU_ATTN_MFMA(GG, 8, false);                      \
    } else {                                                    \
      if (nt) MIVGPU_ATTN_MFMA(GG, 4, true);                    \
      else MIVGPU_ATTN_MFMA(GG, 4, false);                      \
    }                                                           \
    break;
    switch (G) {
      MIVGPU_ATTN_MFMA_G(1)
      MIVGPU_ATTN_MFMA_G(2)
      MIVGPU_ATTN_MFMA_G(4)
      MIVGPU_ATTN_MFMA_G(8)
      MIVGPU_ATTN_MFMA_G(16)
      default:
        return -1;
    }
#undef MIVGPU_ATTN_MFMA_G
#undef MIVGPU_ATTN_MFMA
    hipLaunchKernelGGL(decode_attn_combine_kernel, dim3(Hq, B), dim3(ATT_D), 0, s,
                       (const float*)o_part, (const float*)ml_part, (bf16_t*)out, Hq, nsplit, nsplit, seqlens,
                       waves * ATT_KPW, max_ctx);
    return (int)hipGetLastError();
  }
  // Load scheduling variant (see the kernel); MIVGPU_ATTN_PF overrides for experiments.
  static const int pf_env = [] {
    const char* e = getenv("MIVGPU_ATTN_PF");
    return e ? atoi(e) : -1;
  }();
  // PF=0 keeps the most workgroups resident (5 per CU at G=4): best when the
  // whole grid fits at once (full MI355X).  When a CU partition must run many
  // rounds of workgroups (a 64- or 32-CU slice), PF=2 hides HBM latency
  // inside each workgroup: 90 -> 73 us at 64 CUs, 160 -> 132 us at 32 CUs
  // (bench/attention.py, profiles/attention_variants.json).
  static const int cus = mivgpu_ops_visible_cus();
  const int resident0 = G <= 2 ? 8 : (G == 4 ? 5 : 3);
  const int pf = pf_env >= 0 ? pf_env : ((long long)grid.x * grid.y * grid.z > (long long)cus * resident0 ? 2 : 0);
#define MIVGPU_ATTN_LAUNCH(GG, PP)                                                                          \
  hipLaunchKernelGGL((decode_attn_partial_kernel<GG, PP>), grid, dim3(256), 0, s, (const bf16_t*)q,        \
                     (const bf16_t*)k_cache, (const bf16_t*)v_cache, seqlens, (float*)o_part,              \
                     (float*)ml_part, Hq, Hkv, max_ctx, nsplit, scale)
#define MIVGPU_ATTN_G(GG)                            \
  case GG:                                           \
    if (pf == 1) MIVGPU_ATTN_LAUNCH(GG, 1);          \
    else if (pf == 2) MIVGPU_ATTN_LAUNCH(GG, 2);     \
    else MIVGPU_ATTN_LAUNCH(GG, 0);                  \
    break;
  switch (G) {
    MIVGPU_ATTN_G(1)
    MIVGPU_ATTN_G(2)
    MIVGPU_ATTN_G(4)
    MIVGPU_ATTN_G(8)
    default:
      return -1;
  }
#undef MIVGPU_ATTN_G
#undef MIVGPU_ATTN_LAUNCH
  hipLaunchKernelGGL(decode_attn_combine_kernel, dim3(Hq, B), dim3(ATT_D), 0, s,
                     (const float*)o_part, (const float*)ml_part, (bf16_t*)out, Hq, nsplit, nsplit, seqlens,
                     ATT_SPLIT, max_ctx);
  return (int)hipGetLastError();
}

// One-launch decode attention step for one layer (fragment-packed caches only):
// QK-norm + RoPE of the G query heads and the new key, KV append at pos[b],
// GQA attention over seqlens[b] keys, split combine.  counters: B*Hkv ints,
// zero before the first call; every launch leaves them zero.  Launches that
// share `counters` must not run concurrently.
int mivgpu_decode_attention_fused(const void* qkv, const void* q_norm_w, const void* k_norm_w,
                                  const int* pos, const int* seqlens, void* k_cache, void* v_cache,
                                  void* out, void* o_part, void* ml_part, int* counters, int B, int Hq,
                                  int Hkv, int head_dim, int max_ctx, int nsplit, float scale, float eps,
                                  float theta, int defer_combine, hipStream_t s) {
  if (!attn_impl() || head_dim != ATT_D || Hq % Hkv || nsplit <= 0 || B <= 0) return -1;
  const int G = Hq / Hkv;
  const int waves = attn_impl();
  if (max_ctx % ATT_KPW || G + 2 > waves) return -1;
  // One split per (b, kv-head) with four query heads per kv-head: twelve-wave
  // workgroups (one per CU at batch 32 x 8 kv-heads; 158 VGPRs, three waves
  // per SIMD -- sixteen spilled) that merge their waves in LDS and write the
  // output, no partials and no combine launch: 25.5 us per layer vs 26.0 +
  // 4.9 for five 8-wave splits + combine (profiles/round6/w12/).
  // MIVGPU_ATTN_W12=0 keeps the 8-wave kernel.
  static const bool w12 = [] {
    const char* e = getenv("MIVGPU_ATTN_W12");
    return !e || atoi(e) != 0;
  }();
  if (w12 && nsplit == 1 && G == 4 && !defer_combine) {
    const int iters12 = (max_ctx + 12 * ATT_KPW - 1) / (12 * ATT_KPW);
    const float sl2 = scale * 1.44269504f, lt = log2f(theta);
    hipLaunchKernelGGL((decode_attn_fused_kernel<4, 12, true, false, true>), dim3(1, Hkv, B), dim3(768), 0, s,
                       (const bf16_t*)qkv, (const bf16_t*)q_norm_w, (const bf16_t*)k_norm_w, pos, seqlens,
                       (bf16_t*)k_cache, (bf16_t*)v_cache, (bf16_t*)out, (float*)o_part, (float*)ml_part, counters,
                       Hq, Hkv, max_ctx, 1, iters12, sl2, eps, lt);
    return (int)hipGetLastError();
  }
  // 32-key groups per wave so that nsplit splits cover max_ctx; nsplit = 1
  // (one workgroup per (b, kv-head), each wave looping over its groups) writes
  // the output itself and needs no combine
  const int per = waves * ATT_KPW;
  const int iters = (int)((max_ctx + (long long)nsplit * per - 1) / ((long long)nsplit * per));
  const bool nt = attn_nt() != 0;
  const float scale_log2 = scale * 1.44269504f;
  const float log2_theta = log2f(theta);
  dim3 grid(nsplit, Hkv, B);
  // defer_combine: leave the partials for a consumer that combines them
  // itself (the o_proj GEMM's X staging, mivgpu_skinny_gemm_norm_xcomb)
  const bool comb = attn_fused_mode() >= 2 && nsplit > 1 && !defer_combine;
#define MIVGPU_ATTN_FUSED3(GG, WW, NN, CC, MM)                                                                 \
  hipLaunchKernelGGL((decode_attn_fused_kernel<GG, WW, NN, CC, MM>), grid, dim3(WW * 64), 0, s,              \
                     (const bf16_t*)qkv, (const bf16_t*)q_norm_w, (const bf16_t*)k_norm_w, pos, seqlens,     \
                     (bf16_t*)k_cache, (bf16_t*)v_cache, (bf16_t*)out, (float*)o_part, (float*)ml_part,      \
                     counters, Hq, Hkv, max_ctx, nsplit, iters, scale_log2, eps, log2_theta)
#define MIVGPU_ATTN_FUSED2(GG, WW, NN, CC)                  \
  do {                                                      \
    if (iters > 1) MIVGPU_ATTN_FUSED3(GG, WW, NN, CC, true); \
    else MIVGPU_ATTN_FUSED3(GG, WW, NN, CC, false);         \
  } while (0)
#define MIVGPU_ATTN_FUSED(GG, WW, NN)                      \
  do {                                                     \
    if (comb) MIVGPU_ATTN_FUSED2(GG, WW, NN, true);        \
    else MIVGPU_ATTN_FUSED2(GG, WW, NN, false);            \
  } while (0)
#define MIVGPU_ATTN_FUSED_G(GG)                                  \
  case GG:                                                       \
    if (waves == 8) {                                            \
      if (nt) MIVGPU_ATTN_FUSED(GG, 8, true);                    \
      else MIVGPU_ATTN_FUSED(GG, 8, false);                      \
    } else {                                                     \
      if (nt) MIVGPU_ATTN_FUSED(GG, 4, true);                    \
      else MIVGPU_ATTN_FUSED(GG, 4, false);                      \
    }                                                            \
    break;
  switch (G) {
    MIVGPU_ATTN_FUSED_G(1)
    MIVGPU_ATTN_FUSED_G(2)
    MIVGPU_ATTN_FUSED_G(4)
    case 6:
      if (waves != 8) return -1;
      if (nt) MIVGPU_ATTN_FUSED(6, 8, true);
      else MIVGPU_ATTN_FUSED(6, 8, false);
      break;
    default:
      return -1;
  }
#undef MIVGPU_ATTN_FUSED_G
#undef MIVGPU_ATTN_FUSED
#undef MIVGPU_ATTN_FUSED2
#undef MIVGPU_ATTN_FUSED3
  if (!comb && nsplit > 1 && !defer_combine)
    hipLaunchKernelGGL(decode_attn_combine_kernel, dim3(Hq, B), dim3(ATT_D), 0, s, (const float*)o_part,
                       (const float*)ml_part, (bf16_t*)out, Hq, nsplit, nsplit, seqlens, iters * per, max_ctx);
  return (int)hipGetLastError();
}

int mivgpu_silu_mul(const void* gate_up, void* out, int rows, int inter, hipStream_t s) {
  if (inter % 8 || rows <= 0) return -1;
  const size_t total = (size_t)rows * (inter / 8);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(silu_mul_kernel, dim3(blocks), dim3(256), 0, s, (const bf16_t*)gate_up,
                     (bf16_t*)out, inter, rows);
  return (int)hipGetLastError();
}

int mivgpu_ops_attn_split() { return attn_impl() ? attn_impl() * ATT_KPW : ATT_SPLIT; }

// CUs this process can run on: the HSA_CU_MASK bits of the current device
// (a vGPU slice's partition, "i:lo-hi,..;j:..") or, without a mask, the
// device's CU count.  Kernel variants whose best schedule depends on the
// number of resident workgroups per CU key off this.
int mivgpu_ops_visible_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const char* m = getenv("HSA_CU_MASK");
  if (m && *m) {
    const char* p = m;
    while (*p) {
      char* end = nullptr;
      const long idx = strtol(p, &end, 10);
      if (end == p || *end != ':') break;
      p = end + 1;
      int count = 0;
      while (*p && *p != ';') {
        const long lo = strtol(p, &end, 10);
        if (end == p) break;
        long hi = lo;
        p = end;
        if (*p == '-') {
          hi = strtol(p + 1, &end, 10);
          p = end;
        }
        if (hi >= lo) count += (int)(hi - lo + 1);
        if (*p == ',') ++p;
      }
      if (idx == dev && count > 0) return count;
      if (*p == ';') ++p;
    }
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  return cus;
}

}  // extern "C"
