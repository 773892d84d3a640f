// Synthetic load generators for isolation / overhead measurement (gfx950).
//
// a compute-bound matrix-core load and a memory-bound
// stream, used by shim/probe.py to check CU partitions, the governor's duty
// cycle and the shim's per-launch overhead with code whose work is known
// exactly (no library heuristics in between).
//
//   mivgpu_mfma_burn   each wave runs `iters` rounds of 8 independent
//                      v_mfma_f32_32x32x16_bf16 chains (register-only, so the
//                      matrix pipe is the only bottleneck); 32*32*16*2 FLOP
//                      per MFMA.  The chains' sums are written out so nothing
//                      is dead code.
//   mivgpu_stream_copy dst = src, 16-byte non-temporal loads/stores, grid
//                      stride over the whole buffer (HBM read + write).
//   mivgpu_stream_read sum of all 32-bit words of src as uint64 (HBM read only),
//                      one atomic per wave; exact, so tests can check it.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;

namespace {

constexpr int CHAINS = 8;

__global__ void __launch_bounds__(256) mfma_burn_kernel(float* __restrict__ out, int iters, unsigned seed) {
  const int lane = threadIdx.x & 63;
  u32x4_t a, b;
  // small bf16 values (|x| < 2^-6) so 32k-long chains stay finite
  const unsigned v = 0x3c003c00u ^ ((seed + lane) & 0x007f007fu);
  a = (u32x4_t){v, v ^ 0x10001u, v ^ 0x20002u, v ^ 0x30003u};
  b = (u32x4_t){v ^ 0x40004u, v ^ 0x50005u, v ^ 0x60006u, v ^ 0x70007u};
  f32x16_t acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[c][e] = 0.f;
  const bf16x8_t A = __builtin_bit_cast(bf16x8_t, a), B = __builtin_bit_cast(bf16x8_t, b);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int e = 0; e < 16; ++e) s += acc[c][e];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) stream_copy_kernel(const u32x4_t* __restrict__ src, u32x4_t* __restrict__ dst,
                                                          size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4_t v0 = __builtin_nontemporal_load(src + i);
    const u32x4_t v1 = __builtin_nontemporal_load(src + i + stride);
    const u32x4_t v2 = __builtin_nontemporal_load(src + i + 2 * stride);
    const u32x4_t v3 = __builtin_nontemporal_load(src + i + 3 * stride);
    __builtin_nontemporal_store(v0, dst + i);
    __builtin_nontemporal_store(v1, dst + i + stride);
    __builtin_nontemporal_store(v2, dst + i + 2 * stride);
    __builtin_nontemporal_store(v3, dst + i + 3 * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__device__ __forceinline__ unsigned long long wsum(const u32x4_t& v) {
  return (unsigned long long)v.x + v.y + v.z + v.w;
}

__global__ void __launch_bounds__(256) stream_read_kernel(const u32x4_t* __restrict__ src, size_t n16,
                                                          unsigned long long* __restrict__ out) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long acc = 0;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4_t v0 = __builtin_nontemporal_load(src + i);
    const u32x4_t v1 = __builtin_nontemporal_load(src + i + stride);
    const u32x4_t v2 = __builtin_nontemporal_load(src + i + 2 * stride);
    const u32x4_t v3 = __builtin_nontemporal_load(src + i + 3 * stride);
    acc += wsum(v0) + wsum(v1) + wsum(v2) + wsum(v3);
  }
  for (; i < n16; i += stride) acc += wsum(__builtin_nontemporal_load(src + i));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

}  // namespace

extern "C" {

// FLOPs one mivgpu_mfma_burn launch performs.
double mivgpu_mfma_burn_flops(int blocks, int iters) {
  return (double)blocks * 4 /*waves*/ * CHAINS * iters * (32.0 * 32 * 16 * 2);
}

int mivgpu_mfma_burn(float* out, int blocks, int iters, unsigned seed, hipStream_t s) {
  if (blocks <= 0 || iters <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mfma_burn_kernel, dim3(blocks), dim3(256), 0, s, out, iters, seed);
  return (int)hipGetLastError();
}

int mivgpu_stream_copy(const void* src, void* dst, long long bytes, int blocks, hipStream_t s) {
  if (bytes <= 0 || (bytes & 15) || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15)) return (int)hipErrorInvalidValue;
  if (blocks <= 0) blocks = 256 * 8;  // 8 workgroups per CU
  hipLaunchKernelGGL(stream_copy_kernel, dim3(blocks), dim3(256), 0, s, (const u32x4_t*)src, (u32x4_t*)dst,
                     (size_t)bytes / 16);
  return (int)hipGetLastError();
}

int mivgpu_stream_read(const void* src, long long bytes, unsigned long long* out, int blocks, hipStream_t s) {
  if (bytes <= 0 || (bytes & 15) || ((uintptr_t)src & 15)) return (int)hipErrorInvalidValue;
  if (blocks <= 0) blocks = 256 * 8;
  hipLaunchKernelGGL(stream_read_kernel, dim3(blocks), dim3(256), 0, s, (const u32x4_t*)src, (size_t)bytes / 16,
                     out);
  return (int)hipGetLastError();
}

}  // extern "C"
