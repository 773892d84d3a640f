// Hardware placement probe (gfx950): where do workgroups land under a CU mask?
//
// Each one-wave workgroup records HW_REG_HW_ID (wave/simd/cu/sh/se fields) and
// HW_REG_XCC_ID.  Launched under different HSA_CU_MASK values it maps the
// mask's logical CU indices onto XCDs / shader engines, which is what the
// device plugin needs to hand out XCD-aligned CU ranges (per-XCD L2 isolation:
// MI355X_MICROARCH.md "XCD").  The kernel spins ~20 us so the dispatcher has
// to spread the grid over every enabled CU.
#include <hip/hip_runtime.h>
#include <stdint.h>

// s_getreg encodings: (size-1) << 11 | offset << 6 | hwreg id
#define HWREG_FULL(id) ((31 << 11) | (0 << 6) | (id))

extern "C" __global__ void __launch_bounds__(64) mivgpu_hwid_probe_kernel(uint32_t* out) {
  if (threadIdx.x == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg(HWREG_FULL(4));   // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg(HWREG_FULL(20)); // HW_REG_XCC_ID
    out[blockIdx.x * 2 + 0] = hw;
    out[blockIdx.x * 2 + 1] = xcc;
  }
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(10);
}

extern "C" int mivgpu_hwid_probe(uint32_t* out_dev, int blocks, hipStream_t s) {
  if (blocks <= 0 || blocks > (1 << 20)) return -1;
  hipLaunchKernelGGL(mivgpu_hwid_probe_kernel, dim3(blocks), dim3(64), 0, s, out_dev);
  return (int)hipGetLastError();
}
