// CPU stand-in for libamdhip64.so used ONLY by the CPU test-suite to exercise
// libmivgpu.so's interposition, accounting and virtualisation logic without a
// GPU.  It exports the subset of the HIP runtime the shim resolves, under the
// same ELF version nodes as the real library (mock_amdhip.map), so a driver
// linked against it carries exactly the versioned references a PyTorch binary
// carries.  "Device memory" is host malloc bounded by MOCKHIP_TOTAL_MIB.
#include <hip/hip_runtime_api.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <mutex>
#include <unordered_map>

#define EXPORT extern "C" __attribute__((visibility("default")))

namespace {
std::mutex mu;
std::unordered_map<void*, size_t> allocs;
size_t used_bytes[16] = {0};
thread_local int cur_dev = 0;
std::atomic<unsigned long long> launches{0};

size_t total_bytes() {
  const char* t = getenv("MOCKHIP_TOTAL_MIB");
  size_t mib = t ? strtoull(t, nullptr, 10) : 65536;
  return mib << 20;
}
int ndev() {
  const char* n = getenv("MOCKHIP_DEVICES");
  return n ? atoi(n) : 1;
}
// KFD's per-process VRAM file, simulated when MOCKHIP_KFD_SYSFS is set:
// <root>/proc/<MOCKHIP_KFD_PID or getpid()>/vram_<MOCKHIP_KFD_GPU_ID + dev>
// = runtime "context" bytes (mockhip_set_kfd_context) + live allocations.
// MOCKHIP_KFD_PID != getpid() stands for a container's pid namespace.
size_t kfd_context[16] = {0};
// Simulated runtime VRAM of loaded code objects (MOCKHIP_MODULES=1):
// MOCKHIP_MODULE_KIB per module (default 2048, one 2 MiB fragment), part of
// the KFD per-process total like the runtime's real code-object allocations.
size_t module_bytes[16] = {0};
std::unordered_map<void*, size_t> modules;
size_t module_cost() {
  const char* k = getenv("MOCKHIP_MODULE_KIB");
  return (size_t)(k ? strtoull(k, nullptr, 10) : 2048) << 10;
}

void kfd_publish_locked(int dev) {
  const char* root = getenv("MOCKHIP_KFD_SYSFS");
  if (!root) return;
  const char* gid = getenv("MOCKHIP_KFD_GPU_ID");
  const char* kp = getenv("MOCKHIP_KFD_PID");
  const int pid = kp ? atoi(kp) : (int)getpid();
  char path[512];
  snprintf(path, sizeof(path), "%s/proc", root);
  mkdir(path, 0755);
  snprintf(path, sizeof(path), "%s/proc/%d", root, pid);
  mkdir(path, 0755);
  snprintf(path, sizeof(path), "%s/proc/%d/vram_%d", root, pid, (gid ? atoi(gid) : 1) + dev);
  FILE* f = fopen(path, "w");
  if (!f) return;
  fprintf(f, "%zu\n", kfd_context[dev] + used_bytes[dev] + module_bytes[dev]);
  fclose(f);
  // with MOCKHIP_KFD_OCC=1, also the per-process wave count the occupancy
  // sampler reads: one CU-unit per 64 MiB in use (moves with the traffic)
  if (!getenv("MOCKHIP_KFD_OCC")) return;
  snprintf(path, sizeof(path), "%s/proc/%d/stats_%d", root, pid, (gid ? atoi(gid) : 1) + dev);
  mkdir(path, 0755);
  snprintf(path, sizeof(path), "%s/proc/%d/stats_%d/cu_occupancy", root, pid, (gid ? atoi(gid) : 1) + dev);
  f = fopen(path, "w");
  if (!f) return;
  fprintf(f, "%zu\n", used_bytes[dev] >> 26);
  fclose(f);
}
hipError_t do_alloc(void** p, size_t sz) {
  std::lock_guard<std::mutex> lk(mu);
  if (used_bytes[cur_dev] + sz > total_bytes()) return hipErrorOutOfMemory;
  // Never touch the pages: tests allocate "GiB" without committing RAM.
  void* m = malloc(sz < 64 ? 64 : (sz > (1u << 20) ? 4096 : sz));
  if (!m) return hipErrorOutOfMemory;
  allocs[m] = sz;
  used_bytes[cur_dev] += sz;
  kfd_publish_locked(cur_dev);
  *p = m;
  return hipSuccess;
}
hipError_t do_free(void* p) {
  if (!p) return hipSuccess;
  std::lock_guard<std::mutex> lk(mu);
  auto it = allocs.find(p);
  if (it == allocs.end()) return hipErrorInvalidValue;
  used_bytes[cur_dev] -= it->second;
  kfd_publish_locked(cur_dev);
  allocs.erase(it);
  free(p);
  return hipSuccess;
}
}  // namespace

EXPORT void mockhip_set_kfd_context(unsigned long long mib) {
  std::lock_guard<std::mutex> lk(mu);
  kfd_context[cur_dev] = (size_t)mib << 20;
  kfd_publish_locked(cur_dev);
}
EXPORT hipError_t hipGetDeviceCount(int* n) { *n = ndev(); return hipSuccess; }
EXPORT hipError_t hipGetDevice(int* d) { *d = cur_dev; return hipSuccess; }
EXPORT hipError_t hipSetDevice(int d) {
  if (d < 0 || d >= ndev()) return hipErrorInvalidDevice;
  cur_dev = d;
  return hipSuccess;
}
EXPORT hipError_t hipMalloc(void** p, size_t sz) { return do_alloc(p, sz); }
EXPORT hipError_t hipExtMallocWithFlags(void** p, size_t sz, unsigned int) { return do_alloc(p, sz); }
EXPORT hipError_t hipMallocManaged(void** p, size_t sz, unsigned int) { return do_alloc(p, sz); }
EXPORT hipError_t hipMallocAsync(void** p, size_t sz, hipStream_t) { return do_alloc(p, sz); }
EXPORT hipError_t hipMallocFromPoolAsync(void** p, size_t sz, hipMemPool_t, hipStream_t) {
  return do_alloc(p, sz);
}
EXPORT hipError_t hipMallocPitch(void** p, size_t* pitch, size_t w, size_t h) {
  *pitch = (w + 255) & ~size_t(255);
  return do_alloc(p, *pitch * h);
}
EXPORT hipError_t hipMemAllocPitch(hipDeviceptr_t* p, size_t* pitch, size_t w, size_t h, unsigned int) {
  *pitch = (w + 255) & ~size_t(255);
  return do_alloc(reinterpret_cast<void**>(p), *pitch * h);
}
EXPORT hipError_t hipFree(void* p) { return do_free(p); }
EXPORT hipError_t hipFreeAsync(void* p, hipStream_t) { return do_free(p); }
EXPORT hipError_t hipMemCreate(hipMemGenericAllocationHandle_t* h, size_t sz,
                               const hipMemAllocationProp*, unsigned long long) {
  void* p = nullptr;
  hipError_t rc = do_alloc(&p, sz);
  *h = reinterpret_cast<hipMemGenericAllocationHandle_t>(p);
  return rc;
}
EXPORT hipError_t hipMemRelease(hipMemGenericAllocationHandle_t h) {
  return do_free(reinterpret_cast<void*>(h));
}
EXPORT hipError_t hipHostMalloc(void** p, size_t sz, unsigned int) {
  *p = malloc(sz < 64 ? 64 : (sz > (1u << 20) ? 4096 : sz));
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
EXPORT hipError_t hipHostFree(void* p) { free(p); return hipSuccess; }
EXPORT hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned int) { *d = h; return hipSuccess; }
EXPORT hipError_t hipMemset(void* p, int v, size_t n) { (void)p; (void)v; (void)n; return hipSuccess; }
EXPORT hipError_t hipMemGetInfo(size_t* f, size_t* t) {
  std::lock_guard<std::mutex> lk(mu);
  *t = total_bytes();
  *f = total_bytes() - used_bytes[cur_dev];
  return hipSuccess;
}
EXPORT hipError_t hipDeviceTotalMem(size_t* b, hipDevice_t) { *b = total_bytes(); return hipSuccess; }
EXPORT hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* p, int) {
  memset(p, 0, sizeof(*p));
  strcpy(p->name, "AMD Instinct MI355X (mock)");
  p->totalGlobalMem = total_bytes();
  p->multiProcessorCount = 256;
  return hipSuccess;
}
EXPORT hipError_t hipGetDevicePropertiesR0000(void* p, int) {
  memset(p, 0, 512);
  strcpy(static_cast<char*>(p), "AMD Instinct MI355X (mock)");
  *reinterpret_cast<size_t*>(static_cast<char*>(p) + 256) = total_bytes();
  return hipSuccess;
}
// PCI location of mock device d: domain 0, bus 0x75 + 0x10 * d, device 0
// (what the shim matches against the KFD topology in context accounting).
EXPORT hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t a, int dev) {
  *v = a == hipDeviceAttributePciBusId ? 0x75 + 0x10 * dev : 0;
  return hipSuccess;
}
EXPORT hipError_t hipLaunchKernel(const void*, dim3, dim3, void**, size_t, hipStream_t) {
  launches++;
  return hipSuccess;
}
// MOCKHIP_GOVERNOR=1: the governor's code object "loads" and its two kernels
// run on the host at launch (the clock kernel writes CLOCK_MONOTONIC, the gate
// counts itself done in the host stats without holding), so the shim's whole
// gating path -- enqueue, idle stamper, occupancy sampler -- runs on the CPU
// (race tests under ThreadSanitizer).  Otherwise no code object loads.
enum MockFn : uintptr_t { kNoFn = 0, kGateFn = 0x6a7e, kClockFn = 0xc10c };
long long mono_now() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (long long)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}
// MOCKHIP_GATE_HOLD=1: the gate holds like governor.hip host_bucket_gate
// (the launching thread stands in for the stream): while the host bucket is
// in debt, up to max_hold, publishing the same hold markers.
void mock_host_bucket_hold(unsigned long long* hs, int slot, long long max_hold) {
  long long* h = reinterpret_cast<long long*>(hs);
  constexpr int kTokens = 7, kEnd = 8 + 128 * 8, kStart = kEnd + 64, kCum = kEnd + 128;
  if (slot < 0 || slot >= 64 || __atomic_load_n(&h[kTokens], __ATOMIC_RELAXED) >= 0) return;
  const long long t0 = mono_now();
  long long t = t0;
  __atomic_store_n(&h[kStart + slot], t0, __ATOMIC_RELAXED);
  __atomic_store_n(&h[kEnd + slot], t0 + max_hold, __ATOMIC_RELEASE);
  while (__atomic_load_n(&h[kTokens], __ATOMIC_RELAXED) < 0 && t < t0 + max_hold) {
    usleep(20);
    t = mono_now();
  }
  __atomic_store_n(&h[kEnd + slot], t, __ATOMIC_RELAXED);
  __atomic_store_n(&h[kCum + slot], __atomic_load_n(&h[kCum + slot], __ATOMIC_RELAXED) + (t - t0), __ATOMIC_RELEASE);
  __atomic_fetch_add(&hs[1], (unsigned long long)(t - t0), __ATOMIC_RELAXED);   // held_total_ns
}
bool mock_governor() { return getenv("MOCKHIP_GOVERNOR") != nullptr; }
EXPORT hipError_t hipModuleLaunchKernel(hipFunction_t f, unsigned, unsigned, unsigned, unsigned,
                                        unsigned, unsigned, unsigned, hipStream_t, void** args, void**) {
  launches++;
  const uintptr_t fn = reinterpret_cast<uintptr_t>(f);
  if (fn == kClockFn && args) {
    long long* out = *static_cast<long long**>(args[0]);
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    __atomic_store_n(out, (long long)ts.tv_sec * 1000000000ll + ts.tv_nsec, __ATOMIC_RELEASE);
  } else if (fn == kGateFn && args) {
    unsigned long long* hs = *static_cast<unsigned long long**>(args[1]);
    const int slot = *static_cast<int*>(args[3]);
    const long long max_hold = *static_cast<long long*>(args[6]);
    const unsigned flags = *static_cast<unsigned*>(args[8]);
    if (hs && (flags & 2u) && getenv("MOCKHIP_GATE_HOLD")) mock_host_bucket_hold(hs, slot, max_hold);
    if (hs) __atomic_fetch_add(&hs[2], 1ull, __ATOMIC_ACQ_REL);   // gates done
  }
  return hipSuccess;
}
EXPORT hipError_t hipGraphLaunch(hipGraphExec_t, hipStream_t) { launches++; return hipSuccess; }
EXPORT hipError_t hipStreamIsCapturing(hipStream_t, hipStreamCaptureStatus* s) {
  *s = hipStreamCaptureStatusNone;
  return hipSuccess;
}
EXPORT hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
// No GPU: the governor code object loads only in MOCKHIP_GOVERNOR mode, any
// other image only in MOCKHIP_MODULES mode (as a fake module with simulated
// code-object VRAM).
hipError_t mock_module_load(hipModule_t* m) {
  if (mock_governor()) {
    *m = reinterpret_cast<hipModule_t>(0x10001);
    return hipSuccess;
  }
  if (!getenv("MOCKHIP_MODULES")) return hipErrorNoBinaryForGpu;
  std::lock_guard<std::mutex> lk(mu);
  void* h = malloc(64);
  modules[h] = module_cost();
  module_bytes[cur_dev] += module_cost();
  kfd_publish_locked(cur_dev);
  *m = reinterpret_cast<hipModule_t>(h);
  return hipSuccess;
}
EXPORT hipError_t hipModuleLoadData(hipModule_t* m, const void*) { return mock_module_load(m); }
EXPORT hipError_t hipModuleLoadDataEx(hipModule_t* m, const void*, unsigned int, hipJitOption*, void**) {
  return mock_module_load(m);
}
EXPORT hipError_t hipModuleLoad(hipModule_t* m, const char* path) {
  struct stat st;
  if (!path || stat(path, &st) != 0) return hipErrorFileNotFound;
  return mock_module_load(m);
}
EXPORT hipError_t hipModuleUnload(hipModule_t m) {
  std::lock_guard<std::mutex> lk(mu);
  auto it = modules.find(reinterpret_cast<void*>(m));
  if (it == modules.end()) return hipErrorInvalidResourceHandle;
  module_bytes[cur_dev] -= it->second;
  kfd_publish_locked(cur_dev);
  free(it->first);
  modules.erase(it);
  return hipSuccess;
}
EXPORT hipError_t hipModuleGetFunction(hipFunction_t* f, hipModule_t, const char* name) {
  if (!mock_governor()) return hipErrorNotFound;
  if (!strcmp(name, "mivgpu_gate")) *f = reinterpret_cast<hipFunction_t>(kGateFn);
  else if (!strcmp(name, "mivgpu_clock")) *f = reinterpret_cast<hipFunction_t>(kClockFn);
  else return hipErrorNotFound;
  return hipSuccess;
}
EXPORT unsigned long long mockhip_launch_count(void) { return launches.load(); }

// ---- launch entry points beyond the classic ones (hip_6.5, multi-device) ----
EXPORT hipError_t hipLaunchKernelExC(const hipLaunchConfig_t*, const void*, void**) { launches++; return hipSuccess; }
EXPORT hipError_t hipDrvLaunchKernelEx(const HIP_LAUNCH_CONFIG*, hipFunction_t, void**, void**) {
  launches++;
  return hipSuccess;
}
EXPORT hipError_t hipLaunchCooperativeKernelMultiDevice(hipLaunchParams*, int n, unsigned int) {
  launches += (unsigned long long)n;
  return hipSuccess;
}
EXPORT hipError_t hipExtLaunchMultiKernelMultiDevice(hipLaunchParams*, int n, unsigned int) {
  launches += (unsigned long long)n;
  return hipSuccess;
}
// Mock streams are the device index + 1 cast to a handle (nullptr: current device).
EXPORT hipError_t hipStreamGetDevice(hipStream_t s, hipDevice_t* d) {
  *d = s ? (int)(reinterpret_cast<uintptr_t>(s) - 1) : cur_dev;
  return hipSuccess;
}

// ---- arrays: a handle whose "VRAM" is width x height x depth x element ----
EXPORT hipError_t hipMallocArray(hipArray_t* a, const hipChannelFormatDesc* d, size_t w, size_t h, unsigned int) {
  const size_t e = d ? (size_t)(d->x + d->y + d->z + d->w) / 8 : 4;
  return do_alloc(reinterpret_cast<void**>(a), w * (h ? h : 1) * (e ? e : 4));
}
EXPORT hipError_t hipMalloc3DArray(hipArray_t* a, const hipChannelFormatDesc* d, hipExtent x, unsigned int) {
  const size_t e = d ? (size_t)(d->x + d->y + d->z + d->w) / 8 : 4;
  return do_alloc(reinterpret_cast<void**>(a), x.width * (x.height ? x.height : 1) * (x.depth ? x.depth : 1) * e);
}
EXPORT hipError_t hipArrayCreate(hipArray_t* a, const HIP_ARRAY_DESCRIPTOR* d) {
  return do_alloc(reinterpret_cast<void**>(a), d->Width * (d->Height ? d->Height : 1) * 4 * d->NumChannels);
}
EXPORT hipError_t hipArray3DCreate(hipArray_t* a, const HIP_ARRAY3D_DESCRIPTOR* d) {
  return do_alloc(reinterpret_cast<void**>(a),
                  d->Width * (d->Height ? d->Height : 1) * (d->Depth ? d->Depth : 1) * 4 * d->NumChannels);
}
EXPORT hipError_t hipMallocMipmappedArray(hipMipmappedArray_t* a, const hipChannelFormatDesc*, hipExtent x,
                                          unsigned int, unsigned int) {
  return do_alloc(reinterpret_cast<void**>(a), x.width * (x.height ? x.height : 1) * 4);
}
EXPORT hipError_t hipMipmappedArrayCreate(hipMipmappedArray_t* a, HIP_ARRAY3D_DESCRIPTOR* d, unsigned int) {
  return do_alloc(reinterpret_cast<void**>(a), d->Width * (d->Height ? d->Height : 1) * 4);
}
EXPORT hipError_t hipMalloc3D(hipPitchedPtr* pp, hipExtent x) {
  pp->pitch = (x.width + 255) & ~size_t(255);
  pp->xsize = x.width;
  pp->ysize = x.height;
  return do_alloc(&pp->ptr, pp->pitch * (x.height ? x.height : 1) * (x.depth ? x.depth : 1));
}
EXPORT hipError_t hipFreeArray(hipArray_t a) { return do_free(a); }
EXPORT hipError_t hipArrayDestroy(hipArray_t a) { return do_free(a); }
EXPORT hipError_t hipFreeMipmappedArray(hipMipmappedArray_t a) { return do_free(a); }
EXPORT hipError_t hipMipmappedArrayDestroy(hipMipmappedArray_t a) { return do_free(a); }

// ---- run-time lookup: the runtime's OWN functions by name, like the real
// hipGetProcAddress (never the global binding an interposer would provide) ----
EXPORT hipError_t hipGetProcAddress(const char* sym, void** pfn, int, uint64_t, hipDriverProcAddressQueryResult* st) {
  static const struct { const char* n; void* f; } kTable[] = {
      {"hipMalloc", reinterpret_cast<void*>(static_cast<hipError_t (*)(void**, size_t)>(&hipMalloc))},
      {"hipFree", reinterpret_cast<void*>(&hipFree)},
      {"hipModuleLaunchKernel", reinterpret_cast<void*>(&hipModuleLaunchKernel)},
      {"hipLaunchKernel", reinterpret_cast<void*>(&hipLaunchKernel)},
      {"hipDrvLaunchKernelEx", reinterpret_cast<void*>(&hipDrvLaunchKernelEx)},
      {"hipModuleLoadDataEx", reinterpret_cast<void*>(&hipModuleLoadDataEx)},
      {"hipMemGetInfo", reinterpret_cast<void*>(&hipMemGetInfo)},
      {"hipGetDeviceProperties", reinterpret_cast<void*>(&hipGetDevicePropertiesR0600)},
      {"hipGetDeviceCount", reinterpret_cast<void*>(&hipGetDeviceCount)},
  };
  for (const auto& e : kTable) {
    if (!strcmp(e.n, sym)) {
      *pfn = e.f;
      if (st) *st = HIP_GET_PROC_ADDRESS_SUCCESS;
      return hipSuccess;
    }
  }
  *pfn = nullptr;
  if (st) *st = HIP_GET_PROC_ADDRESS_SYMBOL_NOT_FOUND;
  return hipErrorNotFound;
}
