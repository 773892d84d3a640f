// Test driver for libmivgpu.so against the mock HIP runtime (CPU tests).
// Linked against the mock libamdhip64.so, so its HIP references are versioned
// exactly like PyTorch's.  Commands (argv):
//   alloc <MiB>      hipMalloc, prints rc and slot index
//   allocasync <MiB> hipMallocAsync
//   vmm <MiB>        hipMemCreate
//   freeall          hipFree / hipMemRelease everything allocated so far
//   meminfo          hipMemGetInfo
//   props            hipGetDevicePropertiesR0600 totalGlobalMem + hipDeviceTotalMem
//   launch <n>       n x hipLaunchKernel
//   usage            mivgpu_process_usage(0) via dlsym
//   sleep <ms>
//   kfdctx <MiB>     runtime VRAM outside the hooks in the mock's simulated
//                    KFD per-process file (MOCKHIP_KFD_SYSFS), for context accounting
//   device <i>       hipSetDevice
//   hsainit          hsa_init (interposed by the shim) + the HSA_CU_MASK /
//                    ROCR_VISIBLE_DEVICES ROCr would read
//   stress <threads> <iters> <max MiB>
//                    threads doing random hipMalloc/hipFree and
//                    hipMemCreate/hipMemRelease, one kernel launch per
//                    iteration (sanitizer + race tests)
#include <hip/hip_runtime_api.h>

#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <random>
#include <thread>
#include <vector>

static void stress_thread(int seed, int iters, int max_mib, std::atomic<long>* allocs, std::atomic<long>* ooms,
                          std::atomic<long>* errors) {
  std::mt19937 rng(seed);
  std::vector<void*> bufs;
  std::vector<hipMemGenericAllocationHandle_t> handles;
  static char kernel;
  for (int k = 0; k < iters; ++k) {
    // a launch per iteration: the launch hooks (and the occupancy sampler
    // they start) run concurrently with the allocation hooks
    (void)hipLaunchKernel(&kernel, dim3(1), dim3(64), nullptr, 0, nullptr);
    const int op = rng() % 4;
    const size_t mib = 1 + rng() % max_mib;
    if (op == 0 || (op == 1 && bufs.empty())) {
      void* p = nullptr;
      hipError_t rc = hipMalloc(&p, mib << 20);
      if (rc == hipSuccess) { bufs.push_back(p); ++*allocs; }
      else if (rc == hipErrorOutOfMemory) ++*ooms;
      else ++*errors;
    } else if (op == 1) {
      const size_t i = rng() % bufs.size();
      if (hipFree(bufs[i]) != hipSuccess) ++*errors;
      bufs[i] = bufs.back();
      bufs.pop_back();
    } else if (op == 2 || handles.empty()) {
      hipMemGenericAllocationHandle_t h{};
      hipMemAllocationProp prop{};
      prop.type = hipMemAllocationTypePinned;
      prop.location.type = hipMemLocationTypeDevice;
      prop.location.id = 0;
      hipError_t rc = hipMemCreate(&h, mib << 20, &prop, 0);
      if (rc == hipSuccess) { handles.push_back(h); ++*allocs; }
      else if (rc == hipErrorOutOfMemory) ++*ooms;
      else ++*errors;
    } else {
      const size_t i = rng() % handles.size();
      if (hipMemRelease(handles[i]) != hipSuccess) ++*errors;
      handles[i] = handles.back();
      handles.pop_back();
    }
  }
  for (void* p : bufs) if (hipFree(p) != hipSuccess) ++*errors;
  for (auto h : handles) if (hipMemRelease(h) != hipSuccess) ++*errors;
}

extern "C" hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600*, int);

int main(int argc, char** argv) {
  std::vector<void*> bufs;
  std::vector<hipMemGenericAllocationHandle_t> handles;
  for (int i = 1; i < argc; ++i) {
    const char* c = argv[i];
    if (!strcmp(c, "alloc") || !strcmp(c, "allocasync")) {
      size_t mib = strtoull(argv[++i], nullptr, 10);
      void* p = nullptr;
      hipError_t rc = !strcmp(c, "alloc") ? hipMalloc(&p, mib << 20)
                                         : hipMallocAsync(&p, mib << 20, nullptr);
      printf("{\"op\":\"%s\",\"mib\":%zu,\"rc\":%d}\n", c, mib, (int)rc);
      if (rc == hipSuccess) bufs.push_back(p);
    } else if (!strcmp(c, "vmm")) {
      size_t mib = strtoull(argv[++i], nullptr, 10);
      hipMemGenericAllocationHandle_t h{};
      hipMemAllocationProp prop{};
      prop.type = hipMemAllocationTypePinned;
      prop.location.type = hipMemLocationTypeDevice;
      int d = 0;
      (void)hipGetDevice(&d);
      prop.location.id = d;
      hipError_t rc = hipMemCreate(&h, mib << 20, &prop, 0);
      printf("{\"op\":\"vmm\",\"mib\":%zu,\"rc\":%d}\n", mib, (int)rc);
      if (rc == hipSuccess) handles.push_back(h);
    } else if (!strcmp(c, "freeall")) {
      int bad = 0;
      for (void* p : bufs) bad += hipFree(p) != hipSuccess;
      for (auto h : handles) bad += hipMemRelease(h) != hipSuccess;
      bufs.clear();
      handles.clear();
      printf("{\"op\":\"freeall\",\"errors\":%d}\n", bad);
    } else if (!strcmp(c, "meminfo")) {
      size_t f = 0, t = 0;
      hipError_t rc = hipMemGetInfo(&f, &t);
      printf("{\"op\":\"meminfo\",\"rc\":%d,\"free_mib\":%zu,\"total_mib\":%zu}\n", (int)rc, f >> 20,
             t >> 20);
    } else if (!strcmp(c, "props")) {
      hipDeviceProp_tR0600 p;
      (void)hipGetDevicePropertiesR0600(&p, 0);
      size_t tm = 0;
      (void)hipDeviceTotalMem(&tm, 0);
      printf("{\"op\":\"props\",\"total_mib\":%zu,\"devtotal_mib\":%zu}\n", p.totalGlobalMem >> 20,
             tm >> 20);
    } else if (!strcmp(c, "launch")) {
      long n = strtol(argv[++i], nullptr, 10);
      static char dummy;
      for (long k = 0; k < n; ++k) (void)hipLaunchKernel(&dummy, dim3(1), dim3(64), nullptr, 0, nullptr);
      auto f = (unsigned long long (*)(void))dlsym(RTLD_DEFAULT, "mivgpu_launch_count");
      auto g = (unsigned long long (*)(void))dlsym(RTLD_DEFAULT, "mockhip_launch_count");
      printf("{\"op\":\"launch\",\"n\":%ld,\"shim_seen\":%llu,\"real_seen\":%llu}\n", n,
             f ? f() : 0ull, g ? g() : 0ull);
    } else if (!strcmp(c, "usage")) {
      auto f = (long long (*)(int))dlsym(RTLD_DEFAULT, "mivgpu_process_usage");
      printf("{\"op\":\"usage\",\"bytes\":%lld}\n", f ? f(0) : -2ll);
    } else if (!strcmp(c, "kfdctx")) {
      // runtime bytes outside the allocator hooks, as KFD would count them
      auto f = (void (*)(unsigned long long))dlsym(RTLD_DEFAULT, "mockhip_set_kfd_context");
      const unsigned long long mib = strtoull(argv[++i], nullptr, 10);
      if (f) f(mib);
      printf("{\"op\":\"kfdctx\",\"ok\":%d}\n", f ? 1 : 0);
      usleep(30000);  // past the shim's 20 ms refresh interval
    } else if (!strcmp(c, "hsainit")) {
      // what ROCr would see: HIP calls hsa_init, which the shim interposes
      auto f = (int (*)(void))dlsym(RTLD_DEFAULT, "hsa_init");
      int rc = f ? f() : -1;
      const char* m = getenv("HSA_CU_MASK");
      const char* v = getenv("ROCR_VISIBLE_DEVICES");
      printf("{\"op\":\"hsainit\",\"hooked\":%d,\"rc\":%d,\"mask\":\"%s\",\"visible\":\"%s\"}\n", f ? 1 : 0, rc,
             m ? m : "", v ? v : "");
    } else if (!strcmp(c, "sleep")) {
      usleep((useconds_t)strtoul(argv[++i], nullptr, 10) * 1000);
    } else if (!strcmp(c, "stress")) {
      const int nt = atoi(argv[++i]), iters = atoi(argv[++i]), max_mib = atoi(argv[++i]);
      std::atomic<long> allocs{0}, ooms{0}, errors{0};
      std::vector<std::thread> ts;
      for (int k = 0; k < nt; ++k)
        ts.emplace_back(stress_thread, (int)getpid() * 131 + k, iters, max_mib, &allocs, &ooms, &errors);
      for (auto& t : ts) t.join();
      auto f = (long long (*)(int))dlsym(RTLD_DEFAULT, "mivgpu_process_usage");
      printf("{\"op\":\"stress\",\"allocs\":%ld,\"ooms\":%ld,\"errors\":%ld,\"usage_after\":%lld}\n",
             allocs.load(), ooms.load(), errors.load(), f ? f(0) : -2ll);
    } else if (!strcmp(c, "device")) {
      int d = atoi(argv[++i]);
      printf("{\"op\":\"device\",\"rc\":%d}\n", (int)hipSetDevice(d));
    }
    fflush(stdout);
  }
  return 0;
}
