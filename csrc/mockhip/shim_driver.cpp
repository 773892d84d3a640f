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
//   cfginfo          mivgpu_config_info: charging modes, grant/control loaded
//   hsainit          hsa_init (interposed by the shim) + the HSA_CU_MASK /
//                    ROCR_VISIBLE_DEVICES ROCr would read
//   dlsym_alloc <MiB>  hipMalloc looked up at run time: dlopen + dlsym
//   dlvsym_alloc <MiB> ... dlopen + dlvsym(hip_4.2)
//   gpa_alloc <MiB>    ... dlsym("hipGetProcAddress") + hipGetProcAddress
//                      (Triton's path)
//   gpa_launch <n>     hipModuleLaunchKernel via hipGetProcAddress, n times
//   launchex <n>       n x hipLaunchKernelExC + n x hipDrvLaunchKernelEx
//   multilaunch        hipLaunchCooperativeKernelMultiDevice + hipExt... on
//                      every device (MOCKHIP_DEVICES)
//   array <MiB>        hipMallocArray (float4 texels)
//   array3d <MiB>      hipMalloc3DArray
//   arraycreate <MiB>  hipArrayCreate (driver API)
//   malloc3d <MiB>     hipMalloc3D (pitched)
//   mipmap <MiB>       hipMallocMipmappedArray, 1 level
//   arrayfree          free every array / mipmap (hipFreeArray, hipArrayDestroy ...)
//   modload <path>     hipModuleLoad; moddata <path>: hipModuleLoadData of the
//                      file's bytes; moddataex <path>: hipModuleLoadDataEx
//   modunload          hipModuleUnload every module
//   getenv <KEY>       getenv as the runtime would call it
//   envscan <KEY>      the KEY entry of environ, read directly (ROCclr's way)
//   setenv|putenv <KEY> <VAL>, unsetenv <KEY>   a tenant rewriting its environment
//   balance            the governor's host-bucket balance on device 0
//   launchfor <ms>     hipLaunchKernel every 100 us for <ms> (a busy tenant)
//   smi <lib>          dlopen an SMI library (csrc/mockhip/mock_smi.cpp) and run
//                      the memory queries amd-smi / rocm-smi use
//   sampler            mivgpu_sampler_info: the occupancy sampler's account
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
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <string>
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

extern char** environ;

static void* hip_handle() {
  void* h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_NOLOAD);
  return h;
}

static unsigned long long shim_seen() {
  auto f = (unsigned long long (*)(void))dlsym(RTLD_DEFAULT, "mivgpu_launch_count");
  return f ? f() : 0ull;
}
static unsigned long long real_seen() {
  auto g = (unsigned long long (*)(void))dlsym(RTLD_DEFAULT, "mockhip_launch_count");
  return g ? g() : 0ull;
}

static std::vector<void*> g_arrays;          // hipArray_t / hipMipmappedArray_t (tagged below)
static std::vector<int> g_array_kind;        // 0 FreeArray, 1 ArrayDestroy, 2 FreeMipmappedArray
static std::vector<hipModule_t> g_modules;

static std::vector<char> read_file(const char* path) {
  std::vector<char> b;
  FILE* f = fopen(path, "rb");
  if (!f) return b;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), f)) > 0) b.insert(b.end(), buf, buf + n);
  fclose(f);
  return b;
}

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
    } else if (!strcmp(c, "launchtime")) {
      // host cost per launch: N launches into the mock runtime (which only counts)
      long n = strtol(argv[++i], nullptr, 10);
      static char dummy;
      for (long k = 0; k < 1000; ++k) (void)hipLaunchKernel(&dummy, dim3(1), dim3(64), nullptr, 0, nullptr);
      struct timespec t0, t1;
      clock_gettime(CLOCK_MONOTONIC, &t0);
      for (long k = 0; k < n; ++k) (void)hipLaunchKernel(&dummy, dim3(1), dim3(64), nullptr, 0, nullptr);
      clock_gettime(CLOCK_MONOTONIC, &t1);
      const double ns = ((t1.tv_sec - t0.tv_sec) * 1e9 + (t1.tv_nsec - t0.tv_nsec)) / (double)n;
      printf("{\"op\":\"launchtime\",\"n\":%ld,\"ns_per_launch\":%.1f}\n", n, ns);
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
    } else if (!strcmp(c, "dlsym_alloc") || !strcmp(c, "dlvsym_alloc") || !strcmp(c, "gpa_alloc")) {
      size_t mib = strtoull(argv[++i], nullptr, 10);
      using malloc_fn = hipError_t (*)(void**, size_t);
      malloc_fn f = nullptr;
      void* h = hip_handle();
      if (!strcmp(c, "dlsym_alloc")) {
        f = (malloc_fn)dlsym(h, "hipMalloc");
      } else if (!strcmp(c, "dlvsym_alloc")) {
        f = (malloc_fn)dlvsym(h, "hipMalloc", "hip_4.2");
      } else {
        using gpa_fn = hipError_t (*)(const char*, void**, int, uint64_t, hipDriverProcAddressQueryResult*);
        gpa_fn gpa = (gpa_fn)dlsym(h, "hipGetProcAddress");
        hipDriverProcAddressQueryResult st;
        if (gpa) (void)gpa("hipMalloc", (void**)&f, 700, 0, &st);
      }
      void* p = nullptr;
      hipError_t rc = f ? f(&p, mib << 20) : hipErrorNotFound;
      // the lookup must hand out the interposed entry point (the global binding)
      printf("{\"op\":\"%s\",\"mib\":%zu,\"rc\":%d,\"hooked\":%d}\n", c, mib, (int)rc,
             f == (malloc_fn)&hipMalloc ? 1 : 0);
      if (rc == hipSuccess) bufs.push_back(p);
    } else if (!strcmp(c, "gpa_launch")) {
      long n = strtol(argv[++i], nullptr, 10);
      using gpa_fn = hipError_t (*)(const char*, void**, int, uint64_t, hipDriverProcAddressQueryResult*);
      gpa_fn gpa = (gpa_fn)dlsym(hip_handle(), "hipGetProcAddress");
      using launch_fn = hipError_t (*)(hipFunction_t, unsigned, unsigned, unsigned, unsigned, unsigned, unsigned,
                                       unsigned, hipStream_t, void**, void**);
      launch_fn f = nullptr;
      hipDriverProcAddressQueryResult st;
      if (gpa) (void)gpa("hipModuleLaunchKernel", (void**)&f, 700, 0, &st);
      for (long k = 0; f && k < n; ++k) (void)f(nullptr, 1, 1, 1, 64, 1, 1, 0, nullptr, nullptr, nullptr);
      printf("{\"op\":\"gpa_launch\",\"n\":%ld,\"found\":%d,\"shim_seen\":%llu,\"real_seen\":%llu}\n", n,
             f ? 1 : 0, shim_seen(), real_seen());
    } else if (!strcmp(c, "launchex")) {
      long n = strtol(argv[++i], nullptr, 10);
      static char dummy;
      hipLaunchConfig_t cfg{};
      cfg.gridDim = dim3(1);
      cfg.blockDim = dim3(64);
      HIP_LAUNCH_CONFIG dcfg{};
      dcfg.gridDimX = dcfg.gridDimY = dcfg.gridDimZ = 1;
      dcfg.blockDimX = 64;
      dcfg.blockDimY = dcfg.blockDimZ = 1;
      for (long k = 0; k < n; ++k) {
        (void)hipLaunchKernelExC(&cfg, &dummy, nullptr);
        (void)hipDrvLaunchKernelEx(&dcfg, nullptr, nullptr, nullptr);
      }
      printf("{\"op\":\"launchex\",\"n\":%ld,\"shim_seen\":%llu,\"real_seen\":%llu}\n", n, shim_seen(),
             real_seen());
    } else if (!strcmp(c, "multilaunch")) {
      int nd = 0;
      (void)hipGetDeviceCount(&nd);
      static char dummy;
      std::vector<hipLaunchParams> lp(nd);
      for (int d = 0; d < nd; ++d) {
        lp[d].func = &dummy;
        lp[d].gridDim = dim3(1);
        lp[d].blockDim = dim3(64);
        lp[d].args = nullptr;
        lp[d].sharedMem = 0;
        lp[d].stream = reinterpret_cast<hipStream_t>((uintptr_t)d + 1);   // mock: device d's stream
      }
      (void)hipLaunchCooperativeKernelMultiDevice(lp.data(), nd, 0);
      (void)hipExtLaunchMultiKernelMultiDevice(lp.data(), nd, 0);
      printf("{\"op\":\"multilaunch\",\"devices\":%d,\"shim_seen\":%llu,\"real_seen\":%llu}\n", nd, shim_seen(),
             real_seen());
    } else if (!strcmp(c, "array") || !strcmp(c, "array3d") || !strcmp(c, "arraycreate") || !strcmp(c, "mipmap")) {
      size_t mib = strtoull(argv[++i], nullptr, 10);
      hipChannelFormatDesc desc{};
      desc.x = desc.y = desc.z = desc.w = 32;       // float4 = 16 B per texel
      desc.f = hipChannelFormatKindFloat;
      const size_t w = 4096, h = (mib << 20) / (w * 16);
      void* a = nullptr;
      hipError_t rc;
      int kind = 0;
      if (!strcmp(c, "array")) {
        rc = hipMallocArray((hipArray_t*)&a, &desc, w, h, 0);
      } else if (!strcmp(c, "array3d")) {
        rc = hipMalloc3DArray((hipArray_t*)&a, &desc, make_hipExtent(w, h, 1), 0);
      } else if (!strcmp(c, "arraycreate")) {
        HIP_ARRAY_DESCRIPTOR d{};
        d.Width = w;
        d.Height = h;
        d.Format = HIP_AD_FORMAT_FLOAT;
        d.NumChannels = 4;
        rc = hipArrayCreate((hipArray_t*)&a, &d);
        kind = 1;
      } else {
        rc = hipMallocMipmappedArray((hipMipmappedArray_t*)&a, &desc, make_hipExtent(w, h, 0), 1, 0);
        kind = 2;
      }
      printf("{\"op\":\"%s\",\"mib\":%zu,\"rc\":%d}\n", c, mib, (int)rc);
      if (rc == hipSuccess) {
        g_arrays.push_back(a);
        g_array_kind.push_back(kind);
      }
    } else if (!strcmp(c, "malloc3d")) {
      size_t mib = strtoull(argv[++i], nullptr, 10);
      hipPitchedPtr pp{};
      hipError_t rc = hipMalloc3D(&pp, make_hipExtent(1 << 20, mib, 1));   // mib rows of 1 MiB
      printf("{\"op\":\"malloc3d\",\"mib\":%zu,\"rc\":%d}\n", mib, (int)rc);
      if (rc == hipSuccess) bufs.push_back(pp.ptr);
    } else if (!strcmp(c, "arrayfree")) {
      int bad = 0;
      for (size_t k = 0; k < g_arrays.size(); ++k) {
        hipError_t rc = g_array_kind[k] == 0   ? hipFreeArray((hipArray_t)g_arrays[k])
                        : g_array_kind[k] == 1 ? hipArrayDestroy((hipArray_t)g_arrays[k])
                                               : hipFreeMipmappedArray((hipMipmappedArray_t)g_arrays[k]);
        bad += rc != hipSuccess;
      }
      g_arrays.clear();
      g_array_kind.clear();
      printf("{\"op\":\"arrayfree\",\"errors\":%d}\n", bad);
    } else if (!strcmp(c, "modload") || !strcmp(c, "moddata") || !strcmp(c, "moddataex")) {
      const char* path = argv[++i];
      hipModule_t m = nullptr;
      hipError_t rc;
      if (!strcmp(c, "modload")) {
        rc = hipModuleLoad(&m, path);
      } else {
        std::vector<char> img = read_file(path);
        rc = !strcmp(c, "moddata") ? hipModuleLoadData(&m, img.data())
                                   : hipModuleLoadDataEx(&m, img.data(), 0, nullptr, nullptr);
      }
      printf("{\"op\":\"%s\",\"rc\":%d}\n", c, (int)rc);
      if (rc == hipSuccess) g_modules.push_back(m);
    } else if (!strcmp(c, "modunload")) {
      int bad = 0;
      for (hipModule_t m : g_modules) bad += hipModuleUnload(m) != hipSuccess;
      g_modules.clear();
      printf("{\"op\":\"modunload\",\"errors\":%d}\n", bad);
    } else if (!strcmp(c, "launchfor")) {
      // launch back to back for <ms> milliseconds (a busy tenant)
      const long ms = strtol(argv[++i], nullptr, 10);
      static char dummy;
      struct timespec t0, t;
      clock_gettime(CLOCK_MONOTONIC, &t0);
      long n = 0;
      do {
        (void)hipLaunchKernel(&dummy, dim3(1), dim3(64), nullptr, 0, nullptr);
        ++n;
        usleep(100);
        clock_gettime(CLOCK_MONOTONIC, &t);
      } while ((t.tv_sec - t0.tv_sec) * 1000 + (t.tv_nsec - t0.tv_nsec) / 1000000 < ms);
      printf("{\"op\":\"launchfor\",\"n\":%ld}\n", n);
    } else if (!strcmp(c, "balance")) {
      auto f = (int (*)(int, long long*, unsigned long long*))dlsym(RTLD_DEFAULT, "mivgpu_gate_balance");
      long long t = 0;
      unsigned long long r = 0;
      int rc = f ? f(0, &t, &r) : -2;
      auto st = (int (*)(int, unsigned long long*, unsigned long long*, unsigned long long*))dlsym(
          RTLD_DEFAULT, "mivgpu_gate_stats");
      unsigned long long busy = 0, held = 0, gates = 0;
      if (st) (void)st(0, &busy, &held, &gates);
      printf("{\"op\":\"balance\",\"rc\":%d,\"tokens_ns\":%lld,\"received_ns\":%llu,\"held_ns\":%llu,"
             "\"gates\":%llu}\n", rc, t, r, held, gates);
    } else if (!strcmp(c, "smi")) {
      // what amd-smi / rocm-smi do: dlopen the library, dlsym the queries
      void* lib = dlopen(argv[++i], RTLD_NOW | RTLD_LOCAL);
      typedef int (*mem_fn)(void*, int, uint64_t*);
      typedef int (*rmem_fn)(uint32_t, int, uint64_t*);
      struct vu { uint32_t total, used, reserved[2]; } u = {0, 0, {0, 0}};
      struct vi { int type; char vendor[256]; uint64_t size; uint32_t width; uint64_t bw; uint64_t reserved[37]; } vinf;
      memset(&vinf, 0, sizeof(vinf));
      uint64_t t = 0, us = 0, gtt = 0, rt = 0, ru = 0;
      int ok = lib != nullptr;
      if (ok) {
        auto mt = (mem_fn)dlsym(lib, "amdsmi_get_gpu_memory_total");
        auto mu = (mem_fn)dlsym(lib, "amdsmi_get_gpu_memory_usage");
        auto vuf = (int (*)(void*, vu*))dlsym(lib, "amdsmi_get_gpu_vram_usage");
        auto vif = (int (*)(void*, vi*))dlsym(lib, "amdsmi_get_gpu_vram_info");
        auto rt_f = (rmem_fn)dlsym(lib, "rsmi_dev_memory_total_get");
        auto ru_f = (rmem_fn)dlsym(lib, "rsmi_dev_memory_usage_get");
        ok = mt && mu && vuf && vif && rt_f && ru_f && !mt((void*)1, 0, &t) && !mu((void*)1, 0, &us) &&
             !mt((void*)1, 2, &gtt) && !vuf((void*)1, &u) && !vif((void*)1, &vinf) && !rt_f(0, 0, &rt) &&
             !ru_f(0, 0, &ru);
      }
      printf("{\"op\":\"smi\",\"ok\":%d,\"total_mib\":%llu,\"used_mib\":%llu,\"gtt_mib\":%llu,"
             "\"vram_total_mb\":%u,\"vram_used_mb\":%u,\"vram_size_mb\":%llu,\"rsmi_total_mib\":%llu,"
             "\"rsmi_used_mib\":%llu}\n", ok, (unsigned long long)(t >> 20), (unsigned long long)(us >> 20),
             (unsigned long long)(gtt >> 20), u.total, u.used, (unsigned long long)vinf.size,
             (unsigned long long)(rt >> 20), (unsigned long long)(ru >> 20));
    } else if (!strcmp(c, "sampler")) {
      // the sampler's own account (share board, local estimate), as JSON
      auto f = (int (*)(int, char*, int))dlsym(RTLD_DEFAULT, "mivgpu_sampler_info");
      static char buf[16384];
      int n = f ? f(0, buf, (int)sizeof(buf)) : -2;
      printf("{\"op\":\"sampler\",\"rc\":%d,\"info\":%s}\n", n < 0 ? n : 0, n > 0 ? buf : "null");
    } else if (!strcmp(c, "setenv") || !strcmp(c, "putenv") || !strcmp(c, "unsetenv")) {
      const char* k = argv[++i];
      int rc;
      if (!strcmp(c, "setenv")) {
        rc = setenv(k, argv[++i], 1);
      } else if (!strcmp(c, "putenv")) {
        static std::vector<std::string> keep;      // putenv keeps the pointer
        keep.emplace_back(std::string(k) + "=" + argv[++i]);
        rc = putenv(const_cast<char*>(keep.back().c_str()));
      } else {
        rc = unsetenv(k);
      }
      printf("{\"op\":\"%s\",\"rc\":%d}\n", c, rc);
    } else if (!strcmp(c, "envscan")) {
      // what ROCclr does for its flags: walk environ itself
      const char* k = argv[++i];
      const size_t n = strlen(k);
      const char* v = nullptr;
      for (char** e = environ; e && *e; ++e)
        if (!strncmp(*e, k, n) && (*e)[n] == '=') v = *e + n + 1;
      printf("{\"op\":\"envscan\",\"key\":\"%s\",\"set\":%d,\"value\":\"%s\"}\n", k, v ? 1 : 0, v ? v : "");
    } else if (!strcmp(c, "getenv")) {
      const char* k = argv[++i];
      const char* v = getenv(k);
      printf("{\"op\":\"getenv\",\"key\":\"%s\",\"set\":%d,\"value\":\"%s\"}\n", k, v ? 1 : 0, v ? v : "");
    } else if (!strcmp(c, "cfginfo")) {
      auto f = (int (*)(unsigned long long*))dlsym(RTLD_DEFAULT, "mivgpu_config_info");
      unsigned long long crn = 0;
      const int flags = f ? f(&crn) : -1;
      printf("{\"op\":\"cfginfo\",\"flags\":%d,\"ctx_refresh_ns\":%llu}\n", flags, crn);
    } else if (!strcmp(c, "device")) {
      int d = atoi(argv[++i]);
      printf("{\"op\":\"device\",\"rc\":%d}\n", (int)hipSetDevice(d));
    }
    fflush(stdout);
  }
  return 0;
}
