// libmivgpu.so -- in-container HIP interposition layer for MI355X vGPU slices.
//
// Capability parity target: HAMi-core's libvgpu.so (absent submodule in the
// reference; contract inferred in SURVEY.md §2.6 from
// pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:833-897 and
// pkg/monitor/nvidia/v1/spec.go:24-240).  This is NOT a translation of it:
//
//  * Interposition is by ELF symbol versioning: every hooked entry point is
//    exported under the exact version node libamdhip64 uses (hip_4.2 ...
//    hip_6.5, see mivgpu_shim.map), so the versioned PLT references of
//    PyTorch, hipBLASLt, rocBLAS, MIOpen and RCCL bind to us, and the real
//    implementation is resolved once with dlvsym(RTLD_NEXT, name, version).
//  * Re-entrancy (the failure docs/develop/amd-vgpu.md:18-22 hit with a naive
//    LD_PRELOAD on ROCm 7.x) is handled with a thread-local depth counter: any
//    hooked call made while a hook is already active on the thread is passed
//    straight through, so HIP-internal PLT calls are never double-accounted.
//  * Memory: hard per-device HBM quota (HIP_DEVICE_MEMORY_LIMIT[_i]) checked
//    against an O(1) aggregate counter in the shared region; hipMemGetInfo,
//    hipDeviceTotalMem and hipGetDeviceProperties* report the slice.  The VMM
//    path (hipMemCreate/hipMemRelease) used by PyTorch expandable segments and
//    the stream-ordered allocator are accounted too.
//  * Compute: spatial isolation is HSA_CU_MASK (hardware CU masking set by the
//    device plugin, zero per-launch cost).  When a temporal share must be
//    enforced (policy=force, no CU mask, or the monitor's utilisation switch),
//    the launch hooks enqueue the gfx950 governor gate (governor.hip) in front
//    of the user's work on the same stream: a device-side token bucket, no
//    host blocking.
//  * Priority blocking: recent_kernel == -1 in the shared region (set by the
//    node monitor's feedback loop, cmd/vGPUmonitor/feedback.go:74-134 in the
//    reference) parks launches of the low-priority task.  Under a grant file
//    the monitor's verdicts come from a host-owned control file mapped
//    read-only (block, utilization switch, over-grant, KFD-measured excess
//    VRAM), and the limits from the read-only grant: nothing the tenant can
//    write into its shared region loosens either.
//  * hipIpc* is deliberately NOT wrapped: RCCL and custom all-reduce keep
//    working (the reference breaks CUDA IPC, examples/nvidia/vllm_cross_vgpu.yaml:99-102).
#include <hip/hip_runtime_api.h>

#include <dlfcn.h>
#include <elf.h>
#include <errno.h>
#include <link.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <time.h>
#include <dirent.h>
#include <unistd.h>

#include <atomic>
#include <cstddef>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

#include "mivgpu/shared_region.h"
#include "board.h"
#include <amd_smi/amdsmi.h>

#define MIVGPU_EXPORT extern "C" __attribute__((visibility("default")))

// libstdc++ (linked statically, see glibc_floor.h) reads glibc's
// __libc_single_threaded (GLIBC_2.32) to skip atomics in single-threaded
// processes.  Our own copy, always 0: "assume threads", which is always safe.
extern "C" {
__attribute__((visibility("hidden"))) char __libc_single_threaded = 0;
}
#if defined(__x86_64__) && defined(MIVGPU_GLIBC_FLOOR)
// (glibc_floor.h) the gthr weak references of the static libstdc++ bind here
extern "C" __attribute__((visibility("hidden"))) int pthread_once(pthread_once_t* o, void (*f)(void)) noexcept {
  return mivgpu_glibc_pthread_once(o, f);
}
extern "C" __attribute__((visibility("hidden"))) int __pthread_key_create(pthread_key_t* k, void (*d)(void*)) noexcept {
  return mivgpu_glibc_pthread_key_create(k, d);
}
#endif

namespace {

// ---------------------------------------------------------------- logging --
int g_log_level = 1;  // 0 error, 1 warn, 3 info, 4 debug (LIBCUDA_LOG_LEVEL-like)

void mlog(int lvl, const char* fmt, ...) {
  if (lvl > g_log_level) return;
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  static const char* tags[] = {"ERROR", "WARN", "WARN", "INFO", "DEBUG"};
  fprintf(stderr, "[mivgpu %s pid=%d] %s\n", tags[lvl < 0 ? 0 : (lvl > 4 ? 4 : lvl)], (int)getpid(),
          buf);
}

inline uint64_t mono_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
inline uint64_t coarse_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC_COARSE, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// ------------------------------------------------------------------ roctx --
// MIVGPU_ROCTX=1 puts the shim's own decisions on the profiler timeline
// (rocprofv3 --marker-trace), next to the tenant's kernels: OOM denials, host
// spills, governor gates, priority parking.  The library is dlopen'ed only
// when asked for, so the default path carries one null-pointer test.
struct Roctx {
  void (*mark)(const char*) = nullptr;
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
};
Roctx g_roctx;

void roctx_init(const char* hip_dir) {
  const char* on = getenv("MIVGPU_ROCTX");
  if (!on || !(!strcmp(on, "1") || !strcasecmp(on, "true"))) return;
  const char* lib = getenv("MIVGPU_ROCTX_LIB");
  void* h = nullptr;
  if (lib && *lib) {
    h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
  } else {
    h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h && hip_dir) {  // next to the HIP runtime (/opt/rocm/lib) when not on the loader path
      char path[1024];
      snprintf(path, sizeof(path), "%s/librocprofiler-sdk-roctx.so.1", hip_dir);
      h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
    }
  }
  if (!h) {
    mlog(1, "MIVGPU_ROCTX set but no roctx library could be loaded: %s", dlerror());
    return;
  }
  g_roctx.mark = reinterpret_cast<void (*)(const char*)>(dlsym(h, "roctxMarkA"));
  g_roctx.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
  g_roctx.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
  if (!g_roctx.mark || !g_roctx.push || !g_roctx.pop) g_roctx = Roctx{};
}

__attribute__((format(printf, 1, 2))) void tmark(const char* fmt, ...) {
  if (__builtin_expect(!g_roctx.mark, 1)) return;
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_roctx.mark(buf);
}

struct TRange {
  bool on;
  explicit TRange(const char* name) : on(g_roctx.push != nullptr) {
    if (on) g_roctx.push(name);
  }
  ~TRange() {
    if (on) g_roctx.pop();
  }
};

// ------------------------------------------------------ re-entrancy guard --
// initial-exec TLS: a direct thread-pointer access on every hook instead of a
// __tls_get_addr call (the shim is preloaded, so it has static TLS space)
__attribute__((tls_model("initial-exec"))) thread_local int t_depth = 0;
struct Guard {
  bool outer;
  Guard() : outer(t_depth == 0) { ++t_depth; }
  ~Guard() { --t_depth; }
};

// ------------------------------------------------------- libc's own dl* --
// The shim exports dlsym and dlvsym itself (see "symbol resolution" below), so
// every dlsym/dlvsym call made from this library would bind back to those
// exports.  The real ones are found once by walking the loader's link map
// (_r_debug) to libc and looking the names up in its dynamic symbol table
// (GNU hash) -- no function call at all, so the lookup also works when a
// sanitizer runtime preloaded ahead of the shim resolves its own interceptors
// through the shim's dlsym before that runtime (or this library) is
// initialised.  These functions are therefore never instrumented.
#define MIVGPU_NO_SANITIZE __attribute__((no_sanitize_address, no_sanitize_thread, noinline))

MIVGPU_NO_SANITIZE void* elf_lookup_in(ElfW(Addr) base, const ElfW(Dyn)* dyn, const char* name) {
  if (!dyn) return nullptr;
  // glibc relocates these d_ptr entries in place on x86-64; accept both forms
  // (no helper call here: any instrumented callee would touch sanitizer
  // shadow memory that does not exist yet)
  const ElfW(Sym)* symtab = nullptr;
  const char* strtab = nullptr;
  const uint32_t* gnu = nullptr;
  for (const ElfW(Dyn)* d = dyn; d->d_tag != DT_NULL; ++d) {
    const ElfW(Addr) a = d->d_un.d_ptr < base ? d->d_un.d_ptr + base : d->d_un.d_ptr;
    if (d->d_tag == DT_SYMTAB) symtab = reinterpret_cast<const ElfW(Sym)*>(a);
    else if (d->d_tag == DT_STRTAB) strtab = reinterpret_cast<const char*>(a);
    else if (d->d_tag == DT_GNU_HASH) gnu = reinterpret_cast<const uint32_t*>(a);
  }
  if (!symtab || !strtab || !gnu) return nullptr;
  uint32_t h = 5381;
  for (const unsigned char* c = reinterpret_cast<const unsigned char*>(name); *c; ++c) h = h * 33 + *c;
  const uint32_t nbuckets = gnu[0], symoffset = gnu[1], bloom_words = gnu[2];
  const uint32_t* buckets = gnu + 4 + bloom_words * (sizeof(ElfW(Addr)) / 4);
  const uint32_t* chain = buckets + nbuckets;
  uint32_t i = buckets[h % nbuckets];
  if (i < symoffset) return nullptr;
  for (;; ++i) {
    const uint32_t ch = chain[i - symoffset];
    if ((ch | 1u) == (h | 1u) && symtab[i].st_value && ELF64_ST_TYPE(symtab[i].st_info) == STT_FUNC) {
      const char* a = name;
      const char* b = strtab + symtab[i].st_name;
      while (*a && *a == *b) ++a, ++b;
      if (*a == *b) return reinterpret_cast<void*>(base + symtab[i].st_value);
    }
    if (ch & 1u) break;
  }
  return nullptr;
}

MIVGPU_NO_SANITIZE bool soname_is(const char* path, const char* want) {
  const char* base = path;
  for (const char* c = path; *c; ++c)
    if (*c == '/') base = c + 1;
  while (*want && *base == *want) ++base, ++want;
  return *want == 0 && base[0] == '.' && base[1] == 's' && base[2] == 'o';
}

// libc's definition of `name`; dlsym/dlvsym/dladdr live in libdl.so.2 before
// glibc 2.34 (the shim names libdl.so.2 as NEEDED, so it is in the link map).
MIVGPU_NO_SANITIZE void* libc_sym(const char* name) {
  // (plain indexing: no std::initializer_list helpers, which a sanitizer
  // build instruments, before its runtime is up)
  static const char* const kLibs[2] = {"libc", "libdl"};
  for (int li = 0; li < 2; ++li) {
    const char* lib = kLibs[li];
    for (const struct link_map* m = _r_debug.r_map; m; m = m->l_next) {
      if (!soname_is(m->l_name ? m->l_name : "", lib)) continue;
      if (void* p = elf_lookup_in(m->l_addr, m->l_ld, name)) return p;
    }
  }
  return nullptr;
}

// The shim's own dynamic section (linker-provided): identifies its link_map entry.
extern "C" ElfW(Dyn) _DYNAMIC[];

// Last resort when no libc/libdl dlsym is found (never on a glibc system):
// look `name` up in the loaded objects ourselves -- every object for
// RTLD_DEFAULT, the objects AFTER the shim for RTLD_NEXT (from the head, the
// preloaded shim's own hooks would be found first and resolve() would bind
// the real entry points to themselves), the handle's own map
// otherwise (a glibc handle IS its link_map) -- so lookups keep working,
// unversioned, instead of aborting.
MIVGPU_NO_SANITIZE void* fallback_dlsym(void* handle, const char* name) {
  if (handle && handle != RTLD_DEFAULT && handle != RTLD_NEXT) {
    const struct link_map* m = static_cast<const struct link_map*>(handle);
    return elf_lookup_in(m->l_addr, m->l_ld, name);
  }
  const struct link_map* m = _r_debug.r_map;
  if (handle == RTLD_NEXT) {
    while (m && m->l_ld != _DYNAMIC) m = m->l_next;
    if (!m) return nullptr;   // the shim is not in the link map: nothing is "next"
    m = m->l_next;
  }
  for (; m; m = m->l_next)
    if (void* p = elf_lookup_in(m->l_addr, m->l_ld, name)) return p;
  return nullptr;
}
MIVGPU_NO_SANITIZE void* fallback_dlvsym(void* handle, const char* name, const char*) {
  return fallback_dlsym(handle, name);
}

using dlsym_fn = void* (*)(void*, const char*);
using dlvsym_fn = void* (*)(void*, const char*, const char*);
// Published once; a racing first use computes the same value (plain aligned
// pointer stores, read through volatile: no instrumented atomics here).
dlsym_fn g_real_dlsym = nullptr;
dlvsym_fn g_real_dlvsym = nullptr;

MIVGPU_NO_SANITIZE void warn_no_libc(const char* what) {
  static const char msg[] = "[mivgpu WARN] libc/libdl symbol not found, using the shim's own lookup: ";
  (void)!write(2, msg, sizeof(msg) - 1);
  size_t n = 0;
  while (what[n]) ++n;
  (void)!write(2, what, n);
  (void)!write(2, "\n", 1);
}

MIVGPU_NO_SANITIZE dlsym_fn libc_dlsym() {
  dlsym_fn f = *const_cast<volatile dlsym_fn*>(&g_real_dlsym);
  if (__builtin_expect(!f, 0)) {
    f = reinterpret_cast<dlsym_fn>(libc_sym("dlsym"));
    if (!f) {
      warn_no_libc("dlsym");
      f = &fallback_dlsym;
    }
    *const_cast<volatile dlsym_fn*>(&g_real_dlsym) = f;
  }
  return f;
}

MIVGPU_NO_SANITIZE dlvsym_fn libc_dlvsym() {
  dlvsym_fn f = *const_cast<volatile dlvsym_fn*>(&g_real_dlvsym);
  if (__builtin_expect(!f, 0)) {
    f = reinterpret_cast<dlvsym_fn>(libc_sym("dlvsym"));
    if (!f) {
      warn_no_libc("dlvsym");
      f = &fallback_dlvsym;
    }
    *const_cast<volatile dlvsym_fn*>(&g_real_dlvsym) = f;
  }
  return f;
}

// ----------------------------------------------------------- real symbols --
// A HIP runtime the process opened privately (RTLD_LOCAL, e.g. Triton's own
// copy when nothing else loaded one) and asked the shim's dlsym for a hooked
// entry point of: the hooks forward to it when no HIP library is global.
std::atomic<void*> g_hip_handle{nullptr};

template <typename F>
F resolve(const char* name, const char* version) {
  void* p = libc_dlvsym()(RTLD_NEXT, name, version);
  if (!p) p = libc_dlsym()(RTLD_NEXT, name);
  if (!p) {
    void* h = g_hip_handle.load(std::memory_order_acquire);
    // The shim may have been loaded before any HIP library (LD_PRELOAD into a
    // launcher); fall back to an explicit handle.
    if (!h) h = dlopen("libamdhip64.so", RTLD_LAZY | RTLD_GLOBAL | RTLD_NOLOAD);
    if (!h) h = dlopen("libamdhip64.so", RTLD_LAZY | RTLD_GLOBAL);
    if (h) {
      p = libc_dlvsym()(h, name, version);
      if (!p) p = libc_dlsym()(h, name);
    }
  }
  // (entry points newer than the runtime -- hip_6.5 launches on ROCm 6.4 --
  // are simply absent; their hooks report hipErrorNotSupported)
  if (!p) mlog(3, "cannot resolve real %s@%s", name, version);
  return reinterpret_cast<F>(p);
}

#define REAL_DECL(ret, name, ver, args)                                       \
  using name##_fn = ret(*) args;                                               \
  name##_fn real_##name() {                                                    \
    static name##_fn f = resolve<name##_fn>(#name, ver);                       \
    return f;                                                                  \
  }

REAL_DECL(hipError_t, hipMalloc, "hip_4.2", (void**, size_t))
REAL_DECL(hipError_t, hipFree, "hip_4.2", (void*))
REAL_DECL(hipError_t, hipMallocAsync, "hip_5.1", (void**, size_t, hipStream_t))
REAL_DECL(hipError_t, hipMallocFromPoolAsync, "hip_5.1", (void**, size_t, hipMemPool_t, hipStream_t))
REAL_DECL(hipError_t, hipFreeAsync, "hip_5.1", (void*, hipStream_t))
REAL_DECL(hipError_t, hipMallocManaged, "hip_4.2", (void**, size_t, unsigned int))
REAL_DECL(hipError_t, hipExtMallocWithFlags, "hip_4.2", (void**, size_t, unsigned int))
REAL_DECL(hipError_t, hipMallocPitch, "hip_4.2", (void**, size_t*, size_t, size_t))
REAL_DECL(hipError_t, hipMemAllocPitch, "hip_4.2", (hipDeviceptr_t*, size_t*, size_t, size_t, unsigned int))
REAL_DECL(hipError_t, hipMemCreate, "hip_5.1",
          (hipMemGenericAllocationHandle_t*, size_t, const hipMemAllocationProp*, unsigned long long))
REAL_DECL(hipError_t, hipMemRelease, "hip_5.1", (hipMemGenericAllocationHandle_t))
REAL_DECL(hipError_t, hipMemGetInfo, "hip_4.2", (size_t*, size_t*))
REAL_DECL(hipError_t, hipDeviceTotalMem, "hip_4.2", (size_t*, hipDevice_t))
REAL_DECL(hipError_t, hipGetDevicePropertiesR0600, "hip_6.0", (hipDeviceProp_tR0600*, int))
REAL_DECL(hipError_t, hipGetDevicePropertiesR0000, "hip_4.2", (void*, int))
REAL_DECL(hipError_t, hipLaunchKernel, "hip_4.2", (const void*, dim3, dim3, void**, size_t, hipStream_t))
REAL_DECL(hipError_t, hipLaunchKernel_spt, "hip_5.2", (const void*, dim3, dim3, void**, size_t, hipStream_t))
REAL_DECL(hipError_t, hipModuleLaunchKernel, "hip_4.2",
          (hipFunction_t, unsigned, unsigned, unsigned, unsigned, unsigned, unsigned, unsigned,
           hipStream_t, void**, void**))
REAL_DECL(hipError_t, hipExtModuleLaunchKernel, "hip_4.2",
          (hipFunction_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, size_t,
           hipStream_t, void**, void**, hipEvent_t, hipEvent_t, uint32_t))
REAL_DECL(hipError_t, hipHccModuleLaunchKernel, "hip_4.2",
          (hipFunction_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, size_t,
           hipStream_t, void**, void**, hipEvent_t, hipEvent_t))
REAL_DECL(hipError_t, hipLaunchCooperativeKernel, "hip_4.2",
          (const void*, dim3, dim3, void**, unsigned int, hipStream_t))
REAL_DECL(hipError_t, hipExtLaunchKernel, "hip_4.2",
          (const void*, dim3, dim3, void**, size_t, hipStream_t, hipEvent_t, hipEvent_t, int))
REAL_DECL(hipError_t, hipGraphLaunch, "hip_4.3", (hipGraphExec_t, hipStream_t))
REAL_DECL(hipError_t, hipGraphLaunch_spt, "hip_5.3", (hipGraphExec_t, hipStream_t))
REAL_DECL(hipError_t, hipModuleLaunchCooperativeKernel, "hip_5.5",
          (hipFunction_t, unsigned, unsigned, unsigned, unsigned, unsigned, unsigned, unsigned,
           hipStream_t, void**))
REAL_DECL(hipError_t, hipLaunchKernelExC, "hip_6.5", (const hipLaunchConfig_t*, const void*, void**))
REAL_DECL(hipError_t, hipDrvLaunchKernelEx, "hip_6.5",
          (const HIP_LAUNCH_CONFIG*, hipFunction_t, void**, void**))
REAL_DECL(hipError_t, hipLaunchCooperativeKernelMultiDevice, "hip_4.2", (hipLaunchParams*, int, unsigned int))
REAL_DECL(hipError_t, hipExtLaunchMultiKernelMultiDevice, "hip_4.2", (hipLaunchParams*, int, unsigned int))
REAL_DECL(hipError_t, hipMallocArray, "hip_4.2",
          (hipArray_t*, const hipChannelFormatDesc*, size_t, size_t, unsigned int))
REAL_DECL(hipError_t, hipMalloc3D, "hip_4.2", (hipPitchedPtr*, hipExtent))
REAL_DECL(hipError_t, hipMalloc3DArray, "hip_4.2",
          (hipArray_t*, const hipChannelFormatDesc*, hipExtent, unsigned int))
REAL_DECL(hipError_t, hipArrayCreate, "hip_4.2", (hipArray_t*, const HIP_ARRAY_DESCRIPTOR*))
REAL_DECL(hipError_t, hipArray3DCreate, "hip_4.2", (hipArray_t*, const HIP_ARRAY3D_DESCRIPTOR*))
REAL_DECL(hipError_t, hipMallocMipmappedArray, "hip_4.2",
          (hipMipmappedArray_t*, const hipChannelFormatDesc*, hipExtent, unsigned int, unsigned int))
REAL_DECL(hipError_t, hipMipmappedArrayCreate, "hip_4.2",
          (hipMipmappedArray_t*, HIP_ARRAY3D_DESCRIPTOR*, unsigned int))
REAL_DECL(hipError_t, hipFreeArray, "hip_4.2", (hipArray_t))
REAL_DECL(hipError_t, hipArrayDestroy, "hip_4.3", (hipArray_t))
REAL_DECL(hipError_t, hipFreeMipmappedArray, "hip_4.2", (hipMipmappedArray_t))
REAL_DECL(hipError_t, hipMipmappedArrayDestroy, "hip_4.2", (hipMipmappedArray_t))
REAL_DECL(hipError_t, hipModuleLoad, "hip_4.2", (hipModule_t*, const char*))
REAL_DECL(hipError_t, hipModuleLoadDataEx, "hip_4.2",
          (hipModule_t*, const void*, unsigned int, hipJitOption*, void**))
REAL_DECL(hipError_t, hipModuleUnload, "hip_4.2", (hipModule_t))
REAL_DECL(hipError_t, hipGetProcAddress, "hip_6.1",
          (const char*, void**, int, uint64_t, hipDriverProcAddressQueryResult*))
REAL_DECL(hipError_t, hipStreamGetDevice, "hip_4.2", (hipStream_t, hipDevice_t*))
// Not hooked, used by the shim itself.
REAL_DECL(hipError_t, hipGetDevice, "hip_4.2", (int*))
REAL_DECL(hipError_t, hipGetDeviceCount, "hip_4.2", (int*))
REAL_DECL(hipError_t, hipDeviceGetAttribute, "hip_4.2", (int*, hipDeviceAttribute_t, int))
REAL_DECL(hipError_t, hipStreamIsCapturing, "hip_4.3", (hipStream_t, hipStreamCaptureStatus*))
REAL_DECL(hipError_t, hipModuleLoadData, "hip_4.2", (hipModule_t*, const void*))
REAL_DECL(hipError_t, hipModuleGetFunction, "hip_4.2", (hipFunction_t*, hipModule_t, const char*))
REAL_DECL(hipError_t, hipHostMalloc, "hip_4.2", (void**, size_t, unsigned int))
REAL_DECL(hipError_t, hipHostFree, "hip_4.2", (void*))
REAL_DECL(hipError_t, hipHostGetDevicePointer, "hip_4.2", (void**, void*, unsigned int))
REAL_DECL(hipError_t, hipStreamSynchronize, "hip_4.2", (hipStream_t))
REAL_DECL(hipError_t, hipStreamSynchronize_spt, "hip_5.2", (hipStream_t))
REAL_DECL(hipError_t, hipDeviceSynchronize, "hip_4.2", (void))
REAL_DECL(hipError_t, hipStreamBeginCapture, "hip_4.3", (hipStream_t, hipStreamCaptureMode))
REAL_DECL(hipError_t, hipStreamBeginCaptureToGraph, "hip_6.1",
          (hipStream_t, hipGraph_t, const hipGraphNode_t*, const hipGraphEdgeData*, size_t, hipStreamCaptureMode))
REAL_DECL(hipError_t, hipStreamBeginCapture_spt, "hip_5.3", (hipStream_t, hipStreamCaptureMode))
REAL_DECL(hipError_t, hipStreamEndCapture, "hip_4.3", (hipStream_t, hipGraph_t*))
REAL_DECL(hipError_t, hipStreamEndCapture_spt, "hip_5.3", (hipStream_t, hipGraph_t*))
REAL_DECL(hipError_t, hipDeviceGetPCIBusId, "hip_4.2", (char*, int, int))
REAL_DECL(hipError_t, hipSetDevice, "hip_4.2", (int))
REAL_DECL(hipError_t, hipMemset, "hip_4.2", (void*, int, size_t))

// ------------------------------------------------------------------ config --
// A fixed contention window of the share estimator (ms) for measurement
// builds (-D, utils/build.py build_shim_variant); 0 = the adaptive default
// (per sample with few peers, 200 ms with many; profiles/README.md section 37).
#ifndef MIVGPU_PEER_BUSY_MS_DEFAULT
#define MIVGPU_PEER_BUSY_MS_DEFAULT 0
#endif

struct Config {
  uint64_t mem_limit[MIVGPU_MAX_DEVICES] = {0};
  int cu_limit[MIVGPU_MAX_DEVICES];  // percent per device (HIP_DEVICE_CORE_LIMIT[_i]), rounded half up
  // the same limit in parts per million of the device: the grant states the
  // CUs the scheduler charged as an exact share ("12.5" for 32 of 256 CUs),
  // which whole percents would cut (8 x 12 % left 4 % of the GPU idle)
  uint32_t cu_limit_ppm[MIVGPU_MAX_DEVICES];
  int cu_mask_count[MIVGPU_MAX_DEVICES] = {0};
  int policy = 0;              // 0 default, 1 force, 2 disable
  int priority = 1;
  bool oversubscribe = false;
  bool disabled = false;
  bool account_context = true;  // count runtime/code-object VRAM (KFD per-process view) in the quota
  uint64_t context_refresh_ns = 20000000;  // at most one KFD read per 20 ms (forced before an OOM)
  bool occupancy = true;                   // charge the governor the sampled wave-occupancy share
  uint64_t occ_period_ns = 2000000;        // sampling period while the governor runs (2 ms)
  // a fixed contention window (measurement builds; 0 = adaptive: per sample
  // with few busy peers, kPeerBusyNs with many)
  uint64_t peer_busy_ns = (uint64_t)MIVGPU_PEER_BUSY_MS_DEFAULT * 1000000ull;
  uint64_t occ_idle_period_ns = 50000000;  // ... and for utilisation reporting only (50 ms)
  double share_tau_ns = 250e6;             // EWMA time constant of the occupancy averages (>> holds, batches)
  // A/B switches (not grant keys, ignored under a grant file, see
  // unguarded_env): MIVGPU_GATE_MODE=device keeps the bucket
  // in the gate (busy wall time x share) instead of the sampler;
  // MIVGPU_SHARE_EST=instant averages the per-sample ratio own/(own+others)
  // (ratio: the ratio of the averaged wave counts) instead of counting the
  // contending tenants.
  bool gate_device_mode = false;
  bool share_instant = false;
  bool share_ratio = false;
  char kfd_sysfs[256] = "/sys/class/kfd/kfd";
  // The GPU's share board directory (board.h; grant key MIVGPU_BOARD_DIR,
  // "none" = off).  Default /tmp/mivgpu-board, or off when KFD sysfs is
  // redirected (tests: a fake KFD must not meet a real GPU's board).
  char board_dir[256] = "/tmp/mivgpu-board";
  char board_flags_dir[256] = "";   // this container's own flags directory ("" = <board_dir>/flags)
  uint64_t presence_ns = mivgpu_board::kPresenceNs;   // fair-share presence window when this shim owns the board
  // MIVGPU_BOARD_SPLIT=equal (A/B): a board owner splits each pass equally
  // among the processes with waves resident instead of by their waves
  int board_split = 0;
  uint64_t gate_min_interval_ns = 200000;  // >= 200 us of host submission per gate
  bool gate_trace = false;                 // gates also write their trace ring (mivgpu_gate_trace)
  int64_t gate_cap_ns = 100000000;         // 100 ms burst (absorbs share-measurement noise)
  double fair_lag_frac = 0.03;             // fair-share lag: this part of the GPU time received in the mode
  int64_t gate_max_hold_ns = 25000000;     // 25 ms per gate, bounds every spin (larger debts: later gates)
  char cache_path[512] = {0};
};
Config g_cfg;

uint64_t parse_size(const char* s) {
  if (!s || !*s) return 0;
  char* end = nullptr;
  double v = strtod(s, &end);
  if (end == s || v < 0) return 0;
  uint64_t mult = 1;
  if (end && *end) {
    switch (*end) {
      case 'k': case 'K': mult = 1ull << 10; break;
      case 'm': case 'M': mult = 1ull << 20; break;
      case 'g': case 'G': mult = 1ull << 30; break;
      case 't': case 'T': mult = 1ull << 40; break;
      default: mult = 1; break;
    }
  }
  return (uint64_t)(v * (double)mult);
}

// A core limit in percent with up to four decimals ("25", "12.5", "3.125")
// -> parts per million of the device; 0 = absent or outside (0, 100].
// Integer arithmetic only, so the monitor (shim/__init__.py core_limit_ppm)
// derives the same value from the same grant text.
uint32_t parse_pct_ppm(const char* s) {
  if (!s) return 0;
  uint64_t ip = 0, fp = 0;
  int idig = 0, fdig = 0;
  const char* p = s;
  for (; *p >= '0' && *p <= '9'; ++p, ++idig)
    if (idig < 4) ip = ip * 10 + (uint64_t)(*p - '0');
  if (idig > 3) return 0;
  if (*p == '.') {
    for (++p; *p >= '0' && *p <= '9'; ++p, ++fdig)
      if (fdig < 4) fp = fp * 10 + (uint64_t)(*p - '0');
  }
  if (*p || (idig == 0 && fdig == 0)) return 0;
  for (int k = fdig < 4 ? fdig : 4; k < 4; ++k) fp *= 10;
  const uint64_t ppm = ip * 10000 + fp;
  return (ppm > 0 && ppm <= 1000000) ? (uint32_t)ppm : 0;
}

// ppm -> whole percent for the region field, rounded half up, at least 1.
int pct_of_ppm(uint32_t ppm) {
  const int pct = (int)((ppm + 5000) / 10000);
  return ppm == 0 ? 0 : (pct < 1 ? 1 : pct);
}

// Count CUs granted to device `idx` in an HSA_CU_MASK value such as
// "0:0-63;1:0-31,64-95" (container-local device indices, HSA grammar).
int parse_cu_mask_count(const char* mask, int idx) {
  if (!mask) return 0;
  const char* p = mask;
  while (*p) {
    char* end = nullptr;
    long dev = strtol(p, &end, 10);
    if (end == p || *end != ':') return 0;
    p = end + 1;
    int count = 0;
    while (*p && *p != ';') {
      long a = strtol(p, &end, 10);
      if (end == p) return 0;
      long b = a;
      p = end;
      if (*p == '-') {
        ++p;
        b = strtol(p, &end, 10);
        if (end == p) return 0;
        p = end;
      }
      if (b >= a) count += (int)(b - a + 1);
      if (*p == ',') ++p;
    }
    if (dev == idx) return count;
    if (*p == ';') ++p;
  }
  return 0;
}

// ------------------------------------------------------------ limits file --
// The device plugin's Allocate writes the container's grant (memory limits,
// CU mask, core limit and policy, priority, visible devices, region path) to
// a host file mounted READ-ONLY at kLimitsPath.  When it exists it is the only
// source of those settings: a tenant that unsets or rewrites the environment
// (HSA_CU_MASK, HIP_DEVICE_MEMORY_LIMIT_0, MIVGPU_DISABLE_CONTROL ...) before
// the runtime starts gets exactly its grant anyway.  MIVGPU_LIMITS_FILE names
// a file only where the fixed path is absent (tests, hand-run slices).
constexpr const char* kLimitsPath = "/etc/mivgpu/limits.conf";
// No initialisers: zero-initialised static storage, so the interposed getenv
// can load it before this library's constructors run without a later dynamic
// initialiser wiping it.
struct LimitsFile {
  bool loaded;
  int n;
  char keys[48][64];
  char vals[48][448];
};
LimitsFile g_limits;
std::once_flag g_limits_once;

void read_limits_file() {
  const char* path = kLimitsPath;
  struct stat st;
  if (mivgpu_stat(path, &st) != 0) {
    const char* alt = getenv("MIVGPU_LIMITS_FILE");
    if (!alt || !*alt || mivgpu_stat(alt, &st) != 0) return;
    path = alt;
  }
  FILE* f = fopen(path, "re");
  if (!f) return;
  char line[560];
  while (fgets(line, sizeof(line), f) && g_limits.n < 48) {
    char* eq = strchr(line, '=');
    if (!eq || line[0] == '#') continue;
    *eq = 0;
    char* v = eq + 1;
    size_t lv = strlen(v);
    while (lv && (v[lv - 1] == '\n' || v[lv - 1] == '\r')) v[--lv] = 0;
    snprintf(g_limits.keys[g_limits.n], sizeof(g_limits.keys[0]), "%s", line);
    snprintf(g_limits.vals[g_limits.n], sizeof(g_limits.vals[0]), "%s", v);
    ++g_limits.n;
  }
  fclose(f);
  g_limits.loaded = true;
}

inline void ensure_limits() { std::call_once(g_limits_once, read_limits_file); }

// Settings that are part of the grant.  With a limits file they come from it
// alone (absent there = not granted); without one, from the environment.
bool is_grant_key(const char* key) {
  static const char* const kKeys[] = {"HIP_DEVICE_MEMORY_LIMIT", "HIP_DEVICE_CORE_LIMIT", "HSA_CU_MASK",
                                      "GPU_CORE_UTILIZATION_POLICY", "HIP_TASK_PRIORITY", "MIVGPU_OVERSUBSCRIBE",
                                      "MIVGPU_SHARED_CACHE", "MIVGPU_DEVICE_UUIDS", "MIVGPU_DISABLE_CONTROL",
                                      "MIVGPU_ACCOUNT_CONTEXT", "ROCR_VISIBLE_DEVICES", "MIVGPU_KFD_SYSFS",
                                      "MIVGPU_OCCUPANCY", "MIVGPU_OCC_PERIOD_US", "MIVGPU_GATE_INTERVAL_US",
                                      "MIVGPU_GATE_BURST_US", "MIVGPU_SHARE_TAU_MS", "GPU_MAX_HW_QUEUES",
                                      "MIVGPU_GATE_MAX_HOLD_US", "MIVGPU_CONTROL_FILE", "MIVGPU_BOARD_DIR",
                                      "MIVGPU_BOARD_FLAGS_DIR", "MIVGPU_FAIR_LAG_PCT"};
  for (const char* k : kKeys)
    if (!strcmp(key, k)) return true;
  return !strncmp(key, "HIP_DEVICE_MEMORY_LIMIT_", 24) || !strncmp(key, "HIP_DEVICE_CORE_LIMIT_", 22);
}

const char* grant_env(const char* key) {
  ensure_limits();
  if (!g_limits.loaded || !is_grant_key(key)) return getenv(key);
  for (int i = 0; i < g_limits.n; ++i)
    if (!strcmp(g_limits.keys[i], key)) return g_limits.vals[i];
  return nullptr;
}

// Measurement switches (A/B gate and share-estimator modes, the context
// refresh period): they change how a tenant is charged, so a container that
// runs under a grant file cannot set them -- honoured only for hand-run
// slices without one.
const char* unguarded_env(const char* key) {
  ensure_limits();
  return g_limits.loaded ? nullptr : getenv(key);
}

void load_config() {
  const char* lvl = getenv("MIVGPU_LOG_LEVEL");
  if (lvl) g_log_level = atoi(lvl);
  ensure_limits();
  if (g_limits.loaded) mlog(3, "grant read from the limits file (%d settings); environment overrides ignored", g_limits.n);
  const char* dis = grant_env("MIVGPU_DISABLE_CONTROL");
  g_cfg.disabled = dis && (!strcmp(dis, "1") || !strcasecmp(dis, "true"));
  const char* all = grant_env("HIP_DEVICE_MEMORY_LIMIT");
  uint64_t all_lim = parse_size(all);
  for (int i = 0; i < MIVGPU_MAX_DEVICES; ++i) {
    char key[64];
    snprintf(key, sizeof(key), "HIP_DEVICE_MEMORY_LIMIT_%d", i);
    uint64_t v = parse_size(grant_env(key));
    g_cfg.mem_limit[i] = v ? v : all_lim;
  }
  // HIP_DEVICE_CORE_LIMIT applies to every device; HIP_DEVICE_CORE_LIMIT_<i>
  // (container-local index) overrides it for one device, so a container that
  // holds a compute partition next to a whole GPU is governed per device.
  uint32_t core_all = 1000000;
  const uint32_t core = parse_pct_ppm(grant_env("HIP_DEVICE_CORE_LIMIT"));
  if (core) core_all = core;
  for (int i = 0; i < MIVGPU_MAX_DEVICES; ++i) {
    char key[64];
    snprintf(key, sizeof(key), "HIP_DEVICE_CORE_LIMIT_%d", i);
    const uint32_t c = parse_pct_ppm(grant_env(key));
    g_cfg.cu_limit_ppm[i] = c ? c : core_all;
    g_cfg.cu_limit[i] = pct_of_ppm(g_cfg.cu_limit_ppm[i]);
  }
  const char* mask = grant_env("HSA_CU_MASK");
  for (int i = 0; i < MIVGPU_MAX_DEVICES; ++i) g_cfg.cu_mask_count[i] = parse_cu_mask_count(mask, i);
  const char* pol = grant_env("GPU_CORE_UTILIZATION_POLICY");
  if (pol) {
    if (!strcasecmp(pol, "force")) g_cfg.policy = 1;
    else if (!strcasecmp(pol, "disable")) g_cfg.policy = 2;
  }
  const char* pri = grant_env("HIP_TASK_PRIORITY");
  if (pri) g_cfg.priority = atoi(pri);
  const char* ov = grant_env("MIVGPU_OVERSUBSCRIBE");
  g_cfg.oversubscribe = ov && (!strcmp(ov, "1") || !strcasecmp(ov, "true"));
  const char* ac = grant_env("MIVGPU_ACCOUNT_CONTEXT");
  g_cfg.account_context = !(ac && (!strcmp(ac, "0") || !strcasecmp(ac, "false")));
  const char* oc = grant_env("MIVGPU_OCCUPANCY");
  g_cfg.occupancy = !(oc && (!strcmp(oc, "0") || !strcasecmp(oc, "false")));
  const char* op = grant_env("MIVGPU_OCC_PERIOD_US");
  if (op && atoll(op) >= 200) g_cfg.occ_period_ns = (uint64_t)atoll(op) * 1000ull;
  if (const char* pb = unguarded_env("MIVGPU_PEER_BUSY_MS")) g_cfg.peer_busy_ns = (uint64_t)atoll(pb) * 1000000ull;
  const char* gm = unguarded_env("MIVGPU_GATE_MODE");
  g_cfg.gate_device_mode = gm && !strcmp(gm, "device");
  const char* se = unguarded_env("MIVGPU_SHARE_EST");
  g_cfg.share_instant = se && !strcmp(se, "instant");
  g_cfg.share_ratio = se && !strcmp(se, "ratio");
  const char* tau = grant_env("MIVGPU_SHARE_TAU_MS");
  if (tau && atof(tau) > 0) g_cfg.share_tau_ns = atof(tau) * 1e6;
  const char* crm = unguarded_env("MIVGPU_CONTEXT_REFRESH_MS");
  if (crm && *crm) g_cfg.context_refresh_ns = (uint64_t)atoll(crm) * 1000000ull;
  const char* kfd = grant_env("MIVGPU_KFD_SYSFS");
  if (kfd && *kfd) {
    snprintf(g_cfg.kfd_sysfs, sizeof(g_cfg.kfd_sysfs), "%s", kfd);
    g_cfg.board_dir[0] = 0;
  }
  const char* bd = grant_env("MIVGPU_BOARD_DIR");
  if (bd) snprintf(g_cfg.board_dir, sizeof(g_cfg.board_dir), "%s", strcmp(bd, "none") ? bd : "");
  const char* bfd = grant_env("MIVGPU_BOARD_FLAGS_DIR");
  if (bfd && *bfd) snprintf(g_cfg.board_flags_dir, sizeof(g_cfg.board_flags_dir), "%s", bfd);
  const char* pw = unguarded_env("MIVGPU_PRESENCE_WINDOW_US");
  if (pw && *pw) g_cfg.presence_ns = (uint64_t)atoll(pw) * 1000ull;
  const char* bs = unguarded_env("MIVGPU_BOARD_SPLIT");
  g_cfg.board_split = bs && !strcmp(bs, "equal") ? mivgpu_board::kSplitEqual : mivgpu_board::kSplitRatio;
  const char* gt = getenv("MIVGPU_GATE_TRACE");
  g_cfg.gate_trace = gt && (!strcmp(gt, "1") || !strcasecmp(gt, "true"));
  // fair-share lag: percent of the GPU time received in the mode (grant key)
  const char* fl = grant_env("MIVGPU_FAIR_LAG_PCT");
  if (fl && atof(fl) >= 0 && atof(fl) <= 50) g_cfg.fair_lag_frac = atof(fl) / 100.0;
  const char* gi = grant_env("MIVGPU_GATE_INTERVAL_US");
  if (gi) g_cfg.gate_min_interval_ns = (uint64_t)atoll(gi) * 1000ull;
  const char* cap = grant_env("MIVGPU_GATE_BURST_US");
  if (cap) g_cfg.gate_cap_ns = (int64_t)atoll(cap) * 1000;
  const char* mh = grant_env("MIVGPU_GATE_MAX_HOLD_US");
  if (mh && atoll(mh) >= 100) g_cfg.gate_max_hold_ns = (int64_t)atoll(mh) * 1000;
  const char* path = grant_env("MIVGPU_SHARED_CACHE");
  if (path && *path) {
    snprintf(g_cfg.cache_path, sizeof(g_cfg.cache_path), "%s", path);
  } else {
    snprintf(g_cfg.cache_path, sizeof(g_cfg.cache_path), "/tmp/mivgpu/%d.cache", (int)getpid());
  }
}

// ------------------------------------------------------------ shared region --
mivgpu_shared_region_t* g_region = nullptr;
int g_slot = -1;
int g_num_devices = 0;

pthread_mutex_t* region_lock() { return reinterpret_cast<pthread_mutex_t*>(g_region->lock); }

void lock_region() {
  int rc = pthread_mutex_lock(region_lock());
  if (rc == EOWNERDEAD) {
    mlog(1, "previous owner of the shared-region lock died; recovering");
    pthread_mutex_consistent(region_lock());
  }
}
void unlock_region() { pthread_mutex_unlock(region_lock()); }

bool pid_alive(int pid) {
  if (pid <= 0) return false;
  if (kill(pid, 0) == 0) return true;
  return errno != ESRCH;
}

// Release a dead process's usage.  Caller holds the region lock.
void reclaim_slot_locked(int i) {
  mivgpu_proc_slot_t* s = &g_region->procs[i];
  for (int d = 0; d < MIVGPU_MAX_DEVICES; ++d) {
    uint64_t t = __atomic_load_n(&s->used[d].total, __ATOMIC_RELAXED);
    if (t) __atomic_fetch_sub(&g_region->dev_used[d], t, __ATOMIC_RELAXED);
  }
  memset(s, 0, sizeof(*s));
}

int reclaim_dead_locked() {
  int n = 0;
  int hi = g_region->procnum;
  for (int i = 0; i < hi && i < MIVGPU_MAX_PROCS; ++i) {
    mivgpu_proc_slot_t* s = &g_region->procs[i];
    if (s->status == MIVGPU_SLOT_ACTIVE && i != g_slot && !pid_alive(s->pid)) {
      mlog(3, "reclaiming slot %d of dead pid %d", i, s->pid);
      reclaim_slot_locked(i);
      ++n;
    }
  }
  return n;
}

void fill_uuids_locked() {
  // UUIDs are informational for the monitor (it matches them against the
  // allocation annotation); take them from MIVGPU_DEVICE_UUIDS if the device
  // plugin provided them, otherwise leave the index.
  const char* ids = grant_env("MIVGPU_DEVICE_UUIDS");
  int i = 0;
  if (ids) {
    const char* p = ids;
    while (*p && i < MIVGPU_MAX_DEVICES) {
      const char* c = strchr(p, ',');
      size_t n = c ? (size_t)(c - p) : strlen(p);
      if (n >= MIVGPU_UUID_LEN) n = MIVGPU_UUID_LEN - 1;
      memcpy(g_region->uuids[i], p, n);
      g_region->uuids[i][n] = 0;
      ++i;
      if (!c) break;
      p = c + 1;
    }
  }
  for (; i < g_num_devices && i < MIVGPU_MAX_DEVICES; ++i) {
    if (!g_region->uuids[i][0]) snprintf(g_region->uuids[i], MIVGPU_UUID_LEN, "hip-device-%d", i);
  }
}

bool open_region() {
  char dir[512];
  snprintf(dir, sizeof(dir), "%s", g_cfg.cache_path);
  char* slash = strrchr(dir, '/');
  if (slash && slash != dir) {
    *slash = 0;
    mkdir(dir, 0777);
  }
  int fd = open(g_cfg.cache_path, O_RDWR | O_CREAT, 0666);
  if (fd < 0) {
    mlog(1, "cannot open shared cache %s: %s (running with a private region)", g_cfg.cache_path,
         strerror(errno));
    void* p = mmap(nullptr, sizeof(mivgpu_shared_region_t), PROT_READ | PROT_WRITE,
                   MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return false;
    g_region = static_cast<mivgpu_shared_region_t*>(p);
  } else {
    flock(fd, LOCK_EX);
    struct stat st;
    mivgpu_fstat(fd, &st);
    if ((size_t)st.st_size < sizeof(mivgpu_shared_region_t)) {
      if (ftruncate(fd, sizeof(mivgpu_shared_region_t)) != 0) {
        mlog(0, "ftruncate(%s) failed: %s", g_cfg.cache_path, strerror(errno));
      }
    }
    void* p = mmap(nullptr, sizeof(mivgpu_shared_region_t), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (p == MAP_FAILED) {
      flock(fd, LOCK_UN);
      close(fd);
      return false;
    }
    g_region = static_cast<mivgpu_shared_region_t*>(p);
    if (g_region->magic != MIVGPU_MAGIC || g_region->major_version != MIVGPU_MAJOR) {
      memset(g_region, 0, sizeof(*g_region) - sizeof(g_region->procs));
      memset(g_region->procs, 0, sizeof(g_region->procs));
      pthread_mutexattr_t a;
      pthread_mutexattr_init(&a);
      pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
      pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
      pthread_mutex_init(region_lock(), &a);
      pthread_mutexattr_destroy(&a);
      g_region->major_version = MIVGPU_MAJOR;
      g_region->minor_version = MIVGPU_MINOR;
      g_region->owner_pid = (uint64_t)getpid();
      g_region->priority = g_cfg.priority;
      g_region->core_policy = g_cfg.policy;
      g_region->oversubscribe = g_cfg.oversubscribe ? 1 : 0;
      for (int d = 0; d < MIVGPU_MAX_DEVICES; ++d) {
        g_region->mem_limit[d] = g_cfg.mem_limit[d];
        g_region->cu_limit[d] = (uint64_t)g_cfg.cu_limit[d];
        g_region->cu_mask_count[d] = (uint64_t)g_cfg.cu_mask_count[d];
      }
      __atomic_store_n(&g_region->magic, MIVGPU_MAGIC, __ATOMIC_RELEASE);
      g_region->initialized = 1;
    }
    flock(fd, LOCK_UN);
    close(fd);
  }
  if (g_region->magic != MIVGPU_MAGIC) {  // private anonymous region
    pthread_mutexattr_t a;
    pthread_mutexattr_init(&a);
    pthread_mutex_init(region_lock(), &a);
    g_region->magic = MIVGPU_MAGIC;
    g_region->major_version = MIVGPU_MAJOR;
    g_region->minor_version = MIVGPU_MINOR;
    for (int d = 0; d < MIVGPU_MAX_DEVICES; ++d) {
      g_region->mem_limit[d] = g_cfg.mem_limit[d];
      g_region->cu_limit[d] = (uint64_t)g_cfg.cu_limit[d];
      g_region->cu_mask_count[d] = (uint64_t)g_cfg.cu_mask_count[d];
    }
    g_region->initialized = 1;
  }
  // Claim a process slot.
  lock_region();
  reclaim_dead_locked();
  for (int i = 0; i < MIVGPU_MAX_PROCS; ++i) {
    mivgpu_proc_slot_t* s = &g_region->procs[i];
    if (s->status == MIVGPU_SLOT_ACTIVE && s->pid == getpid()) {  // re-init after fork+exec reuse
      reclaim_slot_locked(i);
    }
    if (s->status == MIVGPU_SLOT_FREE) {
      memset(s, 0, sizeof(*s));
      s->pid = getpid();
      s->hostpid = 0;
      s->priority = g_cfg.priority;
      s->start_ns = mono_ns();
      s->heartbeat_ns = s->start_ns;
      __atomic_store_n(&s->status, MIVGPU_SLOT_ACTIVE, __ATOMIC_RELEASE);
      g_slot = i;
      if (i + 1 > g_region->procnum) g_region->procnum = i + 1;
      break;
    }
  }
  g_region->num_devices = (uint64_t)g_num_devices;
  fill_uuids_locked();
  unlock_region();
  if (g_slot < 0) mlog(0, "no free process slot in %s", g_cfg.cache_path);
  return true;
}

// Set first thing at exit: the background threads (governor stamper,
// occupancy sampler) stop issuing HIP calls before the runtime tears down.
std::atomic<bool> g_exiting{false};
void quiesce_background_threads();

void housekeeping_final();

void on_exit_release() {
  g_exiting.store(true, std::memory_order_release);
  quiesce_background_threads();
  if (g_region) housekeeping_final();
  if (!g_region || g_slot < 0) return;
  lock_region();
  reclaim_slot_locked(g_slot);
  unlock_region();
  g_slot = -1;
}

// ----------------------------------------------------------- control file --
// The monitor's verdicts (shared_region.h mivgpu_control_t): mapped read-only,
// so neither a block nor the host-measured excess can be cleared from inside
// the container.  Named by the grant (MIVGPU_CONTROL_FILE, a grant key: with
// a grant file only the device plugin can point it anywhere).
const mivgpu_control_t* g_ctl = nullptr;
// Under a grant file the core limits are fixed: whether any device has one is
// computed once at bootstrap (-1: no grant file, read the region per launch).
int g_any_limit_static = -1;

void open_control() {
  const char* path = grant_env("MIVGPU_CONTROL_FILE");
  if (!path || !*path) return;
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    mlog(1, "control file %s: %s (monitor verdicts only through the shared region)", path, strerror(errno));
    return;
  }
  struct stat st;
  if (mivgpu_fstat(fd, &st) == 0 && (size_t)st.st_size >= sizeof(mivgpu_control_t)) {
    void* p = mmap(nullptr, sizeof(mivgpu_control_t), PROT_READ, MAP_SHARED, fd, 0);
    if (p != MAP_FAILED) g_ctl = static_cast<const mivgpu_control_t*>(p);
  } else {
    mlog(1, "control file %s is too short; ignored", path);
  }
  close(fd);
}

inline int64_t realtime_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME_COARSE, &ts);
  return (int64_t)ts.tv_sec * 1000000000ll + (int64_t)ts.tv_nsec;
}

// The verdicts hold while the monitor's lease is live.
inline bool ctl_live() {
  return g_ctl && __atomic_load_n(&g_ctl->magic, __ATOMIC_ACQUIRE) == MIVGPU_CTL_MAGIC &&
         realtime_ns() < __atomic_load_n(&g_ctl->lease_until_ns, __ATOMIC_RELAXED);
}
inline bool ctl_block() {
  return g_ctl && __atomic_load_n(&g_ctl->block, __ATOMIC_RELAXED) != 0 && ctl_live();
}
inline bool ctl_over() {
  return g_ctl && __atomic_load_n(&g_ctl->over_grant, __ATOMIC_RELAXED) != 0 && ctl_live();
}
inline uint64_t ctl_excess(int dev) {
  if (!g_ctl || !__atomic_load_n(&g_ctl->host_excess[dev], __ATOMIC_RELAXED) || !ctl_live()) return 0;
  return __atomic_load_n(&g_ctl->host_excess[dev], __ATOMIC_RELAXED);
}

// --------------------------------------------------------- lazy bootstrap --
pthread_once_t g_once = PTHREAD_ONCE_INIT;
std::atomic<bool> g_ready{false};

void bootstrap() {
  Guard g;
  load_config();
  {
    Dl_info di;
    char dir[1024] = {0};
    if (real_hipGetDevice() && dladdr(reinterpret_cast<void*>(real_hipGetDevice()), &di) && di.dli_fname) {
      snprintf(dir, sizeof(dir), "%s", di.dli_fname);
      char* slash = strrchr(dir, '/');
      if (slash) *slash = 0; else dir[0] = 0;
    }
    roctx_init(dir[0] ? dir : nullptr);
  }
  int n = 0;
  if (real_hipGetDeviceCount() && real_hipGetDeviceCount()(&n) == hipSuccess) g_num_devices = n;
  if (g_num_devices > MIVGPU_MAX_DEVICES) g_num_devices = MIVGPU_MAX_DEVICES;
  if (!open_region()) {
    mlog(0, "shared region unavailable; memory limits enforced per process only");
  }
  open_control();
  if (g_limits.loaded) {
    g_any_limit_static = 0;
    for (int d = 0; d < (g_num_devices > 0 ? g_num_devices : 1); ++d)
      if (g_cfg.cu_limit_ppm[d] > 0 && g_cfg.cu_limit_ppm[d] < 1000000) g_any_limit_static = 1;
  }
  atexit(on_exit_release);
  for (int d = 0; d < g_num_devices; ++d) {
    if (g_cfg.mem_limit[d] || g_cfg.cu_limit_ppm[d] < 1000000 || g_cfg.cu_mask_count[d])
      tmark("mivgpu:config dev=%d limit_mib=%llu cu_limit=%d cu_mask=%d cu_limit_ppm=%u", d,
            (unsigned long long)(g_cfg.mem_limit[d] >> 20), g_cfg.cu_limit[d], g_cfg.cu_mask_count[d],
            g_cfg.cu_limit_ppm[d]);
    if (g_cfg.mem_limit[d])
      mlog(3, "device %d: HBM limit %llu MiB, CU limit %d%%, CU mask %d CUs", d,
           (unsigned long long)(g_cfg.mem_limit[d] >> 20), g_cfg.cu_limit[d], g_cfg.cu_mask_count[d]);
  }
  g_ready.store(true, std::memory_order_release);
}

inline void ensure_init() {
  if (__builtin_expect(!g_ready.load(std::memory_order_acquire), 0)) pthread_once(&g_once, bootstrap);
}

inline int current_device() {
  // one visible device (the common pod): no runtime call on the launch path
  if (g_num_devices == 1) return 0;
  int d = 0;
  if (real_hipGetDevice()) (void)real_hipGetDevice()(&d);  // on failure: device 0
  if (d < 0 || d >= MIVGPU_MAX_DEVICES) d = 0;
  return d;
}

// The enforced grant.  Under a grant file it is the file's (host-owned,
// read-only): the region's copies sit in tenant-writable memory and are only
// mirrors for the monitor.  Without one (hand-run slices) the region's values
// rule, so a region-level limit change reaches every process of the container.
inline uint64_t limit_of(int dev) {
  if (g_cfg.disabled) return 0;
  if (g_limits.loaded || !g_region) return g_cfg.mem_limit[dev];
  return __atomic_load_n(&g_region->mem_limit[dev], __ATOMIC_RELAXED);
}
// The core limit in parts per million of the device.  The region holds it in
// whole percents (the monitor's field); while it still holds the percent this
// process published, the exact share from the grant stands, a changed value
// (the monitor's reconcile, a hand-run slice) is taken as it is.
inline uint64_t cu_limit_ppm_of(int dev) {
  if (g_limits.loaded || !g_region) return g_cfg.cu_limit_ppm[dev];
  const uint64_t pct = __atomic_load_n(&g_region->cu_limit[dev], __ATOMIC_RELAXED);
  return pct == (uint64_t)g_cfg.cu_limit[dev] ? g_cfg.cu_limit_ppm[dev] : pct * 10000ull;
}
inline uint64_t cu_mask_of(int dev) {
  if (g_limits.loaded || !g_region) return (uint64_t)g_cfg.cu_mask_count[dev];
  return __atomic_load_n(&g_region->cu_mask_count[dev], __ATOMIC_RELAXED);
}
inline int core_policy() {
  if (g_limits.loaded || !g_region) return g_cfg.policy;
  return __atomic_load_n(&g_region->core_policy, __ATOMIC_RELAXED);
}
// The monitor's contention switch (feedback.go:74-134): from the control file
// when there is one, else from the region.
inline int util_switch() {
  if (g_ctl) {
    // the flag first: the lease check (a clock read) only when it is set
    const int sw = __atomic_load_n(&g_ctl->utilization_switch, __ATOMIC_RELAXED);
    return sw && ctl_live() ? sw : 0;
  }
  return g_region ? __atomic_load_n(&g_region->utilization_switch, __ATOMIC_RELAXED) : 0;
}

// ------------------------------------------------------ allocation tracker --
enum AllocKind : uint8_t { K_BUFFER = 0, K_VMM = 1, K_HOST_SPILL = 2, K_MODULE = 3 };
struct AllocRec {
  uint64_t size;
  int16_t dev;
  uint8_t kind;
};

constexpr int kShards = 32;
struct Shard {
  std::mutex mu;
  std::unordered_map<uintptr_t, AllocRec> map;
};
Shard g_shards[kShards];

inline Shard& shard_of(uintptr_t key) { return g_shards[(key >> 12) % kShards]; }

void account_slot_add(int dev, uint64_t bytes, AllocKind kind) {
  if (g_slot >= 0) {
    mivgpu_mem_t* m = &g_region->procs[g_slot].used[dev];
    __atomic_fetch_add(kind == K_VMM ? &m->vmm : kind == K_MODULE ? &m->module : &m->buffer, bytes, __ATOMIC_RELAXED);
    uint64_t t = __atomic_add_fetch(&m->total, bytes, __ATOMIC_RELAXED);
    uint64_t pk = __atomic_load_n(&m->peak, __ATOMIC_RELAXED);
    while (t > pk && !__atomic_compare_exchange_n(&m->peak, &pk, t, true, __ATOMIC_RELAXED,
                                                  __ATOMIC_RELAXED)) {
    }
  }
}

void account_add(int dev, uint64_t bytes, AllocKind kind) {
  if (!g_region) return;
  __atomic_fetch_add(&g_region->dev_used[dev], bytes, __ATOMIC_RELAXED);
  account_slot_add(dev, bytes, kind);
}

void account_sub(int dev, uint64_t bytes, AllocKind kind) {
  if (!g_region) return;
  __atomic_fetch_sub(&g_region->dev_used[dev], bytes, __ATOMIC_RELAXED);
  if (g_slot >= 0) {
    mivgpu_mem_t* m = &g_region->procs[g_slot].used[dev];
    __atomic_fetch_sub(kind == K_VMM ? &m->vmm : kind == K_MODULE ? &m->module : &m->buffer, bytes, __ATOMIC_RELAXED);
    __atomic_fetch_sub(&m->total, bytes, __ATOMIC_RELAXED);
  }
}

// ------------------------------------------------ context / code-object VRAM --
// VRAM a process holds outside the hooked allocators -- HIP/ROCr pools,
// kernarg and signal buffers, code objects, scratch -- is invisible to the
// hooks (SURVEY.md 7.5 "memory accounting truthfulness"; the reference's
// libvgpu reconciles the same gap against NVML).  KFD publishes the process's
// total VRAM per GPU in <kfd>/proc/<pid>/vram_<gpu_id>; the shim charges
// context = that - (buffer + vmm) to the slot and to the container's quota,
// so the hard limit covers everything the process holds on the device.
// Refreshed at most every 20 ms, from the allocation and meminfo hooks.
struct CtxDev {
  int gpu_id = -2;        // KFD gpu_id of the HIP device (-2 unresolved, -1 unavailable)
  int kfd_pid = -2;       // KFD's name for this process (-2 unresolved, -1 unavailable)
  uint64_t last_ns = 0;
};
CtxDev g_ctx[MIVGPU_MAX_DEVICES];
std::mutex g_ctx_mu;
// Stream captures in flight (begin/end hooks): the pid probe below frees
// memory, which a global-mode capture forbids, so it waits for none.
std::atomic<int> g_captures{0};

bool read_u64_file(const char* path, uint64_t* out) {
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  char buf[64];
  ssize_t n = read(fd, buf, sizeof(buf) - 1);
  close(fd);
  if (n <= 0) return false;
  buf[n] = 0;
  char* end = nullptr;
  unsigned long long v = strtoull(buf, &end, 10);
  if (end == buf) return false;
  *out = v;
  return true;
}

// Physical CUs of each device (KFD topology simd_count / simd_per_cu, else
// HIP's multiprocessor count); 0 = not known yet.
std::atomic<int> g_dev_cus[MIVGPU_MAX_DEVICES];
// XCDs (KFD num_xcc) of each device: the CU-mask granule is one CU per XCD.
std::atomic<int> g_dev_xcds[MIVGPU_MAX_DEVICES];

int device_xcds(int dev) {
  const int n = g_dev_xcds[dev].load(std::memory_order_relaxed);
  return n > 0 ? n : 8;   // MI355X: 8 XCDs
}

int device_cus(int dev) {
  int n = g_dev_cus[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (real_hipDeviceGetAttribute() &&
      real_hipDeviceGetAttribute()(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) {
    g_dev_cus[dev].store(n, std::memory_order_relaxed);
    return n;
  }
  return 256;
}

// KFD topology node of HIP device `dev`: match the PCI domain and bus/device
// (location_id = bus << 8 | device << 3 | function) against every GPU node;
// an ambiguous match (several nodes behind one function) leaves it unknown.
int resolve_kfd_gpu_id(int dev) {
  if (!real_hipDeviceGetAttribute()) return -1;
  int bus = 0, slot = 0, domain = 0;
  if (real_hipDeviceGetAttribute()(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
      real_hipDeviceGetAttribute()(&slot, hipDeviceAttributePciDeviceId, dev) != hipSuccess ||
      real_hipDeviceGetAttribute()(&domain, hipDeviceAttributePciDomainId, dev) != hipSuccess)
    return -1;
  int found = -1, matches = 0;
  for (int node = 0; node < 256; ++node) {
    char path[512];
    snprintf(path, sizeof(path), "%s/topology/nodes/%d/properties", g_cfg.kfd_sysfs, node);
    FILE* f = fopen(path, "re");
    if (!f) {
      if (node > 0) break;  // nodes are numbered densely from 0
      continue;
    }
    long long loc = -1, dom = -1, simds = 0, simd_per_cu = 0, xcc = 0;
    char key[96];
    long long val;
    while (fscanf(f, "%95s %lld", key, &val) == 2) {
      if (!strcmp(key, "location_id")) loc = val;
      else if (!strcmp(key, "domain")) dom = val;
      else if (!strcmp(key, "simd_count")) simds = val;
      else if (!strcmp(key, "simd_per_cu")) simd_per_cu = val;
      else if (!strcmp(key, "num_xcc")) xcc = val;
    }
    fclose(f);
    uint64_t gid = 0;
    snprintf(path, sizeof(path), "%s/topology/nodes/%d/gpu_id", g_cfg.kfd_sysfs, node);
    if (!read_u64_file(path, &gid) || gid == 0) continue;  // CPU node
    if (loc < 0 || (loc >> 8) != bus || ((loc >> 3) & 0x1f) != slot || (dom >= 0 && dom != domain)) continue;
    ++matches;
    found = (int)gid;
    if (simds > 0 && simd_per_cu > 0) g_dev_cus[dev].store((int)(simds / simd_per_cu), std::memory_order_relaxed);
    if (xcc > 0) g_dev_xcds[dev].store((int)xcc, std::memory_order_relaxed);
  }
  return matches == 1 ? found : -1;
}

// KFD names /proc/<pid> by the host pid, which a process in a container's pid
// namespace does not know (the monitor fills slot->hostpid when it runs with
// hostPID; before that, or without it, the shim finds itself): snapshot
// vram_<gpu_id> of every KFD process, make one distinctive allocation through
// the real allocator, and keep the single process whose VRAM grew by exactly
// that much.  Three attempts with different sizes; ambiguity -> unavailable.
int probe_kfd_pid(int gpu_id) {
  if (!real_hipMalloc() || !real_hipFree()) return -1;
  char dir[512];
  snprintf(dir, sizeof(dir), "%s/proc", g_cfg.kfd_sysfs);
  for (int attempt = 0; attempt < 3; ++attempt) {
    std::vector<std::pair<int, uint64_t>> before;
    DIR* d = opendir(dir);
    if (!d) return -1;
    while (struct dirent* e = readdir(d)) {
      char* end = nullptr;
      long pid = strtol(e->d_name, &end, 10);
      if (end == e->d_name || *end || pid <= 0) continue;
      char path[640];
      uint64_t v = 0;
      snprintf(path, sizeof(path), "%s/%ld/vram_%d", dir, pid, gpu_id);
      if (read_u64_file(path, &v)) before.emplace_back((int)pid, v);
    }
    closedir(d);
    if (before.empty()) return -1;
    // per-process sizes (64-298 MiB in 6 MiB steps): tenants that start
    // together and probe at the same instant still see distinct deltas
    const uint64_t seed = (mono_ns() >> 10) ^ ((uint64_t)getpid() * 0x9E3779B97F4A7C15ull);
    const uint64_t probe = (64ull + 6ull * ((seed + 17ull * (uint64_t)attempt) % 40ull)) << 20;
    void* p = nullptr;
    if (real_hipMalloc()(&p, probe) != hipSuccess || !p) return -1;
    int found = -1, hits = 0;
    for (auto& pv : before) {
      char path[640];
      uint64_t v = 0;
      snprintf(path, sizeof(path), "%s/%d/vram_%d", dir, pv.first, gpu_id);
      if (read_u64_file(path, &v) && v >= pv.second + probe && v < pv.second + probe + (4ull << 20)) {
        found = pv.first;
        ++hits;
      }
    }
    (void)real_hipFree()(p);
    if (hits == 1) return found;
  }
  return -1;
}

// KFD's names for this process on `dev`: the GPU's gpu_id and the process's
// KFD pid.  Resolved once (the gpu_id from the topology, the pid from the
// monitor's hostpid mapping or the shim's own probe); the caller holds
// g_ctx_mu.  Used by the context accounting and the occupancy sampler.
bool kfd_identity_locked(int dev, int* gid, int* pid, bool may_probe) {
  CtxDev& c = g_ctx[dev];
  if (c.gpu_id == -1) return false;
  if (c.gpu_id == -2) {
    c.gpu_id = resolve_kfd_gpu_id(dev);
    if (c.gpu_id < 0) {
      mlog(3, "device %d: no KFD node matched; runtime VRAM and occupancy unavailable", dev);
      return false;
    }
  }
  mivgpu_proc_slot_t* s = &g_region->procs[g_slot];
  int p = __atomic_load_n(&s->hostpid, __ATOMIC_RELAXED);  // the monitor's mapping wins
  if (p <= 0) {
    if (c.kfd_pid == -2) {
      // the probe allocates on the calling thread's device: only from a hook
      if (!may_probe || g_captures.load(std::memory_order_acquire) > 0) return false;
      c.kfd_pid = probe_kfd_pid(c.gpu_id);
      if (c.kfd_pid < 0) {
        mlog(3, "device %d: own KFD process entry not identified; runtime VRAM and occupancy unavailable", dev);
      } else {
        int zero = 0;
        __atomic_compare_exchange_n(&s->hostpid, &zero, c.kfd_pid, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED);
      }
    }
    p = c.kfd_pid;
  }
  if (p <= 0) return false;
  *gid = c.gpu_id;
  *pid = p;
  return true;
}

// Returns true when the context charge went down (a forced refresh before an
// OOM verdict: the charge read between a hooked free's accounting and the real
// free can briefly count the freed buffer as context).
bool refresh_context(int dev, bool force) {
  if (!g_region || g_slot < 0 || dev < 0 || dev >= MIVGPU_MAX_DEVICES) return false;
  if (!g_cfg.account_context && !g_cfg.occupancy) return false;
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  CtxDev& c = g_ctx[dev];
  uint64_t now = coarse_ns();
  if (c.gpu_id == -1 || (!force && c.last_ns && now - c.last_ns < g_cfg.context_refresh_ns)) return false;
  c.last_ns = now;
  int gpu_id = -1, pid = -1;
  if (!kfd_identity_locked(dev, &gpu_id, &pid, true) || !g_cfg.account_context) return false;
  mivgpu_proc_slot_t* s = &g_region->procs[g_slot];
  char path[512];
  uint64_t vram = 0;
  snprintf(path, sizeof(path), "%s/proc/%d/vram_%d", g_cfg.kfd_sysfs, pid, gpu_id);
  if (!read_u64_file(path, &vram)) return false;
  mivgpu_mem_t* m = &s->used[dev];
  // code objects loaded through the module hooks are charged as `module`;
  // context is the rest of what KFD counts, so context + module + buffer +
  // vmm is KFD's number whenever the hooked bytes fit in it
  uint64_t hooked = __atomic_load_n(&m->buffer, __ATOMIC_RELAXED) + __atomic_load_n(&m->vmm, __ATOMIC_RELAXED) +
                    __atomic_load_n(&m->module, __ATOMIC_RELAXED);
  uint64_t ctx = vram > hooked ? vram - hooked : 0;
  uint64_t old = __atomic_exchange_n(&m->context, ctx, __ATOMIC_RELAXED);
  if (ctx == old) return false;
  if (ctx > old) {
    uint64_t d = ctx - old;
    __atomic_fetch_add(&g_region->dev_used[dev], d, __ATOMIC_RELAXED);
    uint64_t t = __atomic_add_fetch(&m->total, d, __ATOMIC_RELAXED);
    uint64_t pk = __atomic_load_n(&m->peak, __ATOMIC_RELAXED);
    while (t > pk && !__atomic_compare_exchange_n(&m->peak, &pk, t, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
    return false;
  }
  uint64_t d = old - ctx;
  __atomic_fetch_sub(&g_region->dev_used[dev], d, __ATOMIC_RELAXED);
  __atomic_fetch_sub(&m->total, d, __ATOMIC_RELAXED);
  return true;
}

// Reserve `bytes` on `dev` against the quota before calling the real
// allocator.  Returns false if the slice is exhausted.
bool reserve(int dev, uint64_t bytes, AllocKind kind) {
  uint64_t lim = limit_of(dev);
  if (!g_region) return true;
  refresh_context(dev, false);
  if (lim == 0) {
    account_add(dev, bytes, kind);
    return true;
  }
  // Over its grant by host truth (the monitor's verdict, control file): no
  // allocation at all until a pass finds it back under, whatever the counters
  // in the (tenant-writable) region say.
  if (ctl_over()) {
    tmark("mivgpu:oom-over-grant dev=%d req_mib=%llu", dev, (unsigned long long)(bytes >> 20));
    mlog(1, "device %d: allocation of %llu MiB refused: the container is over its HBM grant (host truth)", dev,
         (unsigned long long)(bytes >> 20));
    return false;
  }
  // VRAM the host sees the container hold beyond this counter (the monitor's
  // KFD truth, control file): a zeroed or stale counter cannot buy headroom
  const uint64_t excess = ctl_excess(dev);
  for (int attempt = 0; attempt < 2; ++attempt) {
    uint64_t cur = __atomic_load_n(&g_region->dev_used[dev], __ATOMIC_RELAXED);
    while (cur + excess + bytes <= lim) {
      if (__atomic_compare_exchange_n(&g_region->dev_used[dev], &cur, cur + bytes, true,
                                      __ATOMIC_ACQ_REL, __ATOMIC_RELAXED)) {
        // dev_used already bumped by the CAS; mirror into the process slot.
        account_slot_add(dev, bytes, kind);
        return true;
      }
    }
    if (attempt == 0) {  // a dead process may still hold quota, or our context charge be stale
      lock_region();
      int n = reclaim_dead_locked();
      unlock_region();
      bool shrank = refresh_context(dev, true);
      if (n == 0 && !shrank) break;
    }
  }
  tmark("mivgpu:oom dev=%d req_mib=%llu used_mib=%llu limit_mib=%llu", dev, (unsigned long long)(bytes >> 20),
        (unsigned long long)(__atomic_load_n(&g_region->dev_used[dev], __ATOMIC_RELAXED) >> 20),
        (unsigned long long)(lim >> 20));
  mlog(1, "device %d: allocation of %llu MiB exceeds the slice (%llu / %llu MiB in use)", dev,
       (unsigned long long)(bytes >> 20),
       (unsigned long long)(__atomic_load_n(&g_region->dev_used[dev], __ATOMIC_RELAXED) >> 20),
       (unsigned long long)(lim >> 20));
  return false;
}

void track(void* p, uint64_t size, int dev, AllocKind kind) {
  uintptr_t k = reinterpret_cast<uintptr_t>(p);
  Shard& s = shard_of(k);
  std::lock_guard<std::mutex> lk(s.mu);
  s.map[k] = AllocRec{size, (int16_t)dev, (uint8_t)kind};
}

bool untrack(uintptr_t k, AllocRec* out) {
  Shard& s = shard_of(k);
  std::lock_guard<std::mutex> lk(s.mu);
  auto it = s.map.find(k);
  if (it == s.map.end()) return false;
  *out = it->second;
  s.map.erase(it);
  return true;
}

bool lookup(uintptr_t k, AllocRec* out) {
  Shard& s = shard_of(k);
  std::lock_guard<std::mutex> lk(s.mu);
  auto it = s.map.find(k);
  if (it == s.map.end()) return false;
  *out = it->second;
  return true;
}

// Common body for the hipMalloc family.
template <typename Call>
hipError_t guarded_alloc(void** ptr, uint64_t bytes, Call&& call) {
  ensure_init();
  Guard g;
  if (!g.outer || bytes == 0) return call();
  int dev = current_device();
  if (!reserve(dev, bytes, K_BUFFER)) {
    if (ptr) *ptr = nullptr;
    if (g_cfg.oversubscribe && real_hipHostMalloc()) {
      // Host spill: device-visible pinned host memory stands in for HBM beyond
      // the slice (the AMD reading of HAMi's CUDA_OVERSUBSCRIBE).
      void* h = nullptr;
      if (real_hipHostMalloc()(&h, bytes, hipHostMallocMapped) == hipSuccess) {
        void* dptr = h;
        // mapped host memory is addressable by its host pointer if this fails
        if (real_hipHostGetDevicePointer()) (void)real_hipHostGetDevicePointer()(&dptr, h, 0);
        *ptr = dptr;
        track(dptr, bytes, dev, K_HOST_SPILL);
        tmark("mivgpu:host-spill dev=%d mib=%llu", dev, (unsigned long long)(bytes >> 20));
        return hipSuccess;
      }
    }
    return hipErrorOutOfMemory;
  }
  hipError_t rc = call();
  if (rc != hipSuccess || !ptr || !*ptr) {
    account_sub(dev, bytes, K_BUFFER);
    return rc;
  }
  track(*ptr, bytes, dev, K_BUFFER);
  return rc;
}

// Returns true if `p` was a host-spill allocation (already released).
bool release_tracked(void* p) {
  AllocRec r;
  if (!p || !untrack(reinterpret_cast<uintptr_t>(p), &r)) return false;
  if (r.kind == K_HOST_SPILL) {
    if (real_hipHostFree() && real_hipHostFree()(p) != hipSuccess) mlog(1, "host-spill free of %p failed", p);
    return true;
  }
  account_sub(r.dev, r.size, (AllocKind)r.kind);
  return false;
}

// ------------------------------------------------- arrays (texture memory) --
// hipArray allocations have opaque handles and a driver-chosen layout: the
// quota is charged an estimate (rows padded to 256 B, the gfx9 image pitch
// alignment), keyed by the handle and released by the matching free.
constexpr uint64_t kRowAlign = 256;

uint64_t channel_bytes(const hipChannelFormatDesc* d) {
  if (!d) return 4;
  const int bits = d->x + d->y + d->z + d->w;
  return bits > 0 ? (uint64_t)(bits + 7) / 8 : 4;
}

uint64_t format_bytes(hipArray_Format f, unsigned int channels) {
  uint64_t e = 4;
  switch (f) {
    case HIP_AD_FORMAT_UNSIGNED_INT8: case HIP_AD_FORMAT_SIGNED_INT8: e = 1; break;
    case HIP_AD_FORMAT_UNSIGNED_INT16: case HIP_AD_FORMAT_SIGNED_INT16: case HIP_AD_FORMAT_HALF: e = 2; break;
    default: e = 4; break;
  }
  return e * (channels ? channels : 1);
}

uint64_t array_bytes(uint64_t elem, uint64_t w, uint64_t h, uint64_t d) {
  const uint64_t row = ((w ? w : 1) * elem + kRowAlign - 1) & ~(kRowAlign - 1);
  return row * (h ? h : 1) * (d ? d : 1);
}

uint64_t mip_bytes(uint64_t elem, uint64_t w, uint64_t h, uint64_t d, unsigned int levels) {
  uint64_t sum = 0;
  for (unsigned int l = 0; l < (levels ? levels : 1) && l < 32; ++l) {
    sum += array_bytes(elem, w, h, d);
    w = w > 1 ? w >> 1 : 1;
    h = h > 1 ? h >> 1 : (h ? 1 : 0);
    d = d > 1 ? d >> 1 : (d ? 1 : 0);
  }
  return sum;
}

// Reserve-call-track for a handle-returning allocator: OOM past the slice.
template <typename Call>
hipError_t guarded_handle_alloc(void** handle, uint64_t bytes, Call&& call) {
  ensure_init();
  Guard g;
  if (!g.outer || bytes == 0) return call();
  const int dev = current_device();
  if (!reserve(dev, bytes, K_BUFFER)) return hipErrorOutOfMemory;
  hipError_t rc = call();
  if (rc != hipSuccess || !handle || !*handle) {
    account_sub(dev, bytes, K_BUFFER);
    return rc;
  }
  track(*handle, bytes, dev, K_BUFFER);
  return rc;
}

// ----------------------------------------------------------- code objects --
// Modules loaded through hipModuleLoad* are charged as `module` bytes (the
// reference's per-process moduleSize, pkg/monitor/nvidia/v1/spec.go:120-126):
// the load span of the gfx950 code object -- an ELF image, or the gfx950
// entry of a clang offload bundle -- rounded to 4 KiB.  A module load past the
// slice fails like an allocation.
uint64_t elf_span(const unsigned char* p, uint64_t avail) {
  if (avail < sizeof(Elf64_Ehdr) || memcmp(p, ELFMAG, SELFMAG) != 0 || p[EI_CLASS] != ELFCLASS64) return 0;
  Elf64_Ehdr eh;
  memcpy(&eh, p, sizeof(eh));
  if (eh.e_phentsize != sizeof(Elf64_Phdr) || eh.e_phnum == 0 || eh.e_phnum > 256) return 0;
  if (eh.e_phoff + (uint64_t)eh.e_phnum * sizeof(Elf64_Phdr) > avail) return 0;
  uint64_t lo = ~0ull, hi = 0;
  for (int i = 0; i < eh.e_phnum; ++i) {
    Elf64_Phdr ph;
    memcpy(&ph, p + eh.e_phoff + (uint64_t)i * sizeof(Elf64_Phdr), sizeof(ph));
    if (ph.p_type != PT_LOAD || ph.p_memsz == 0) continue;
    if (ph.p_vaddr < lo) lo = ph.p_vaddr;
    if (ph.p_vaddr + ph.p_memsz > hi) hi = ph.p_vaddr + ph.p_memsz;
  }
  if (hi <= lo) return 0;
  return (hi - lo + 4095) & ~4095ull;
}

// `avail` bounds the reads (SIZE_MAX for an in-memory image of unknown size:
// the headers then say how far to read).
uint64_t code_object_bytes(const void* image, uint64_t avail) {
  if (!image) return 0;
  const unsigned char* p = static_cast<const unsigned char*>(image);
  static const char kBundle[] = "__CLANG_OFFLOAD_BUNDLE__";
  if (avail >= 4 && memcmp(p, ELFMAG, SELFMAG) == 0) return elf_span(p, avail);
  if (avail < 32 || memcmp(p, kBundle, 24) != 0) return 0;
  uint64_t n = 0, off = 32, pick_off = 0, pick_size = 0;
  memcpy(&n, p + 24, 8);
  bool exact = false;
  for (uint64_t i = 0; i < n && i < 64 && off + 24 <= avail; ++i) {
    uint64_t eo, es, il;
    memcpy(&eo, p + off, 8);
    memcpy(&es, p + off + 8, 8);
    memcpy(&il, p + off + 16, 8);
    if (il > 256 || off + 24 + il > avail) break;
    char id[260];
    memcpy(id, p + off + 24, il);
    id[il] = 0;
    off += 24 + il;
    if (!strstr(id, "amdgcn") || es == 0) continue;
    const bool match = strstr(id, "gfx950") != nullptr;
    if (match || (!exact && !pick_size)) {
      pick_off = eo;
      pick_size = es;
      exact = match;
    }
  }
  if (!pick_size || pick_off + pick_size > avail) return 0;
  return elf_span(p + pick_off, pick_size);
}

uint64_t code_object_file_bytes(const char* path) {
  if (!path) return 0;
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return 0;
  struct stat st;
  uint64_t n = 0;
  if (mivgpu_fstat(fd, &st) == 0 && st.st_size > 0) {
    void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m != MAP_FAILED) {
      n = code_object_bytes(m, (uint64_t)st.st_size);
      munmap(m, (size_t)st.st_size);
    }
  }
  close(fd);
  return n;
}

template <typename Call>
hipError_t guarded_module_load(hipModule_t* module, uint64_t bytes, Call&& call) {
  ensure_init();
  Guard g;
  if (!g.outer || bytes == 0) return call();
  const int dev = current_device();
  if (!reserve(dev, bytes, K_MODULE)) return hipErrorOutOfMemory;
  hipError_t rc = call();
  if (rc != hipSuccess || !module || !*module) {
    account_sub(dev, bytes, K_MODULE);
    return rc;
  }
  track(reinterpret_cast<void*>(*module), bytes, dev, K_MODULE);
  refresh_context(dev, true);   // the runtime's own share of the load moves out of `context`
  return rc;
}

// ------------------------------------------------------- launch-side state --
std::atomic<uint64_t> g_launches_local{0};
// Launches per device (device 0 for the common one-device container: no
// runtime call on the launch path), published by the housekeeping thread.
std::atomic<uint64_t> g_dev_launches[MIVGPU_MAX_DEVICES];

// Governor (gate) per device.  Host stats = 8 counters + a 128-entry trace
// ring of 8 x int64 per gate + 64 per-slot hold ends, hold starts and held
// totals (layout: governor.hip mivgpu_gate_host_stats; counter 6 is the
// sampler's measured share).
constexpr size_t kHostStatsBytes = 64 + 128 * 64 + 3 * 64 * 8;
constexpr int kHsSharePpm = 6;          // u64 index of share_ppm (sampler -> gate)
constexpr int kHsHostTokens = 7;        // u64 index of host_tokens_ns (sampler -> gate, host-bucket mode)
constexpr int kHsHoldEnd = 8 + 128 * 8; // u64 index of hold_end_ns[0]
constexpr int kHsHoldStart = kHsHoldEnd + 64;
constexpr int kHsHeldCum = kHsHoldEnd + 128;
// Written under G.mu; the launch fast path (maybe_gate) reads them lock-free.
struct GateSlot {
  std::atomic<hipStream_t> stream;
  std::atomic<uint64_t> last_gate_host_ns;
  std::atomic<uint64_t> first_submit_host_ns;   // first launch since the last gate (0 = none pending)
  std::atomic<bool> used;
  // most recent launch on this stream, and the host threads inside a launch
  // call on it: raised under G.mu, lowered lock-free when the call returns
  // (LaunchScope), so a governed launch takes the mutex once
  std::atomic<uint64_t> last_launch_host_ns;
  std::atomic<int> batch_launches; // launches since the last gate
  std::atomic<int> in_launch;
};
struct DeviceGate {
  std::mutex mu;
  bool tried = false;
  bool ok = false;
  std::atomic<bool> ok_pub{false};    // `ok`, for the lock-free launch fast path
  hipModule_t module = nullptr;
  hipFunction_t gate_fn = nullptr;
  hipFunction_t clock_fn = nullptr;
  void* state = nullptr;        // device memory
  void* host_stats = nullptr;   // fine-grained host memory
  long long* clock_host = nullptr;
  int64_t offset_ns = 0;        // device_ns - host_mono_ns
  bool stamper_started = false;
  std::atomic<void*> hs_pub{nullptr};  // host_stats, published for the sampler thread
  std::atomic<uint64_t> enqueued{0};   // gates enqueued; host_stats[2] counts the ones that ran
  GateSlot slots[64];
};
DeviceGate g_gates[MIVGPU_MAX_DEVICES];

}  // namespace

// The embedded gfx950 code object for governor.hip (generated at build time).
#include "governor_hsaco.inc"

namespace {

// Makes `dev` current for the scope (the gate's code object, state and clock
// calibration belong to the device the gate will run on, which for a
// multi-device launch is not the calling thread's current device).
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    if (real_hipGetDevice() && real_hipSetDevice() && real_hipGetDevice()(&prev) == hipSuccess && prev != dev)
      (void)real_hipSetDevice()(dev);
    else
      prev = -1;
  }
  ~DeviceScope() {
    if (prev >= 0) (void)real_hipSetDevice()(prev);
  }
};

bool gate_init_locked(int dev, DeviceGate& G) {
  G.tried = true;
  TRange r("mivgpu:governor-init");
  DeviceScope scope(dev);
  if (!real_hipModuleLoadData() || !real_hipModuleGetFunction() || !real_hipModuleLaunchKernel())
    return false;
  if (real_hipModuleLoadData()(&G.module, mivgpu_governor_hsaco) != hipSuccess) {
    mlog(1, "device %d: governor code object failed to load; temporal throttling off", dev);
    return false;
  }
  if (real_hipModuleGetFunction()(&G.gate_fn, G.module, "mivgpu_gate") != hipSuccess ||
      real_hipModuleGetFunction()(&G.clock_fn, G.module, "mivgpu_clock") != hipSuccess)
    return false;
  // State lives in device memory; it is not charged to the tenant's quota.
  if (real_hipMalloc()(&G.state, 4096) != hipSuccess) return false;
  if (!real_hipMemset() || real_hipMemset()(G.state, 0, 4096) != hipSuccess) return false;
  if (real_hipHostMalloc()(&G.host_stats, kHostStatsBytes, hipHostMallocCoherent | hipHostMallocMapped) !=
      hipSuccess)
    G.host_stats = nullptr;
  if (G.host_stats) memset(G.host_stats, 0, kHostStatsBytes);
  if (real_hipHostMalloc()((void**)&G.clock_host, 64, hipHostMallocCoherent | hipHostMallocMapped) !=
      hipSuccess)
    return false;
  // Calibrate device realtime vs host CLOCK_MONOTONIC on the null stream.
  int64_t best = 0;
  uint64_t best_span = ~0ull;
  for (int i = 0; i < 5; ++i) {
    *G.clock_host = 0;
    void* args[] = {&G.clock_host};
    uint64_t t0 = mono_ns();
    if (real_hipModuleLaunchKernel()(G.clock_fn, 1, 1, 1, 64, 1, 1, 0, nullptr, args, nullptr) !=
        hipSuccess)
      return false;
    if (real_hipStreamSynchronize()(nullptr) != hipSuccess) return false;
    uint64_t t1 = mono_ns();
    if (t1 - t0 < best_span && *G.clock_host) {
      best_span = t1 - t0;
      best = (int64_t)*G.clock_host - (int64_t)((t0 + t1) / 2);
    }
  }
  G.offset_ns = best;
  G.hs_pub.store(G.host_stats, std::memory_order_release);
  mlog(3, "device %d: governor ready (clock offset %lld ns, calibration span %llu ns)", dev,
       (long long)best, (unsigned long long)best_span);
  return true;
}

// ------------------------------------------------- wave-occupancy sampler --
// The share of the GPU a tenant receives is measured, not inferred: KFD
// publishes every process's resident wavefronts per GPU
// (<kfd>/proc/<pid>/stats_<gpu_id>/cu_occupancy: SPI_CSQ_WF_ACTIVE_COUNT of
// its queues in CU units; ~7 us per read on MI355X, profiles/governor_occupancy).
// A sampler thread reads this process's count and every other process's count
// on the same GPU; per sample
//     share = own / (own + others)
// capped at the CU-mask fraction for a spatially masked tenant (it cannot hold
// more of the GPU than its CUs).  Two products:
//   * share_ppm -- the share averaged (EWMA, ~20 ms) over the samples in which
//     the process was contending (waves resident, or a launch within the last
//     5 ms while others ran).  The gate kernel weights a stream's busy wall
//     time by it (governor.hip): alone -> wall time; N tenants time-sliced by
//     the hardware scheduler or co-resident -> ~1/N each; idle neighbours ->
//     no dilution.
//   * share_ns -- the plain time integral of the share (0 while no waves are
//     resident): GPU time received, whose rate over the last window is the
//     utilisation the monitor exports (util_pct; the reference's per-process
//     SM utilisation, pkg/monitor/nvidia/v1/spec.go:164).
struct OccPeer {
  int pid;
  int fd;
  uint64_t busy_ns;   // last sample that saw waves of it resident (beyond a gate wave)
  int v;              // its reading this sample
  double avg;         // EWMA of its readings over this process's owing samples
};
// Busy peers whose average resident waves are within this factor of this
// process's own (either way) contend as equals; a peer this many times
// lighter is ignored, one this many times heavier is shared with by ratio.
constexpr double kContendFrac = 0.1;
// Local estimate (no live share board): a peer is busy for this long after
// its last sample with waves resident.
constexpr uint64_t kPeerBusyNs = 200000000ull;   // 200 ms
// A board whose owner has not completed a pass for this long is not used.
constexpr uint64_t kBoardStaleNs = 50000000ull;   // 50 ms
// Idle time after which the host bucket stops accruing entitlement.
constexpr uint64_t kAccrueIdleNs = 20000000ull;   // 20 ms
// Fair-share mode (board.h): lead over the backlogged tenants' mean at which
// the gate holds (GPU time beyond the weighted fair share).  Per decode step
// a tenant's wave-share estimate scatters by ~0.7 ms at eight tenants; a
// 5 ms lag held symmetric tenants 20-40 % of their samples on noise.
constexpr uint64_t kFairLagNs = 10000000ull;       // 10 ms
// A governed peer held behind its gate has exactly its gate kernel's wave
// resident (governor.hip host_bucket_gate: one 64-lane wave).
constexpr int kGateWaves = 1;
struct OccDev {
  bool live = false;           // sampler has this device's KFD view
  int gpu_id = -1;
  int own_fd = -1;
  int own_pid = -1;
  std::vector<OccPeer> peers;
  uint64_t list_ns = 0;        // last peer directory scan
  uint64_t last_ns = 0;        // last sample
  double share_ns = 0;         // integral of the share, GPU-ns
  double share_avg = -1;       // the share while owing work (-1 = no sample yet)
  double own_avg = 0;          // EWMAs of own / other tenants' resident waves while owing work
  double others_avg = 0;
  double inst_avg = -1;        // MIVGPU_SHARE_EST=instant: EWMA of the per-sample ratio
  uint64_t win_start_ns = 0;   // utilisation window
  double win_start_share = 0;
  bool bucket = false;         // host bucket started (the device's gate is up)
  double tokens_ns = 0;        // host bucket balance: rate x wall time - GPU time received
  uint64_t owed_ns = 0;        // last sample in which the process owed GPU work
  uint64_t window_ns = 0;      // this sample's contention window (0: per sample)
  uint64_t batch_win_ns = 0;   // batch-size estimate window (host mode)
  uint64_t batch_win_launches = 0;
  double batch_win_share = 0;
  double ns_per_launch = 0;    // GPU time received per launch (EWMA)
  // wall time by sampler state (mivgpu_occ_states): own waves resident,
  // alone + busy with none resident, held by its gate, others only, idle
  double state_ns[5] = {0, 0, 0, 0, 0};
  uint64_t samples = 0;
  // exact held time (host mode): each slot's held total incl. a hold in
  // progress at the previous sample, and the held time counted late (a hold
  // published after its interval) carried into the next interval
  int64_t held_prev[64] = {};
  double held_carry = 0;
  // share board (board.h): the GPU's one sampler
  mivgpu_board::Handle board;
  uint64_t board_open_ns = 0;  // last attempt to map it
  uint64_t board_try_ns = 0;   // last attempt to take the owner role
  uint64_t board_flags_ns = 0; // last attempt to map the flags file
  uint64_t board_wave_ns = 0;  // owner: last pass with any process's waves resident
  int board_hint = -1;
  bool board_prev_ok = false;
  uint64_t board_prev_obs = 0, board_prev_frac = 0;
  double board_share = -1;     // the board's mean share over the latest observed interval
  mivgpu_board::View board_view;
  uint64_t board_charged = 0;  // samples charged from the board / from the local estimate
  uint64_t local_charged = 0;
  uint64_t fair_samples = 0;   // samples in fair-share mode / held there on the lead
  uint64_t fair_held_samples = 0;
  // the samples outside the fair-share mode, last 16 (sampler_info "nonfair"):
  // interval, share charged, run time, bucket after, previous sample in the mode
  struct NonFair {
    uint64_t t_ns, dt_ns;
    double share, run_ns, tokens_ns;
    int prev_fair;
  } nonfair[16];
  uint64_t nonfair_n = 0;
  int64_t last_lead_ns = -1;
  double fair_recv_ns = 0;     // GPU time received since fair-share mode began
  std::vector<mivgpu_board::Reading> readings;
};
// Background stamper idle threshold and the batch bounds (see stamper_main
// and maybe_gate below).
constexpr uint64_t kStampIdleNs = 1000000;  // 1 ms
constexpr int kMaxBatchLaunches = 256;
// Host mode: launches per batch sized by the sampler to ~2 ms of GPU time.
std::atomic<int> g_batch_max[MIVGPU_MAX_DEVICES];

// Heap-allocated and never freed: the sampler thread is detached, and a
// static array's destructor at exit would free the peer vectors under it.
OccDev* const g_occ = new OccDev[MIVGPU_MAX_DEVICES];
std::mutex& g_occ_pass_mu = *new std::mutex;   // held for one sampling pass; exit waits on it (never destroyed)
std::atomic<bool> g_occ_started{false};
std::atomic<bool> g_occ_live[MIVGPU_MAX_DEVICES];
std::atomic<uint64_t> g_last_gate_ns[MIVGPU_MAX_DEVICES];   // coarse clock of the latest gate
std::atomic<uint64_t> g_last_launch_ns{0};                   // coarse clock of the latest launch

int read_occ(int fd) {
  char buf[32];
  ssize_t n = pread(fd, buf, sizeof(buf) - 1, 0);
  if (n <= 0) return -1;
  buf[n] = 0;
  return atoi(buf);
}

int open_occ(int pid, int gpu_id) {
  char path[512];
  snprintf(path, sizeof(path), "%s/proc/%d/stats_%d/cu_occupancy", g_cfg.kfd_sysfs, pid, gpu_id);
  return open(path, O_RDONLY | O_CLOEXEC);
}

// Re-list the KFD processes on this GPU (every 100 ms): tenants come and go.
void occ_rescan(OccDev& o, uint64_t now) {
  o.list_ns = now;
  char dir[512];
  snprintf(dir, sizeof(dir), "%s/proc", g_cfg.kfd_sysfs);
  DIR* d = opendir(dir);
  if (!d) return;
  std::vector<OccPeer> next;
  while (struct dirent* e = readdir(d)) {
    char* end = nullptr;
    long pid = strtol(e->d_name, &end, 10);
    if (end == e->d_name || *end || pid <= 0 || pid == o.own_pid) continue;
    int fd = -1;
    uint64_t busy = 0;
    double avg = 0;
    for (auto& p : o.peers)
      if (p.pid == pid && p.fd >= 0) { fd = p.fd; busy = p.busy_ns; avg = p.avg; p.fd = -1; break; }
    if (fd < 0) fd = open_occ((int)pid, o.gpu_id);   // no stats_<gpu_id>: not on this GPU
    if (fd >= 0) next.push_back(OccPeer{(int)pid, fd, busy, 0, avg});
  }
  closedir(d);
  for (auto& p : o.peers)
    if (p.fd >= 0) close(p.fd);
  o.peers.swap(next);
}

std::atomic<bool> g_board_fast{false};   // an owner pass saw waves or a governed tenant asked within 1 s

// The share board of the sampler's GPU: map it (retried every second), hold
// or give up the owner role, run the owner pass over this sample's readings
// (this process and every peer on the GPU), then read this process's slot.
// Returns the mean share over the passes since the previous sample in which
// this process was not held, or -1 when no live board covers it.
double board_step(OccDev& o, uint64_t now, int own_raw, bool gating, int flags, uint32_t limit_ppm) {
  namespace mb = mivgpu_board;
  if (!g_cfg.board_dir[0]) return -1;
  if (!o.board.b) {
    if (o.board_open_ns && now - o.board_open_ns < 1000000000ull) return -1;
    o.board_open_ns = now;
    if (!mb::open_board(o.board, g_cfg.board_dir, o.gpu_id, true)) return -1;
    snprintf(o.board.flags_dir, sizeof(o.board.flags_dir), "%s", g_cfg.board_flags_dir);
    o.board.presence_ns = g_cfg.presence_ns;
    mlog(3, "KFD gpu %d: share board %s/gpu-%d.board mapped %s", o.gpu_id, g_cfg.board_dir, o.gpu_id,
         o.board.writable ? "read-write" : "read-only");
  }
  if (!o.board.flags && now - o.board_flags_ns >= 1000000000ull) {
    o.board_flags_ns = now;
    if (!mb::open_flags(o.board)) mlog(3, "KFD gpu %d: board flags not writable; the owner reads occupancy only", o.gpu_id);
  }
  mb::publish_flags(o.board, o.own_pid, flags, limit_ppm, now);
  mivgpu_board_t* b = o.board.b;
  const int self = o.own_pid;
  if (o.board.owner) {
    if (mb::node_owner_live(b, self, now)) {
      mb::release_own(o.board);
      mlog(3, "KFD gpu %d: node sampler live, share board owner role released", o.gpu_id);
    }
  } else if (o.board.writable && gating && now - o.board_try_ns >= 50000000ull) {
    o.board_try_ns = now;
    if (mb::try_own(o.board, self, now)) mlog(3, "KFD gpu %d: share board owner (pid %d)", o.gpu_id, self);
  }
  if (o.board.owner) {
    o.readings.clear();
    o.readings.push_back(mb::Reading{self, own_raw});
    for (const auto& p : o.peers) o.readings.push_back(mb::Reading{p.pid, p.v});
    for (const auto& r : o.readings)
      if (r.v > mb::kGateUnits) o.board_wave_ns = now;
    const bool fast = now - o.board_wave_ns < 1000000000ull ||
                      __atomic_load_n(&b->want_fast_ns, __ATOMIC_RELAXED) + 1000000000ull > now;
    g_board_fast.store(fast, std::memory_order_relaxed);
    mb::owner_pass(o.board, o.readings.data(), (int)o.readings.size(), now,
                   fast ? g_cfg.occ_period_ns : g_cfg.occ_idle_period_ns, MIVGPU_BOARD_OWNER_SHIM, self,
                   g_cfg.board_split, mono_ns() - now);
  } else if (o.board.writable && gating) {
    __atomic_store_n(&b->want_fast_ns, now, __ATOMIC_RELAXED);
  }
  mb::View v;
  // stale: older than 50 ms, or than three of the owner's own passes (a node
  // sampler with no governed tenant runs dormant, 50 ms apart)
  const bool got = mb::read_slot(b, self, &o.board_hint, &v);
  const uint64_t stale_ns = v.period_ns && 3 * v.period_ns > kBoardStaleNs ? 3 * v.period_ns : kBoardStaleNs;
  if (!got || v.beat_ns + stale_ns < now) {
    o.board_prev_ok = false;
    o.board_view.lead_ns = -1;
    return -1;
  }
  if (o.board_prev_ok && v.obs_ns >= o.board_prev_obs && v.frac_ns >= o.board_prev_frac) {
    const uint64_t dobs = v.obs_ns - o.board_prev_obs;
    if (dobs > 0) {
      const double f = (double)(v.frac_ns - o.board_prev_frac) / (double)dobs;
      o.board_share = f > 1.0 ? 1.0 : f;
    }
  }
  o.board_prev_ok = true;
  o.board_prev_obs = v.obs_ns;
  o.board_prev_frac = v.frac_ns;
  o.board_view = v;
  return o.board_share;
}

// One sample of device `dev`.  Returns false if the device has no KFD view.
bool occ_sample(int dev, uint64_t now) {
  OccDev& o = g_occ[dev];
  if (!o.live) {
    int gid = -1, pid = -1;
    {
      std::lock_guard<std::mutex> lk(g_ctx_mu);
      if (!kfd_identity_locked(dev, &gid, &pid, false)) return false;
    }
    o.gpu_id = gid;
    o.own_pid = pid;
    o.own_fd = open_occ(pid, gid);
    if (o.own_fd < 0) return false;
    o.live = true;
    o.last_ns = o.win_start_ns = now;
    occ_rescan(o, now);
    g_occ_live[dev].store(true, std::memory_order_release);
    mlog(3, "device %d: occupancy sampler on (KFD gpu_id %d, pid %d, %zu peers)", dev, gid, pid, o.peers.size());
  }
  if (now - o.list_ns > 100000000ull) occ_rescan(o, now);
  int own = read_occ(o.own_fd);
  if (own < 0) own = 0;
  // Other tenants' waves, counted like this process's own (a held peer's gate
  // wave among them: discounting one CU's worth for peers but not for itself
  // billed every symmetric tenant above 1/N -- measured, 8 x 12 % decode
  // tenants held 27 % of the time).
  // Local estimate (used only while no share board is live, board.h): a peer
  // contends while it showed more than a gate's wave within the last 200 ms
  // (the round-3 rule; MIVGPU_PEER_BUSY_MS sets another window).  Per-sample
  // decisions made by each tenant on its own clock charged four symmetric
  // 25 % tenants 100 / 33 / 100 / 100 % of their busy time: a
  // time-sliced busy peer often shows no waves in a given sample.
  const uint64_t window = g_cfg.peer_busy_ns ? g_cfg.peer_busy_ns : kPeerBusyNs;
  long others = 0;
  int busy_peers = 0;
  // With a live board only its owner reads the peers: every cu_occupancy read
  // walks the waves of all eight XCDs in the driver, and eight tenants each
  // reading all nine processes every 2 ms stretched their sampler passes to
  // ~5.5 ms (flags going stale, the subscription test failing half the time).
  const bool read_peers = o.board.owner || !o.board_prev_ok;
  for (auto& p : o.peers) {
    if (!read_peers) {
      p.v = 0;
      continue;
    }
    int v = read_occ(p.fd);
    p.v = v > 0 ? v : 0;
    if (v > 0) others += v;
    if (v > kGateWaves) p.busy_ns = now;
    if (p.busy_ns && now - p.busy_ns < window) ++busy_peers;
  }
  o.window_ns = window;
  const int own_raw = own;
  // The gate's own resident wave is not consumption: discount one unit per
  // gate slot holding right now.
  DeviceGate& G = g_gates[dev];
  const uint64_t* hs = static_cast<const uint64_t*>(G.hs_pub.load(std::memory_order_acquire));
  int holding = 0;
  int64_t held_dt = 0;   // time the process sat in its gates since the previous sample (longest slot)
  if (hs) {
    const int64_t now_dev = (int64_t)mono_ns() + G.offset_ns;
    const int64_t* hi = reinterpret_cast<const int64_t*>(hs);
    for (int i = 0; i < 64; ++i) {
      // total first, then end, then start (governor.hip host_bucket_gate
      // writes them in the opposite orders)
      int64_t f = __atomic_load_n(&hi[kHsHeldCum + i], __ATOMIC_ACQUIRE);
      const int64_t end = __atomic_load_n(&hi[kHsHoldEnd + i], __ATOMIC_ACQUIRE);
      if (end > now_dev) {
        ++holding;
        const int64_t start = __atomic_load_n(&hi[kHsHoldStart + i], __ATOMIC_RELAXED);
        if (start > 0 && start < now_dev) f += now_dev - start;
      }
      if (f != o.held_prev[i]) {
        if (o.bucket && f - o.held_prev[i] > held_dt) held_dt = f - o.held_prev[i];
        o.held_prev[i] = f;
      }
    }
    own = own > holding ? own - holding : 0;
  }
  // Busy: the streams still owe GPU work -- a gate enqueued that has not run
  // (every batch is closed by the next launch's gate or the idle stamper),
  // or a launch within the stamper's idle window.
  bool pending = false;
  const uint64_t since_launch = coarse_ns() - g_last_launch_ns.load(std::memory_order_relaxed);
  if (hs) {
    const uint64_t done = __atomic_load_n(&hs[2], __ATOMIC_RELAXED);
    pending = G.enqueued.load(std::memory_order_acquire) > done || since_launch < 2 * kStampIdleNs;
  } else {
    pending = since_launch < 5000000ull;
  }
  uint64_t dt = now - o.last_ns;
  if (dt > 100000000ull) dt = 100000000ull;   // a stalled sampler does not invent history
  o.last_ns = now;
  // While the process owes work (waves resident, a batch queued or running,
  // or held in the interval) it is charged an equal split of that time with
  // the other tenants contending for the GPU as equals: busy ones (waves seen
  // within 200 ms) whose average resident waves -- averaged over the samples
  // in which this process owes work and is not held -- are within 10x of its
  // own.  A tenant that occupies the GPU far less (a light neighbour's small
  // kernels, a peer held behind its gate) does not dilute the charge, so alone
  // or next to light tenants the process pays its whole busy time (dispatch
  // gaps included); N symmetric busy tenants pay 1/N each; next to a tenant
  // 10x heavier it pays its ratio of the waves (queued behind it with none of
  // its own resident: nothing).  Measured on
  // MI355X, magnitudes read by each tenant's own sampler are not comparable
  // across tenants: a decode step is hundreds of short kernels, the hardware
  // scheduler time-slices processes' queues, and the sampler thread runs when
  // its process lets it -- the ratio of averaged wave counts put 8 symmetric
  // 12 % tenants at 3-55 % each (fairness 0.91), per-sample ratios at 2-80 %
  // (0.81).  The count needs only "is it busy, and not much lighter".  The
  // time held by its gates is known exactly and charged nothing.
  // the GPU's share board: publish this pass's state (held / owing), run the
  // owner pass if this process holds the role, read this process's share
  const bool gating = coarse_ns() - g_last_gate_ns[dev].load(std::memory_order_relaxed) < 1000000000ull;
  // GATED: the node sampler runs its fast passes only while some tenant is
  // governed (a CU-masked tenant never gates: sampling for it is pure cost)
  const int flags = (holding > 0 ? MIVGPU_FLAG_HELD : 0) |
                    ((pending || own > 0) && holding == 0 ? MIVGPU_FLAG_OWES : 0) | (gating ? MIVGPU_FLAG_GATED : 0);
  const uint64_t lim_ppm = cu_limit_ppm_of(dev);
  const double board_f = board_step(o, now, own_raw, gating, flags,
                                    lim_ppm > 0 && lim_ppm < 1000000 ? (uint32_t)lim_ppm : 0u);
  // fair-share mode (board.h): the GPU is fully subscribed by backlogged
  // tenants; this process is held on its lead over the furthest-behind one
  const int64_t lead = board_f >= 0 ? o.board_view.lead_ns : -1;
  const bool owes = own > 0 || pending || holding > 0 || held_dt > 0;
  const double a = (double)dt / g_cfg.share_tau_ns < 1.0 ? (double)dt / g_cfg.share_tau_ns : 1.0;
  if (owes && holding == 0) {
    o.own_avg += a * ((double)own - o.own_avg);
    o.others_avg += a * ((double)others - o.others_avg);
    for (auto& p : o.peers) p.avg += a * ((double)p.v - p.avg);
  }
  if (g_cfg.share_instant && holding == 0 && (own > 0 || (others > 0 && pending))) {
    const double inst = (double)own / (double)(own + others);
    o.inst_avg = o.inst_avg < 0 ? inst : o.inst_avg + a * (inst - o.inst_avg);
  }
  double share = 0.0;
  int state = 4;
  if (owes) {
    if (board_f >= 0) {
      // the GPU's one sampler: this process's mean share of the resident
      // waves over the passes since the previous sample in which it was not
      // held, taken at the same instants as every other tenant's
      share = board_f;
      ++o.board_charged;
    } else if (g_cfg.share_ratio) {
      const double tot = o.own_avg + o.others_avg;
      share = tot > 0 ? o.own_avg / tot : 1.0 / (double)(1 + busy_peers);
    } else if (g_cfg.share_instant && o.inst_avg >= 0) {
      share = o.inst_avg;
    } else {
      int comparable = 0;
      double heavier = 0;
      for (const auto& p : o.peers) {
        if (!p.busy_ns || now - p.busy_ns >= o.window_ns) continue;
        if (p.avg * kContendFrac > o.own_avg) heavier += p.avg;
        else if (p.avg >= kContendFrac * o.own_avg) ++comparable;
      }
      const double base = o.own_avg + heavier > 0 ? o.own_avg / (o.own_avg + heavier) : 1.0;
      share = base / (double)(1 + comparable);
    }
    if (board_f < 0) ++o.local_charged;
    state = own > 0 ? 0 : (others > 0 ? 3 : 1);
  }
  const int mask = (int)cu_mask_of(dev);
  if (mask > 0) {
    const double f = (double)mask / (double)device_cus(dev);
    if (share > f) share = f;
  }
  double run = (double)dt - (double)held_dt + o.held_carry;
  o.held_carry = run < 0 ? run : 0;
  if (run < 0) run = 0;
  const double held = (double)dt - run;
  o.share_ns += share * run;
  o.state_ns[state] += run;
  o.state_ns[2] += held;
  ++o.samples;
  const uint64_t total = (uint64_t)o.share_ns;
  // Host bucket (governor.hip host_bucket_gate): entitlement accrues at the
  // core limit, the GPU time actually received (the share integral) is
  // charged, the balance is bounded by one burst either way.  The gates read
  // it at execution time and hold while it is negative.
  if (hs) {
    const uint64_t lim = cu_limit_ppm_of(dev);
    const double rate = (lim > 0 && lim < 1000000) ? (double)lim / 1e6 : 1.0;
    const double cap = (double)g_cfg.gate_cap_ns;
    if (!o.bucket) {
      // nearly empty, not full: a burst is earned by idling below the limit,
      // not granted at start (a 100 ms start burst put a 1.5 s job at 0.32 of
      // its unthrottled rate under a 25 % limit).  It starts with the
      // fair-share mode's lag (10 ms), as a tenant leaving the mode does:
      // eight pooled tenants whose governor the monitor's switch engaged all
      // at once each went a few ms into debt on the wave-share noise before
      // the mode took over and sat out a 25 ms hold (round 6)
      o.bucket = true;
      o.tokens_ns = (double)kFairLagNs;
    } else {
      // Entitlement accrues while the process owes work and through short
      // gaps (host syncs, batch edges), not over long idle stretches: a
      // torch.compile'd loop otherwise banked the whole 100 ms burst while
      // Inductor compiled on the CPU and spent it at the start of its timed
      // loop (0.311 of unthrottled under a 25 % limit)
      if (owes) o.owed_ns = now;
      const bool accrue = owes || (o.owed_ns && now - o.owed_ns < kAccrueIdleNs);
      o.tokens_ns += (accrue ? rate * (double)dt : 0.0) - share * run;
      if (o.tokens_ns > cap) o.tokens_ns = cap;
      if (o.tokens_ns < -cap) o.tokens_ns = -cap;
    }
    // Fully subscribed, every tenant's bucket is at equilibrium: what they are
    // charged sums to what they accrue, so holding one only moves its GPU time
    // to the others and a debt (one carried in from a phase alone, or noise)
    // is never repaid -- measured, four symmetric 25 % tenants held 0.4-1.1 s
    // each over a 1.6 s run, at 0.82 of native.  There the tenant is held on
    // its lead over the backlogged tenants' mean instead (the tenants behind
    // always run: work-conserving, shares by core limit) and its bucket
    // carries no debt and no burst out of the mode, only the mode's own lag
    // (a 25 % tenant left alone by a 75 % one that finished spent up to the
    // whole 100 ms burst it had banked while held on its lead: 27 % of the GPU).
    // The lag grows with the GPU time received in the mode: 3 % of it, at
    // least 10 ms.  The wave-share estimate is not exact per tenant (four
    // symmetric 25 % tenants: one was held 120 ms of a 100-step run on it and
    // came out slowest, fairness 0.93 where the hardware alone gave 0.995);
    // unequal limits drift by far more than 3 % and are still held.
    if (lead < 0) {
      OccDev::NonFair& nf = o.nonfair[o.nonfair_n++ % 16];
      nf = OccDev::NonFair{now, dt, share, run, o.tokens_ns, o.last_lead_ns >= 0 ? 1 : 0};
    }
    double eff = o.tokens_ns;
    if (lead >= 0) {
      // out of the mode with the mode's own slack (kFairLagNs), not empty:
      // eight pooled tenants pausing together (a batch edge) left the mode,
      // and coming back each started its bucket at zero, went a few ms into
      // debt before the mode re-engaged and sat out a 25 ms hold -- every
      // tenant, every time (5 % of a 20-step window, round 6)
      o.tokens_ns = (double)kFairLagNs;
      o.fair_recv_ns += share * run;
      const double rel = g_cfg.fair_lag_frac * o.fair_recv_ns;
      const double lag = rel > (double)kFairLagNs ? rel : (double)kFairLagNs;
      eff = lag - (double)lead;
      ++o.fair_samples;
      if (eff < 0) ++o.fair_held_samples;
    } else {
      o.fair_recv_ns = 0;
    }
    o.last_lead_ns = lead;
    __atomic_store_n(reinterpret_cast<int64_t*>(const_cast<uint64_t*>(&hs[kHsHostTokens])), (int64_t)eff,
                     __ATOMIC_RELAXED);
  }
  // Host mode: size the batches between gates to ~2 ms of GPU time from the
  // GPU time received per launch (a gate is a few us; a batch of 256 long
  // kernels -- a Triton GEMM loop -- was ~300 ms, far coarser than a 25 ms hold)
  if (hs && now - o.batch_win_ns >= 20000000ull) {
    const uint64_t l = g_launches_local.load(std::memory_order_relaxed);
    // only windows in which the process received GPU time: a window spent
    // held (launches queued, nothing received) read as ~0 ns per launch and
    // sized the next batches to the 256-launch maximum
    if (o.batch_win_ns && l > o.batch_win_launches && o.share_ns - o.batch_win_share > 1e6) {
      const double per = (o.share_ns - o.batch_win_share) / (double)(l - o.batch_win_launches);
      o.ns_per_launch = o.ns_per_launch <= 0 ? per : 0.7 * o.ns_per_launch + 0.3 * per;
      const double n = o.ns_per_launch > 0 ? 2e6 / o.ns_per_launch : (double)kMaxBatchLaunches;
      g_batch_max[dev].store(n < 1 ? 1 : (n > kMaxBatchLaunches ? kMaxBatchLaunches : (int)n),
                             std::memory_order_relaxed);
    }
    o.batch_win_ns = now;
    o.batch_win_launches = l;
    o.batch_win_share = o.share_ns;
  }
  // The reported share (and the device-bucket gate's weight): the share
  // while owing work, as charged.
  if (owes && holding == 0) {
    o.share_avg = share;
    uint64_t ppm = (uint64_t)(o.share_avg * 1e6 + 0.5);
    if (!ppm) ppm = 1;   // 0 means "no sample yet" to the gate
    if (hs) __atomic_store_n(const_cast<uint64_t*>(&hs[kHsSharePpm]), ppm, __ATOMIC_RELAXED);
    if (g_slot >= 0) __atomic_store_n(&g_region->procs[g_slot].util[dev].share_ppm, ppm, __ATOMIC_RELAXED);
  }
  if (g_slot >= 0) {
    mivgpu_util_t* u = &g_region->procs[g_slot].util[dev];
    __atomic_store_n(&u->share_ns, total, __ATOMIC_RELAXED);
    __atomic_store_n(&u->occupancy, (uint64_t)own, __ATOMIC_RELAXED);
    if (now - o.win_start_ns >= 500000000ull) {   // utilisation over the last >= 0.5 s
      const double pct = 100.0 * (o.share_ns - o.win_start_share) / (double)(now - o.win_start_ns);
      __atomic_store_n(&u->util_pct, (uint64_t)(pct + 0.5), __ATOMIC_RELAXED);
      o.win_start_ns = now;
      o.win_start_share = o.share_ns;
    }
  }
  return true;
}

uint64_t g_occ_pass_ns = 0, g_occ_passes = 0, g_occ_pass_max_ns = 0;   // under g_occ_pass_mu

uint64_t g_hk_launches = 0;   // launches seen by the previous pass (under g_occ_pass_mu)

// The launch hooks' publishing, off the launch path: when the process launched
// since the previous pass -- the heartbeat and last-kernel time, the launch
// counts, the monitor's activity flag (recent_kernel = 2, feedback.go:74-134),
// and the latest-launch clock the sampler's "owes work" test reads.
void housekeeping(uint64_t now) {
  const uint64_t l = g_launches_local.load(std::memory_order_relaxed);
  if (l == g_hk_launches) return;
  g_hk_launches = l;
  const uint64_t c = coarse_ns();
  if (c > g_last_launch_ns.load(std::memory_order_relaxed)) g_last_launch_ns.store(c, std::memory_order_relaxed);
  __atomic_store_n(&g_region->last_kernel_time, (int64_t)time(nullptr), __ATOMIC_RELAXED);
  const int rk = __atomic_load_n(&g_region->recent_kernel, __ATOMIC_RELAXED);
  if (rk >= 0 && rk < 2) __atomic_store_n(&g_region->recent_kernel, 2, __ATOMIC_RELAXED);
  if (g_slot >= 0) {
    mivgpu_proc_slot_t* s = &g_region->procs[g_slot];
    __atomic_store_n(&s->heartbeat_ns, now, __ATOMIC_RELAXED);
    for (int d = 0; d < g_num_devices && d < MIVGPU_MAX_DEVICES; ++d)
      __atomic_store_n(&s->util[d].launches, g_dev_launches[d].load(std::memory_order_relaxed), __ATOMIC_RELAXED);
  }
}

void housekeeping_final() {
  std::lock_guard<std::mutex> pass(g_occ_pass_mu);
  housekeeping(mono_ns());
}

void* occ_main(void*) {
  int tries[MIVGPU_MAX_DEVICES] = {0};
  {   // the first launch is published at once
    std::lock_guard<std::mutex> pass(g_occ_pass_mu);
    Guard g;
    if (!g_exiting.load(std::memory_order_acquire)) housekeeping(mono_ns());
  }
  for (;;) {
    // fast while a gate ran within the last second, slow for reporting only
    const uint64_t t = coarse_ns();
    bool fast = false;
    for (int d = 0; d < g_num_devices; ++d) fast |= t - g_last_gate_ns[d].load(std::memory_order_relaxed) < 1000000000ull;
    fast |= g_board_fast.load(std::memory_order_relaxed);   // the GPU's board owner samples for every tenant
    usleep((useconds_t)((fast ? g_cfg.occ_period_ns : g_cfg.occ_idle_period_ns) / 1000));
    std::lock_guard<std::mutex> pass(g_occ_pass_mu);
    if (g_exiting.load(std::memory_order_acquire)) return nullptr;
    Guard g;
    const uint64_t now = mono_ns();
    housekeeping(now);
    if (!g_cfg.occupancy) continue;
    for (int d = 0; d < g_num_devices; ++d) {
      // a device without a KFD view is retried a few times (its identity
      // resolves at the first allocation), then left to wall-time charging
      if (!g_occ[d].live && tries[d] >= 40) continue;
      if (!occ_sample(d, now)) ++tries[d];
    }
    // the cost of a pass (KFD's cu_occupancy reads walk every XCD's waves)
    const uint64_t took = mono_ns() - now;
    g_occ_pass_ns += took;
    ++g_occ_passes;
    if (took > g_occ_pass_max_ns) g_occ_pass_max_ns = took;
  }
  return nullptr;
}

// The sampler thread doubles as the housekeeping thread (heartbeat, activity
// flag, launch counts): started at the first launch, with or without the
// occupancy sampling.
void start_occ_sampler() {
  if (g_cfg.disabled || !g_region || g_occ_started.exchange(true)) return;
  pthread_t th;
  pthread_attr_t a;
  pthread_attr_init(&a);
  pthread_attr_setdetachstate(&a, PTHREAD_CREATE_DETACHED);
  if (pthread_create(&th, &a, occ_main, nullptr) != 0) mlog(1, "occupancy sampler thread failed to start");
  pthread_attr_destroy(&a);
}

inline bool gate_wanted(int dev) {
  if (g_cfg.disabled || !g_region) return false;
  int policy = core_policy();
  if (policy == 2) return false;
  const uint64_t lim = cu_limit_ppm_of(dev);
  if (lim == 0 || lim >= 1000000) return false;   // no core limit: no switch or clock read either
  // A CU mask no wider than the limit (within one granule of one CU per XCD:
  // the device plugin rounds grants to whole granules) already enforces it in
  // hardware; time-slicing on top would charge the tenant for a GPU it cannot
  // reach (VERDICT r1 "double throttle").  This holds under policy force too:
  // force asks for the limit to be enforced, and the mask enforces it.
  const uint64_t mask = cu_mask_of(dev);
  if (mask > 0 && mask * 1000000ull <= lim * (uint64_t)device_cus(dev) + 1000000ull * (uint64_t)device_xcds(dev))
    return false;
  if (policy == 1) return true;
  // default: time-slice when there is no mask or the monitor asks for
  // contention enforcement (utilization_switch, feedback.go:74-134)
  return mask == 0 || util_switch() == 1;
}

// Enqueue one gate on `stream` for slot S (caller holds G.mu, G.ok).
void enqueue_gate_locked(int dev, DeviceGate& G, int slot, hipStream_t stream, uint64_t now) {
  GateSlot& S = G.slots[slot];
  const uint64_t first = S.first_submit_host_ns.load(std::memory_order_relaxed);
  long long submit_dev = first ? (long long)first + G.offset_ns : -1;
  const uint64_t rate = cu_limit_ppm_of(dev);
  unsigned int rate_ppm = (unsigned int)(rate < 1000000ull ? rate : 1000000ull);
  long long cap = g_cfg.gate_cap_ns, hold = g_cfg.gate_max_hold_ns;
  int slot_arg = slot;
  unsigned int use_share = g_occ_live[dev].load(std::memory_order_acquire) ? 1u : 0u;
  // bit 0: trace ring; bit 1: host-bucket mode (the sampler keeps the bucket)
  unsigned int flags = (g_cfg.gate_trace ? 1u : 0u) | (use_share && !g_cfg.gate_device_mode ? 2u : 0u);
  const bool occupancy = use_share != 0;
  void* state = G.state;
  void* hs = G.host_stats;
  void* args[] = {&state, &hs, &submit_dev, &slot_arg, &rate_ppm, &cap, &hold, &use_share, &flags};
  if (real_hipModuleLaunchKernel()(G.gate_fn, 1, 1, 1, 64, 1, 1, 0, stream, args, nullptr) != hipSuccess) {
    static std::atomic<bool> warned{false};
    if (!warned.exchange(true)) mlog(1, "device %d: governor gate launch failed; this batch is not throttled", dev);
    return;
  }
  g_last_gate_ns[dev].store(coarse_ns(), std::memory_order_relaxed);
  G.enqueued.fetch_add(1, std::memory_order_release);
  tmark("mivgpu:gate dev=%d slot=%d rate_pct=%u charge=%s", dev, slot, rate_ppm / 10000u,
        occupancy ? "occupancy" : "wall");
  S.last_gate_host_ns.store(now, std::memory_order_relaxed);
  if (g_slot >= 0 && hs) {
    const uint64_t* h = static_cast<const uint64_t*>(hs);
    mivgpu_util_t* u = &g_region->procs[g_slot].util[dev];
    // GPU time received: the share integral in host-bucket mode, the gates'
    // busy wall time otherwise
    __atomic_store_n(&u->busy_ns, occupancy ? __atomic_load_n(&u->share_ns, __ATOMIC_RELAXED) : h[0],
                     __ATOMIC_RELAXED);
    __atomic_store_n(&u->throttled_ns, h[1], __ATOMIC_RELAXED);
    __atomic_store_n(&u->gates, h[2], __ATOMIC_RELAXED);
  }
}

// Only asked of the runtime while a capture begun through the hooks is in
// flight: the common case (no capture anywhere in the process) costs one load.
bool stream_capturing(hipStream_t stream) {
  if (g_captures.load(std::memory_order_acquire) <= 0) return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return real_hipStreamIsCapturing() && real_hipStreamIsCapturing()(stream, &cs) == hipSuccess &&
         cs != hipStreamCaptureStatusNone;
}

int find_slot_locked(DeviceGate& G, hipStream_t stream, bool create, uint64_t now) {
  int free_slot = -1;
  for (int i = 0; i < 64; ++i) {
    const bool used = G.slots[i].used.load(std::memory_order_relaxed);
    if (used && G.slots[i].stream.load(std::memory_order_relaxed) == stream) return i;
    if (!used && free_slot < 0) free_slot = i;
  }
  if (!create) return -1;
  int slot = free_slot >= 0 ? free_slot : (int)(reinterpret_cast<uintptr_t>(stream) % 64);
  GateSlot& S = G.slots[slot];
  S.used.store(false, std::memory_order_release);   // fast path: not this slot while it changes hands
  S.stream.store(stream, std::memory_order_relaxed);
  S.last_gate_host_ns.store(0, std::memory_order_relaxed);
  S.first_submit_host_ns.store(0, std::memory_order_relaxed);
  S.last_launch_host_ns.store(0, std::memory_order_relaxed);
  S.batch_launches.store(0, std::memory_order_relaxed);
  S.in_launch.store(0, std::memory_order_relaxed);
  S.used.store(true, std::memory_order_release);
  (void)now;
  return slot;
}

// Background stamper: once the host has not launched on a stream for
// kStampIdleNs, close that stream's pending batch with a gate, so a host-side
// pause (CPU work, library initialisation, data loading) is never charged to
// the tenant as GPU-busy time.  Runs under G.mu, which hipStreamBeginCapture
// also takes, so a stamp can never be captured into a user graph.
void enqueue_gate_locked(int dev, DeviceGate& G, int slot, hipStream_t stream, uint64_t now);
bool stream_capturing(hipStream_t stream);

// Wait out a stamper that is inside an enqueue (it holds G.mu), so no gate
// launch races the runtime's teardown; later passes see g_exiting and stop.
void quiesce_background_threads() {
  { std::lock_guard<std::mutex> pass(g_occ_pass_mu); }   // an occupancy pass in flight ends first
  for (int d = 0; d < MIVGPU_MAX_DEVICES; ++d) {
    DeviceGate& G = g_gates[d];
    if (!G.stamper_started) continue;
    std::lock_guard<std::mutex> lk(G.mu);
  }
}

void* stamper_main(void* arg) {
  const int dev = (int)(intptr_t)arg;
  DeviceGate& G = g_gates[dev];
  {
    Guard g;  // our own HIP calls must never re-enter the hooks' accounting
    if (real_hipSetDevice() && real_hipSetDevice()(dev) != hipSuccess)
      mlog(1, "device %d: governor stamper could not select the device", dev);
  }
  for (;;) {
    usleep(500);
    Guard g;
    std::lock_guard<std::mutex> lk(G.mu);
    if (g_exiting.load(std::memory_order_acquire)) return nullptr;
    const uint64_t now = mono_ns();
    for (int i = 0; i < 64; ++i) {
      GateSlot& S = G.slots[i];
      if (!S.used.load(std::memory_order_relaxed) || S.first_submit_host_ns.load(std::memory_order_relaxed) == 0)
        continue;
      // a launch call still in progress (e.g. blocked on a full queue) is not
      // idleness: a gate enqueued now could land in front of that launch's
      // packets and close its batch before the work is in it (measured: a
      // 50 % limit ran at 67-86 % of the unthrottled rate under backpressure)
      // the idle clock is stored before in_launch drops (release)
      if (S.in_launch.load(std::memory_order_acquire) > 0) continue;
      if (now - S.last_launch_host_ns.load(std::memory_order_relaxed) < kStampIdleNs) continue;
      const hipStream_t st = S.stream.load(std::memory_order_relaxed);
      if (stream_capturing(st)) continue;
      enqueue_gate_locked(dev, G, i, st, now);
      S.first_submit_host_ns.store(0, std::memory_order_relaxed);
    }
  }
  return nullptr;
}

void start_stamper_locked(int dev, DeviceGate& G) {
  G.stamper_started = true;
  pthread_t th;
  pthread_attr_t a;
  pthread_attr_init(&a);
  pthread_attr_setdetachstate(&a, PTHREAD_CREATE_DETACHED);
  if (pthread_create(&th, &a, stamper_main, (void*)(intptr_t)dev) != 0)
    mlog(1, "device %d: governor stamper thread failed to start", dev);
  pthread_attr_destroy(&a);
}

// A gate settles the batch submitted since the previous one; its debt is
// capped at one burst, so a batch must not hold much more GPU time than that
// (the host can enqueue 100 ms of graph replays within the 200 us interval:
// measured 66 % throughput at a 50 % limit).  Gate in front of every graph
// launch and after at most kMaxBatchLaunches kernels, whatever the host time.

// Returns the gate slot of `stream` (its in_launch count raised; the caller's
// LaunchScope lowers it when the real launch call returns), or -1.
// The host bucket is in debt: the next gate will hold.  While it is, every
// launch gets a gate in front of it -- a gate holds at most gate_max_hold_ns,
// and a batch behind a gate that released on that bound while still in debt
// ran unthrottled (measured: a 12.5 % tenant running 8192^3 GEMMs in 10 ms
// batches behind 25 ms holds got 0.24-0.29 of its unthrottled rate).
inline bool in_debt(int dev) {
  if (g_cfg.gate_device_mode || !g_occ_live[dev].load(std::memory_order_relaxed)) return false;
  const uint64_t* hs = static_cast<const uint64_t*>(g_gates[dev].hs_pub.load(std::memory_order_relaxed));
  return hs && (int64_t)__atomic_load_n(&hs[kHsHostTokens], __ATOMIC_RELAXED) < 0;
}

inline int batch_limit(int dev) {
  if (!g_occ_live[dev].load(std::memory_order_relaxed)) return kMaxBatchLaunches;
  const int b = g_batch_max[dev].load(std::memory_order_relaxed);
  return b > 0 ? b : 16;
}

int maybe_gate(hipStream_t stream, bool graph, int dev) {
  if (!gate_wanted(dev)) return -1;
  // Never inject into a stream that is being captured: the gate would be baked
  // into the graph with stale arguments.  Graph replays are gated at launch.
  if (stream_capturing(stream)) return -1;
  DeviceGate& G = g_gates[dev];
  uint64_t now = mono_ns();
  // Fast path, no mutex: a launch that only extends the open batch of a known
  // stream (no gate due).  in_launch goes up BEFORE the batch state is read,
  // so the idle stamper (which skips a stream with a launch in progress)
  // cannot close the batch under it unseen.
  if (!graph && G.ok_pub.load(std::memory_order_acquire)) {
    for (int i = 0; i < 64; ++i) {
      GateSlot& S = G.slots[i];
      if (!S.used.load(std::memory_order_acquire) || S.stream.load(std::memory_order_relaxed) != stream) continue;
      S.in_launch.fetch_add(1, std::memory_order_acq_rel);
      const uint64_t first = S.first_submit_host_ns.load(std::memory_order_acquire);
      const uint64_t last = S.last_gate_host_ns.load(std::memory_order_relaxed);
      if (first != 0 && last != 0 && now - last < g_cfg.gate_min_interval_ns && !in_debt(dev) &&
          S.batch_launches.fetch_add(1, std::memory_order_relaxed) + 1 <= batch_limit(dev)) {
        S.last_launch_host_ns.store(now, std::memory_order_relaxed);
        return i;
      }
      S.in_launch.fetch_sub(1, std::memory_order_acq_rel);   // a gate is due: the slow path decides
      break;
    }
  }
  std::lock_guard<std::mutex> lk(G.mu);
  if (!G.tried) {
    G.ok = gate_init_locked(dev, G);
    G.ok_pub.store(G.ok, std::memory_order_release);
  }
  if (!G.ok) return -1;
  int slot = find_slot_locked(G, stream, true, now);
  GateSlot& S = G.slots[slot];
  S.last_launch_host_ns.store(now, std::memory_order_relaxed);
  S.in_launch.fetch_add(1, std::memory_order_relaxed);
  if (!G.stamper_started) start_stamper_locked(dev, G);
  const bool pending = S.first_submit_host_ns.load(std::memory_order_relaxed) != 0;
  const uint64_t last_gate = S.last_gate_host_ns.load(std::memory_order_relaxed);
  if (!pending || last_gate == 0 || graph || S.batch_launches.load(std::memory_order_relaxed) >= batch_limit(dev) ||
      now - last_gate >= g_cfg.gate_min_interval_ns || in_debt(dev)) {
    // Gate in front of this launch: settles the batch submitted since the
    // previous gate (if any); this launch starts the next batch.
    enqueue_gate_locked(dev, G, slot, stream, now);
    S.first_submit_host_ns.store(now, std::memory_order_release);
    S.batch_launches.store(1, std::memory_order_relaxed);
    return slot;
  }
  S.batch_launches.fetch_add(1, std::memory_order_relaxed);
  return slot;
}

struct LaunchTicket {
  int dev = -1;
  int slot = -1;
};

// Ends a launch call: the stream's idle clock starts when the call returns.
struct LaunchScope {
  LaunchTicket t;
  explicit LaunchScope(LaunchTicket x) : t(x) {}
  ~LaunchScope() {
    if (t.slot < 0) return;
    GateSlot& S = g_gates[t.dev].slots[t.slot];
    S.last_launch_host_ns.store(mono_ns(), std::memory_order_relaxed);
    int n = S.in_launch.load(std::memory_order_relaxed);
    while (n > 0 && !S.in_launch.compare_exchange_weak(n, n - 1, std::memory_order_release,
                                                       std::memory_order_relaxed)) {
    }
  }
};

// The host is about to wait for the GPU, after which the stream idles: stamp
// the pending batch so that the idle gap is never charged as busy time.
void stamp_before_sync(hipStream_t stream, bool all_streams) {
  if (g_cfg.disabled || !g_region) return;
  int dev = current_device();
  DeviceGate& G = g_gates[dev];
  if (!G.ok_pub.load(std::memory_order_acquire)) return;
  std::lock_guard<std::mutex> lk(G.mu);
  uint64_t now = mono_ns();
  for (int i = 0; i < 64; ++i) {
    GateSlot& S = G.slots[i];
    if (!S.used.load(std::memory_order_relaxed) || S.first_submit_host_ns.load(std::memory_order_relaxed) == 0)
      continue;
    const hipStream_t st = S.stream.load(std::memory_order_relaxed);
    if (!all_streams && st != stream) continue;
    if (stream_capturing(st)) continue;
    enqueue_gate_locked(dev, G, i, st, now);
    S.first_submit_host_ns.store(0, std::memory_order_relaxed);  // nothing pending until the next launch
  }
}

// Any device of the process under a core limit (each device has its own,
// HIP_DEVICE_CORE_LIMIT_<i>; the gate decision itself is per device).
inline bool any_core_limit() {
  if (g_any_limit_static >= 0) return g_any_limit_static != 0;
  const int n = g_num_devices > 0 ? g_num_devices : 1;
  for (int d = 0; d < n; ++d) {
    const uint64_t cl = cu_limit_ppm_of(d);
    if (cl > 0 && cl < 1000000) return true;
  }
  return false;
}

// Parks the calling launch while a block is in force: the monitor's verdict
// in the read-only control file (over grant, or a higher-priority task; held
// while its lease is live), or the legacy region flag (recent_kernel == -1).
void park_while_blocked() {
  TRange r("mivgpu:priority-block");
  const uint64_t t0 = coarse_ns();
  for (;;) {
    const bool ctl = ctl_block();
    const bool reg = __atomic_load_n(&g_region->recent_kernel, __ATOMIC_RELAXED) < 0;
    if (!ctl && !reg) return;
    // the region flag is tenant-writable and has no lease: never wedge on it
    if (!ctl && coarse_ns() - t0 > 60ull * 1000000000ull) return;
    usleep(1000);
  }
}

// Per-launch bookkeeping.  Hot path when nothing throttles: the TLS guard, a
// few relaxed loads and one counter increment -- no clock read, no region
// store (the housekeeping thread publishes the heartbeat, the activity flag
// and the launch counts, see housekeeping()).  `dev` < 0: the calling
// thread's current device (the launch's device).
inline LaunchTicket on_launch(hipStream_t stream, bool graph = false, int dev = -1) {
  ensure_init();
  if (g_cfg.disabled || !g_region) return LaunchTicket{};
  const int hd = dev >= 0 ? dev : (g_num_devices == 1 ? 0 : current_device());
  if (__builtin_expect(g_launches_local.fetch_add(1, std::memory_order_relaxed) == 0, 0)) start_occ_sampler();
  g_dev_launches[hd].fetch_add(1, std::memory_order_relaxed);
  if (__builtin_expect(__atomic_load_n(&g_region->recent_kernel, __ATOMIC_RELAXED) < 0 ||
                       (g_ctl && __atomic_load_n(&g_ctl->block, __ATOMIC_RELAXED)), 0))
    park_while_blocked();
  if (__builtin_expect(any_core_limit() || util_switch(), 0)) {
    g_last_launch_ns.store(coarse_ns(), std::memory_order_relaxed);
    return LaunchTicket{hd, maybe_gate(stream, graph, hd)};
  }
  return LaunchTicket{};
}

}  // namespace

// ======================================================================
// Exported hooks (versions in mivgpu_shim.map must match libamdhip64).
// ======================================================================

MIVGPU_EXPORT hipError_t hipMalloc(void** ptr, size_t size) {
  return guarded_alloc(ptr, size, [&] { return real_hipMalloc()(ptr, size); });
}

MIVGPU_EXPORT hipError_t hipExtMallocWithFlags(void** ptr, size_t size, unsigned int flags) {
  return guarded_alloc(ptr, size, [&] { return real_hipExtMallocWithFlags()(ptr, size, flags); });
}

MIVGPU_EXPORT hipError_t hipMallocManaged(void** ptr, size_t size, unsigned int flags) {
  return guarded_alloc(ptr, size, [&] { return real_hipMallocManaged()(ptr, size, flags); });
}

MIVGPU_EXPORT hipError_t hipMallocAsync(void** ptr, size_t size, hipStream_t stream) {
  return guarded_alloc(ptr, size, [&] { return real_hipMallocAsync()(ptr, size, stream); });
}

MIVGPU_EXPORT hipError_t hipMallocFromPoolAsync(void** ptr, size_t size, hipMemPool_t pool,
                                                hipStream_t stream) {
  return guarded_alloc(ptr, size,
                       [&] { return real_hipMallocFromPoolAsync()(ptr, size, pool, stream); });
}

MIVGPU_EXPORT hipError_t hipMallocPitch(void** ptr, size_t* pitch, size_t width, size_t height) {
  ensure_init();
  Guard g;
  if (!g.outer) return real_hipMallocPitch()(ptr, pitch, width, height);
  // The pitch is only known after the call: reserve a conservative estimate
  // (rows rounded to 512 B), then true it up.
  uint64_t est = ((width + 511) & ~511ull) * height;
  int dev = current_device();
  if (!reserve(dev, est, K_BUFFER)) return hipErrorOutOfMemory;
  hipError_t rc = real_hipMallocPitch()(ptr, pitch, width, height);
  if (rc != hipSuccess) {
    account_sub(dev, est, K_BUFFER);
    return rc;
  }
  uint64_t real_sz = (uint64_t)(*pitch) * height;
  if (real_sz > est) account_add(dev, real_sz - est, K_BUFFER);
  else account_sub(dev, est - real_sz, K_BUFFER);
  track(*ptr, real_sz, dev, K_BUFFER);
  return rc;
}

MIVGPU_EXPORT hipError_t hipMemAllocPitch(hipDeviceptr_t* ptr, size_t* pitch, size_t width,
                                          size_t height, unsigned int elem) {
  ensure_init();
  Guard g;
  if (!g.outer) return real_hipMemAllocPitch()(ptr, pitch, width, height, elem);
  uint64_t est = ((width + 511) & ~511ull) * height;
  int dev = current_device();
  if (!reserve(dev, est, K_BUFFER)) return hipErrorOutOfMemory;
  hipError_t rc = real_hipMemAllocPitch()(ptr, pitch, width, height, elem);
  if (rc != hipSuccess) {
    account_sub(dev, est, K_BUFFER);
    return rc;
  }
  uint64_t real_sz = (uint64_t)(*pitch) * height;
  if (real_sz > est) account_add(dev, real_sz - est, K_BUFFER);
  else account_sub(dev, est - real_sz, K_BUFFER);
  track((void*)*ptr, real_sz, dev, K_BUFFER);
  return rc;
}

// hipMalloc3D: extent.width is in bytes; the pitch is known after the call.
MIVGPU_EXPORT hipError_t hipMalloc3D(hipPitchedPtr* pp, hipExtent extent) {
  ensure_init();
  Guard g;
  if (!g.outer) return real_hipMalloc3D()(pp, extent);
  const uint64_t est = array_bytes(1, extent.width, extent.height, extent.depth);
  const int dev = current_device();
  if (!reserve(dev, est, K_BUFFER)) return hipErrorOutOfMemory;
  hipError_t rc = real_hipMalloc3D()(pp, extent);
  if (rc != hipSuccess || !pp || !pp->ptr) {
    account_sub(dev, est, K_BUFFER);
    return rc;
  }
  const uint64_t real_sz = (uint64_t)pp->pitch * (extent.height ? extent.height : 1) * (extent.depth ? extent.depth : 1);
  if (real_sz > est) account_add(dev, real_sz - est, K_BUFFER);
  else account_sub(dev, est - real_sz, K_BUFFER);
  track(pp->ptr, real_sz, dev, K_BUFFER);
  return rc;
}

MIVGPU_EXPORT hipError_t hipMallocArray(hipArray_t* array, const hipChannelFormatDesc* desc, size_t width,
                                        size_t height, unsigned int flags) {
  return guarded_handle_alloc(reinterpret_cast<void**>(array), array_bytes(channel_bytes(desc), width, height, 1),
                              [&] { return real_hipMallocArray()(array, desc, width, height, flags); });
}

MIVGPU_EXPORT hipError_t hipMalloc3DArray(hipArray_t* array, const hipChannelFormatDesc* desc, hipExtent extent,
                                          unsigned int flags) {
  return guarded_handle_alloc(reinterpret_cast<void**>(array),
                              array_bytes(channel_bytes(desc), extent.width, extent.height, extent.depth),
                              [&] { return real_hipMalloc3DArray()(array, desc, extent, flags); });
}

MIVGPU_EXPORT hipError_t hipArrayCreate(hipArray_t* array, const HIP_ARRAY_DESCRIPTOR* d) {
  const uint64_t bytes = d ? array_bytes(format_bytes(d->Format, d->NumChannels), d->Width, d->Height, 1) : 0;
  return guarded_handle_alloc(reinterpret_cast<void**>(array), bytes, [&] { return real_hipArrayCreate()(array, d); });
}

MIVGPU_EXPORT hipError_t hipArray3DCreate(hipArray_t* array, const HIP_ARRAY3D_DESCRIPTOR* d) {
  const uint64_t bytes =
      d ? array_bytes(format_bytes(d->Format, d->NumChannels), d->Width, d->Height, d->Depth) : 0;
  return guarded_handle_alloc(reinterpret_cast<void**>(array), bytes, [&] { return real_hipArray3DCreate()(array, d); });
}

MIVGPU_EXPORT hipError_t hipMallocMipmappedArray(hipMipmappedArray_t* mip, const hipChannelFormatDesc* desc,
                                                 hipExtent extent, unsigned int levels, unsigned int flags) {
  return guarded_handle_alloc(reinterpret_cast<void**>(mip),
                              mip_bytes(channel_bytes(desc), extent.width, extent.height, extent.depth, levels),
                              [&] { return real_hipMallocMipmappedArray()(mip, desc, extent, levels, flags); });
}

MIVGPU_EXPORT hipError_t hipMipmappedArrayCreate(hipMipmappedArray_t* mip, HIP_ARRAY3D_DESCRIPTOR* d,
                                                 unsigned int levels) {
  const uint64_t bytes =
      d ? mip_bytes(format_bytes(d->Format, d->NumChannels), d->Width, d->Height, d->Depth, levels) : 0;
  return guarded_handle_alloc(reinterpret_cast<void**>(mip), bytes,
                              [&] { return real_hipMipmappedArrayCreate()(mip, d, levels); });
}

#define HANDLE_FREE_HOOK(name, type)                                   \
  MIVGPU_EXPORT hipError_t name(type h) {                               \
    ensure_init();                                                      \
    Guard g;                                                            \
    hipError_t rc = real_##name()(h);                                   \
    if (g.outer && rc == hipSuccess) release_tracked(reinterpret_cast<void*>(h)); \
    return rc;                                                          \
  }
HANDLE_FREE_HOOK(hipFreeArray, hipArray_t)
HANDLE_FREE_HOOK(hipArrayDestroy, hipArray_t)
HANDLE_FREE_HOOK(hipFreeMipmappedArray, hipMipmappedArray_t)
HANDLE_FREE_HOOK(hipMipmappedArrayDestroy, hipMipmappedArray_t)
HANDLE_FREE_HOOK(hipModuleUnload, hipModule_t)

MIVGPU_EXPORT hipError_t hipModuleLoad(hipModule_t* module, const char* fname) {
  return guarded_module_load(module, code_object_file_bytes(fname), [&] { return real_hipModuleLoad()(module, fname); });
}

MIVGPU_EXPORT hipError_t hipModuleLoadData(hipModule_t* module, const void* image) {
  return guarded_module_load(module, code_object_bytes(image, ~0ull),
                             [&] { return real_hipModuleLoadData()(module, image); });
}

MIVGPU_EXPORT hipError_t hipModuleLoadDataEx(hipModule_t* module, const void* image, unsigned int n,
                                             hipJitOption* opts, void** vals) {
  return guarded_module_load(module, code_object_bytes(image, ~0ull),
                             [&] { return real_hipModuleLoadDataEx()(module, image, n, opts, vals); });
}

MIVGPU_EXPORT hipError_t hipFree(void* ptr) {
  ensure_init();
  Guard g;
  if (g.outer && release_tracked(ptr)) return hipSuccess;
  return real_hipFree()(ptr);
}

MIVGPU_EXPORT hipError_t hipFreeAsync(void* ptr, hipStream_t stream) {
  ensure_init();
  Guard g;
  if (g.outer && release_tracked(ptr)) return hipSuccess;
  return real_hipFreeAsync()(ptr, stream);
}

MIVGPU_EXPORT hipError_t hipMemCreate(hipMemGenericAllocationHandle_t* handle, size_t size,
                                      const hipMemAllocationProp* prop, unsigned long long flags) {
  ensure_init();
  Guard g;
  if (!g.outer) return real_hipMemCreate()(handle, size, prop, flags);
  int dev = prop ? prop->location.id : current_device();
  if (dev < 0 || dev >= MIVGPU_MAX_DEVICES) dev = 0;
  if (!reserve(dev, size, K_VMM)) return hipErrorOutOfMemory;
  hipError_t rc = real_hipMemCreate()(handle, size, prop, flags);
  if (rc != hipSuccess) {
    account_sub(dev, size, K_VMM);
    return rc;
  }
  track(reinterpret_cast<void*>(*handle), size, dev, K_VMM);
  return rc;
}

MIVGPU_EXPORT hipError_t hipMemRelease(hipMemGenericAllocationHandle_t handle) {
  ensure_init();
  Guard g;
  hipError_t rc = real_hipMemRelease()(handle);
  if (g.outer && rc == hipSuccess) release_tracked(reinterpret_cast<void*>(handle));
  return rc;
}

MIVGPU_EXPORT hipError_t hipMemGetInfo(size_t* free_b, size_t* total_b) {
  ensure_init();
  Guard g;
  hipError_t rc = real_hipMemGetInfo()(free_b, total_b);
  if (rc != hipSuccess || !g.outer) return rc;
  int dev = current_device();
  uint64_t lim = limit_of(dev);
  if (lim && g_region) {
    refresh_context(dev, false);
    uint64_t used = __atomic_load_n(&g_region->dev_used[dev], __ATOMIC_RELAXED) + ctl_excess(dev);
    uint64_t vfree = used >= lim ? 0 : lim - used;
    if (free_b) *free_b = vfree < *free_b ? vfree : *free_b;
    if (total_b) *total_b = lim;
  }
  return rc;
}

MIVGPU_EXPORT hipError_t hipDeviceTotalMem(size_t* bytes, hipDevice_t device) {
  ensure_init();
  Guard g;
  hipError_t rc = real_hipDeviceTotalMem()(bytes, device);
  if (rc == hipSuccess && bytes && device >= 0 && device < MIVGPU_MAX_DEVICES) {
    uint64_t lim = limit_of(device);
    if (lim) *bytes = lim;
  }
  return rc;
}

MIVGPU_EXPORT hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* prop, int device) {
  ensure_init();
  Guard g;
  hipError_t rc = real_hipGetDevicePropertiesR0600()(prop, device);
  if (rc == hipSuccess && prop && device >= 0 && device < MIVGPU_MAX_DEVICES) {
    uint64_t lim = limit_of(device);
    if (lim) prop->totalGlobalMem = lim;
  }
  return rc;
}

MIVGPU_EXPORT hipError_t hipGetDevicePropertiesR0000(void* prop, int device) {
  ensure_init();
  Guard g;
  hipError_t rc = real_hipGetDevicePropertiesR0000()(prop, device);
  if (rc == hipSuccess && prop && device >= 0 && device < MIVGPU_MAX_DEVICES) {
    uint64_t lim = limit_of(device);
    // hipDeviceProp_tR0000: char name[256]; size_t totalGlobalMem; (hip_deprecated.h:28-30)
    if (lim) *reinterpret_cast<size_t*>(static_cast<char*>(prop) + 256) = lim;
  }
  return rc;
}

// Cost-attribution builds of the launch path (utils/build.py build_hook_diag;
// separate files under build/diag, never the shipped library): level 1
// forwards the launch untouched (the interposition alone), 2 adds the
// re-entrancy guard and the lazy-init check, 3 adds the launch counters.
// The shipped build compiles the full prologue below.
#if defined(MIVGPU_HOOK_DIAG) && MIVGPU_HOOK_DIAG == 1
#define LAUNCH_PROLOGUE(stream) (void)(stream);
#elif defined(MIVGPU_HOOK_DIAG) && MIVGPU_HOOK_DIAG == 2
#define LAUNCH_PROLOGUE(stream) \
  Guard g_guard;                \
  ensure_init();                \
  (void)(stream);
#elif defined(MIVGPU_HOOK_DIAG) && MIVGPU_HOOK_DIAG == 3
#define LAUNCH_PROLOGUE(stream)                                                        \
  Guard g_guard;                                                                       \
  ensure_init();                                                                       \
  if (g_guard.outer && g_launches_local.fetch_add(1, std::memory_order_relaxed) == 0) \
    start_occ_sampler();                                                               \
  g_dev_launches[0].fetch_add(1, std::memory_order_relaxed);                           \
  (void)(stream);
#else
#define LAUNCH_PROLOGUE(stream)   \
  Guard g_guard;                  \
  LaunchScope g_scope(g_guard.outer ? on_launch(stream) : LaunchTicket{});
#endif
#define GRAPH_LAUNCH_PROLOGUE(stream) \
  Guard g_guard;                      \
  LaunchScope g_scope(g_guard.outer ? on_launch(stream, true) : LaunchTicket{});

MIVGPU_EXPORT hipError_t hipLaunchKernel(const void* f, dim3 grid, dim3 block, void** args,
                                         size_t shmem, hipStream_t stream) {
  LAUNCH_PROLOGUE(stream);
  return real_hipLaunchKernel()(f, grid, block, args, shmem, stream);
}

MIVGPU_EXPORT hipError_t hipLaunchKernel_spt(const void* f, dim3 grid, dim3 block, void** args,
                                             size_t shmem, hipStream_t stream) {
  LAUNCH_PROLOGUE(stream);
  return real_hipLaunchKernel_spt()(f, grid, block, args, shmem, stream);
}

MIVGPU_EXPORT hipError_t hipModuleLaunchKernel(hipFunction_t f, unsigned gx, unsigned gy,
                                               unsigned gz, unsigned bx, unsigned by, unsigned bz,
                                               unsigned shmem, hipStream_t stream, void** params,
                                               void** extra) {
  LAUNCH_PROLOGUE(stream);
  return real_hipModuleLaunchKernel()(f, gx, gy, gz, bx, by, bz, shmem, stream, params, extra);
}

MIVGPU_EXPORT hipError_t hipExtModuleLaunchKernel(hipFunction_t f, uint32_t gx, uint32_t gy,
                                                  uint32_t gz, uint32_t lx, uint32_t ly,
                                                  uint32_t lz, size_t shmem, hipStream_t stream,
                                                  void** params, void** extra, hipEvent_t start,
                                                  hipEvent_t stop, uint32_t flags) {
  LAUNCH_PROLOGUE(stream);
  return real_hipExtModuleLaunchKernel()(f, gx, gy, gz, lx, ly, lz, shmem, stream, params, extra,
                                         start, stop, flags);
}

MIVGPU_EXPORT hipError_t hipHccModuleLaunchKernel(hipFunction_t f, uint32_t gx, uint32_t gy,
                                                  uint32_t gz, uint32_t lx, uint32_t ly,
                                                  uint32_t lz, size_t shmem, hipStream_t stream,
                                                  void** params, void** extra, hipEvent_t start,
                                                  hipEvent_t stop) {
  LAUNCH_PROLOGUE(stream);
  return real_hipHccModuleLaunchKernel()(f, gx, gy, gz, lx, ly, lz, shmem, stream, params, extra,
                                         start, stop);
}

MIVGPU_EXPORT hipError_t hipLaunchCooperativeKernel(const void* f, dim3 grid, dim3 block,
                                                    void** args, unsigned int shmem,
                                                    hipStream_t stream) {
  LAUNCH_PROLOGUE(stream);
  return real_hipLaunchCooperativeKernel()(f, grid, block, args, shmem, stream);
}

MIVGPU_EXPORT hipError_t hipModuleLaunchCooperativeKernel(hipFunction_t f, unsigned gx,
                                                          unsigned gy, unsigned gz, unsigned bx,
                                                          unsigned by, unsigned bz, unsigned shmem,
                                                          hipStream_t stream, void** params) {
  LAUNCH_PROLOGUE(stream);
  return real_hipModuleLaunchCooperativeKernel()(f, gx, gy, gz, bx, by, bz, shmem, stream, params);
}

MIVGPU_EXPORT hipError_t hipExtLaunchKernel(const void* f, dim3 grid, dim3 block, void** args,
                                            size_t shmem, hipStream_t stream, hipEvent_t start,
                                            hipEvent_t stop, int flags) {
  LAUNCH_PROLOGUE(stream);
  return real_hipExtLaunchKernel()(f, grid, block, args, shmem, stream, start, stop, flags);
}

MIVGPU_EXPORT hipError_t hipGraphLaunch(hipGraphExec_t exec, hipStream_t stream) {
  GRAPH_LAUNCH_PROLOGUE(stream);
  return real_hipGraphLaunch()(exec, stream);
}

MIVGPU_EXPORT hipError_t hipGraphLaunch_spt(hipGraphExec_t exec, hipStream_t stream) {
  GRAPH_LAUNCH_PROLOGUE(stream);
  return real_hipGraphLaunch_spt()(exec, stream);
}

MIVGPU_EXPORT hipError_t hipLaunchKernelExC(const hipLaunchConfig_t* config, const void* f, void** args) {
  if (!real_hipLaunchKernelExC()) return hipErrorNotSupported;
  LAUNCH_PROLOGUE(config ? config->stream : nullptr);
  return real_hipLaunchKernelExC()(config, f, args);
}

MIVGPU_EXPORT hipError_t hipDrvLaunchKernelEx(const HIP_LAUNCH_CONFIG* config, hipFunction_t f, void** params,
                                              void** extra) {
  if (!real_hipDrvLaunchKernelEx()) return hipErrorNotSupported;
  LAUNCH_PROLOGUE(config ? config->hStream : nullptr);
  return real_hipDrvLaunchKernelEx()(config, f, params, extra);
}

// One launch per device, each on its own stream: every entry is gated on its
// stream's device (the gates of device d run from device d's code object).
template <typename Call>
hipError_t multi_device_launch(hipLaunchParams* list, int n, Call&& call) {
  Guard g;
  if (!g.outer || !list || n <= 0 || n > MIVGPU_MAX_DEVICES) return call();
  LaunchTicket tickets[MIVGPU_MAX_DEVICES];
  for (int i = 0; i < n; ++i) {
    hipDevice_t d = -1;
    if (!real_hipStreamGetDevice() || real_hipStreamGetDevice()(list[i].stream, &d) != hipSuccess || d < 0 ||
        d >= MIVGPU_MAX_DEVICES)
      d = -1;
    tickets[i] = on_launch(list[i].stream, false, d);
  }
  hipError_t rc = call();
  for (int i = 0; i < n; ++i) LaunchScope end(tickets[i]);
  return rc;
}

MIVGPU_EXPORT hipError_t hipLaunchCooperativeKernelMultiDevice(hipLaunchParams* list, int n, unsigned int flags) {
  return multi_device_launch(list, n, [&] { return real_hipLaunchCooperativeKernelMultiDevice()(list, n, flags); });
}

MIVGPU_EXPORT hipError_t hipExtLaunchMultiKernelMultiDevice(hipLaunchParams* list, int n, unsigned int flags) {
  return multi_device_launch(list, n, [&] { return real_hipExtLaunchMultiKernelMultiDevice()(list, n, flags); });
}

// Serialise capture begin with the background stamper (see stamper_main).
MIVGPU_EXPORT hipError_t hipStreamBeginCapture(hipStream_t stream, hipStreamCaptureMode mode) {
  ensure_init();
  Guard g;
  DeviceGate& G = g_gates[current_device()];
  std::lock_guard<std::mutex> lk(G.mu);
  hipError_t rc = real_hipStreamBeginCapture()(stream, mode);
  if (rc == hipSuccess) g_captures.fetch_add(1, std::memory_order_acq_rel);
  return rc;
}

MIVGPU_EXPORT hipError_t hipStreamBeginCapture_spt(hipStream_t stream, hipStreamCaptureMode mode) {
  ensure_init();
  Guard g;
  DeviceGate& G = g_gates[current_device()];
  std::lock_guard<std::mutex> lk(G.mu);
  hipError_t rc = real_hipStreamBeginCapture_spt()(stream, mode);
  if (rc == hipSuccess) g_captures.fetch_add(1, std::memory_order_acq_rel);
  return rc;
}

MIVGPU_EXPORT hipError_t hipStreamBeginCaptureToGraph(hipStream_t stream, hipGraph_t graph,
                                                      const hipGraphNode_t* deps, const hipGraphEdgeData* data,
                                                      size_t ndeps, hipStreamCaptureMode mode) {
  ensure_init();
  Guard g;
  DeviceGate& G = g_gates[current_device()];
  std::lock_guard<std::mutex> lk(G.mu);
  hipError_t rc = real_hipStreamBeginCaptureToGraph()(stream, graph, deps, data, ndeps, mode);
  if (rc == hipSuccess) g_captures.fetch_add(1, std::memory_order_acq_rel);
  return rc;
}

// A capture ends (successfully or invalidated) with hipStreamEndCapture.
MIVGPU_EXPORT hipError_t hipStreamEndCapture(hipStream_t stream, hipGraph_t* graph) {
  hipError_t rc = real_hipStreamEndCapture()(stream, graph);
  if (g_captures.load(std::memory_order_acquire) > 0) g_captures.fetch_sub(1, std::memory_order_acq_rel);
  return rc;
}

MIVGPU_EXPORT hipError_t hipStreamEndCapture_spt(hipStream_t stream, hipGraph_t* graph) {
  hipError_t rc = real_hipStreamEndCapture_spt()(stream, graph);
  if (g_captures.load(std::memory_order_acquire) > 0) g_captures.fetch_sub(1, std::memory_order_acq_rel);
  return rc;
}

MIVGPU_EXPORT hipError_t hipStreamSynchronize(hipStream_t stream) {
  Guard g;
  if (g.outer && g_ready.load(std::memory_order_acquire)) stamp_before_sync(stream, false);
  return real_hipStreamSynchronize()(stream);
}

MIVGPU_EXPORT hipError_t hipStreamSynchronize_spt(hipStream_t stream) {
  Guard g;
  if (g.outer && g_ready.load(std::memory_order_acquire)) stamp_before_sync(stream, false);
  return real_hipStreamSynchronize_spt()(stream);
}

MIVGPU_EXPORT hipError_t hipDeviceSynchronize(void) {
  Guard g;
  if (g.outer && g_ready.load(std::memory_order_acquire)) stamp_before_sync(nullptr, true);
  return real_hipDeviceSynchronize()();
}

// ROCr reads HSA_CU_MASK and ROCR_VISIBLE_DEVICES once, when HIP initialises
// it.  Re-assert the grant in the environment right before that read, so the
// hardware CU mask of every queue the process creates is the granted one even
// if the tenant unset or rewrote the variables (ROCr applies HSA_CU_MASK to
// each queue at creation and ANDs any later hsa_amd_queue_cu_set_mask with it).
MIVGPU_EXPORT int hsa_init(void) {
  using fn_t = int (*)(void);
  static fn_t real = [] {
    void* p = dlvsym(RTLD_NEXT, "hsa_init", "ROCR_1");
    if (!p) p = dlsym(RTLD_NEXT, "hsa_init");
    if (!p) {
      void* h = dlopen("libhsa-runtime64.so.1", RTLD_LAZY | RTLD_GLOBAL | RTLD_NOLOAD);
      if (!h) h = dlopen("libhsa-runtime64.so.1", RTLD_LAZY | RTLD_GLOBAL);
      if (h) p = dlvsym(h, "hsa_init", "ROCR_1");
    }
    return reinterpret_cast<fn_t>(p);
  }();
  ensure_limits();
  if (g_limits.loaded) {
    for (const char* key : {"HSA_CU_MASK", "ROCR_VISIBLE_DEVICES"}) {
      const char* v = grant_env(key);
      const char* cur = getenv(key);
      if (v && (!cur || strcmp(cur, v) != 0)) {
        if (cur) mlog(1, "%s=%s in the environment differs from the grant; using %s", key, cur, v);
        setenv(key, v, 1);
      }
    }
  }
  if (!real) return 0x1000;  // HSA_STATUS_ERROR
  return real();
}

// ======================================================================
// Symbol resolution: dlsym / dlvsym / hipGetProcAddress.
//
// Binding by ELF version covers PLT references only.  A program that looks a
// HIP entry point up at run time -- Triton's launcher (dlopen("libamdhip64.so")
// -> dlsym("hipGetProcAddress") -> hipGetProcAddress("hipModuleLaunchKernel")),
// and with it torch.compile/Inductor; ctypes; anything dlsym'ing hipMalloc --
// would get the runtime's own function and bypass every hook.  The reference's
// AMD design used LD_AUDIT la_symbind64 for exactly this reason
// (docs/develop/amd-vgpu.md:18-22): it sees every binding.  Here the three
// lookup paths are interposed instead, and each returns the shim's hook for a
// hooked HIP name, as an auditor would.
// ======================================================================

namespace {

// ------------------------------------------------- SMI view of the grant --
// amd-smi and rocm-smi inside a vGPU container report the GRANT: the memory
// total of a granted device is its HBM limit and its usage is the
// container's (the reference's one hard-limit artifact is nvidia-smi showing
// the 3000 MiB cap inside the container, README.md:67-74; its AMD support
// gives this up, docs/develop/amd-vgpu.md:156-158).  libamd_smi.so and
// librocm_smi64.so are in-process libraries the CLIs (and `import amdsmi`)
// open with dlopen and resolve with dlsym, which the shim interposes: the
// memory queries below resolve to these wrappers, which call the library
// and clamp.  The device a query names is matched to the grant by PCI
// location -> KFD topology unique_id -> the "GPU-<16 hex>" ids of
// MIVGPU_DEVICE_UUIDS (the grant) or ROCR_VISIBLE_DEVICES.
enum SmiFn {
  SMI_AMD_MEM_TOTAL,
  SMI_AMD_MEM_USAGE,
  SMI_AMD_VRAM_USAGE,
  SMI_AMD_VRAM_INFO,
  SMI_RSMI_MEM_TOTAL,
  SMI_RSMI_MEM_USAGE,
  SMI_COUNT
};
const char* const kSmiNames[SMI_COUNT] = {"amdsmi_get_gpu_memory_total", "amdsmi_get_gpu_memory_usage",
                                          "amdsmi_get_gpu_vram_usage",   "amdsmi_get_gpu_vram_info",
                                          "rsmi_dev_memory_total_get",   "rsmi_dev_memory_usage_get"};
std::atomic<void*> g_smi_real[SMI_COUNT];
std::atomic<void*> g_smi_lib[2];   // the handles the queries were resolved on (amd-smi, rocm-smi)

MIVGPU_NO_SANITIZE int smi_index(const char* name) {
  if (!name || !((name[0] == 'a' && name[1] == 'm' && name[2] == 'd' && name[3] == 's') ||
                 (name[0] == 'r' && name[1] == 's' && name[2] == 'm' && name[3] == 'i')))
    return -1;
  for (int i = 0; i < SMI_COUNT; ++i) {
    const char* a = kSmiNames[i];
    const char* b = name;
    while (*a && *a == *b) ++a, ++b;
    if (*a == *b) return i;
  }
  return -1;
}

// The container-local device index of the GPU at PCI domain:bus:dev.fn, or -1.
int smi_dev_of_bdf(uint64_t domain, uint32_t bus, uint32_t devno, uint32_t fn) {
  const long long want = (long long)((bus << 8) | (devno << 3) | fn);
  uint64_t uid = 0;
  for (int node = 0; node < 256 && !uid; ++node) {
    char path[512];
    snprintf(path, sizeof(path), "%s/topology/nodes/%d/properties", g_cfg.kfd_sysfs, node);
    FILE* f = fopen(path, "re");
    if (!f) {
      if (node > 0) break;
      continue;
    }
    long long loc = -1, dom = -1;
    unsigned long long u = 0;
    char key[96];
    unsigned long long val;
    while (fscanf(f, "%95s %llu", key, &val) == 2) {
      if (!strcmp(key, "location_id")) loc = (long long)val;
      else if (!strcmp(key, "domain")) dom = (long long)val;
      else if (!strcmp(key, "unique_id")) u = val;
    }
    fclose(f);
    if (loc == want && (dom < 0 || (uint64_t)dom == domain)) uid = u;
  }
  if (!uid) return -1;
  // the container's devices, in order: the grant's ids, else the visible ones
  const char* ids = grant_env("MIVGPU_DEVICE_UUIDS");
  if (!ids || !*ids) ids = grant_env("ROCR_VISIBLE_DEVICES");
  if (!ids) return -1;
  int idx = 0;
  for (const char* p = ids; *p; ++idx) {
    const char* e = strchr(p, ',');
    const size_t n = e ? (size_t)(e - p) : strlen(p);
    if (n > 4 && !strncmp(p, "GPU-", 4) && strtoull(p + 4, nullptr, 16) == uid) return idx < MIVGPU_MAX_DEVICES ? idx : -1;
    if (!e) break;
    p = e + 1;
  }
  return -1;
}

// Grant of the device: HBM limit and the container's usage (bytes).  False
// when the device is not the container's or is not limited.
bool smi_grant(int d, uint64_t* limit, uint64_t* used) {
  ensure_init();
  if (d < 0 || d >= MIVGPU_MAX_DEVICES || g_cfg.disabled) return false;
  const uint64_t lim = limit_of(d);
  if (!lim) return false;
  uint64_t u = g_region ? __atomic_load_n(&g_region->dev_used[d], __ATOMIC_RELAXED) : 0;
  u += ctl_excess(d);
  *limit = lim;
  if (used) *used = u < lim ? u : lim;
  return true;
}

bool smi_grant_amd(amdsmi_processor_handle h, uint64_t* limit, uint64_t* used) {
  ensure_init();   // the KFD sysfs root and the grant come from the configuration
  void* lib = g_smi_lib[0].load(std::memory_order_acquire);
  auto bdf_fn = reinterpret_cast<amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_bdf_t*)>(
      libc_dlsym()(lib ? lib : RTLD_DEFAULT, "amdsmi_get_gpu_device_bdf"));
  amdsmi_bdf_t bdf;
  bdf.as_uint = 0;
  if (!bdf_fn || bdf_fn(h, &bdf) != AMDSMI_STATUS_SUCCESS) return false;
  return smi_grant(smi_dev_of_bdf(bdf.domain_number, (uint32_t)bdf.bus_number, (uint32_t)bdf.device_number,
                                  (uint32_t)bdf.function_number), limit, used);
}

bool smi_grant_rsmi(uint32_t dv, uint64_t* limit, uint64_t* used) {
  ensure_init();
  void* lib = g_smi_lib[1].load(std::memory_order_acquire);
  auto pci_fn = reinterpret_cast<int (*)(uint32_t, uint64_t*)>(
      libc_dlsym()(lib ? lib : RTLD_DEFAULT, "rsmi_dev_pci_id_get"));
  uint64_t id = 0;
  if (!pci_fn || pci_fn(dv, &id) != 0) return false;
  return smi_grant(smi_dev_of_bdf(id >> 32, (uint32_t)(id >> 8) & 0xff, (uint32_t)(id >> 3) & 0x1f, (uint32_t)id & 7),
                   limit, used);
}

amdsmi_status_t smi_amd_memory_total(amdsmi_processor_handle h, amdsmi_memory_type_t type, uint64_t* total) {
  auto real = reinterpret_cast<decltype(&smi_amd_memory_total)>(g_smi_real[SMI_AMD_MEM_TOTAL].load());
  if (!real) return AMDSMI_STATUS_NOT_SUPPORTED;
  const amdsmi_status_t rc = real(h, type, total);
  uint64_t lim;
  if (rc == AMDSMI_STATUS_SUCCESS && total && type != AMDSMI_MEM_TYPE_GTT && smi_grant_amd(h, &lim, nullptr) &&
      *total > lim)
    *total = lim;
  return rc;
}

amdsmi_status_t smi_amd_memory_usage(amdsmi_processor_handle h, amdsmi_memory_type_t type, uint64_t* usedp) {
  auto real = reinterpret_cast<decltype(&smi_amd_memory_usage)>(g_smi_real[SMI_AMD_MEM_USAGE].load());
  if (!real) return AMDSMI_STATUS_NOT_SUPPORTED;
  const amdsmi_status_t rc = real(h, type, usedp);
  uint64_t lim, used;
  if (rc == AMDSMI_STATUS_SUCCESS && usedp && type != AMDSMI_MEM_TYPE_GTT && smi_grant_amd(h, &lim, &used))
    *usedp = used;
  return rc;
}

amdsmi_status_t smi_amd_vram_usage(amdsmi_processor_handle h, amdsmi_vram_usage_t* info) {
  auto real = reinterpret_cast<decltype(&smi_amd_vram_usage)>(g_smi_real[SMI_AMD_VRAM_USAGE].load());
  if (!real) return AMDSMI_STATUS_NOT_SUPPORTED;
  const amdsmi_status_t rc = real(h, info);
  uint64_t lim, used;
  if (rc == AMDSMI_STATUS_SUCCESS && info && smi_grant_amd(h, &lim, &used)) {
    info->vram_total = (uint32_t)(lim >> 20);   // MB, as the library reports
    info->vram_used = (uint32_t)(used >> 20);
  }
  return rc;
}

amdsmi_status_t smi_amd_vram_info(amdsmi_processor_handle h, amdsmi_vram_info_t* info) {
  auto real = reinterpret_cast<decltype(&smi_amd_vram_info)>(g_smi_real[SMI_AMD_VRAM_INFO].load());
  if (!real) return AMDSMI_STATUS_NOT_SUPPORTED;
  const amdsmi_status_t rc = real(h, info);
  uint64_t lim;
  if (rc == AMDSMI_STATUS_SUCCESS && info && smi_grant_amd(h, &lim, nullptr) && info->vram_size > (lim >> 20))
    info->vram_size = lim >> 20;
  return rc;
}

int smi_rsmi_memory_total(uint32_t dv, int type, uint64_t* total) {
  auto real = reinterpret_cast<decltype(&smi_rsmi_memory_total)>(g_smi_real[SMI_RSMI_MEM_TOTAL].load());
  if (!real) return 2;   // RSMI_STATUS_NOT_SUPPORTED
  const int rc = real(dv, type, total);
  uint64_t lim;
  if (rc == 0 && total && type != 2 /* GTT */ && smi_grant_rsmi(dv, &lim, nullptr) && *total > lim) *total = lim;
  return rc;
}

int smi_rsmi_memory_usage(uint32_t dv, int type, uint64_t* usedp) {
  auto real = reinterpret_cast<decltype(&smi_rsmi_memory_usage)>(g_smi_real[SMI_RSMI_MEM_USAGE].load());
  if (!real) return 2;
  const int rc = real(dv, type, usedp);
  uint64_t lim, used;
  if (rc == 0 && usedp && type != 2 && smi_grant_rsmi(dv, &lim, &used)) *usedp = used;
  return rc;
}

void* const kSmiHooks[SMI_COUNT] = {
    reinterpret_cast<void*>(&smi_amd_memory_total), reinterpret_cast<void*>(&smi_amd_memory_usage),
    reinterpret_cast<void*>(&smi_amd_vram_usage),   reinterpret_cast<void*>(&smi_amd_vram_info),
    reinterpret_cast<void*>(&smi_rsmi_memory_total), reinterpret_cast<void*>(&smi_rsmi_memory_usage)};

// `r`: the library's own function for SMI query `i`, resolved on `handle`.
void* smi_result(int i, void* handle, void* r) {
  if (!r || r == kSmiHooks[i] || g_cfg.disabled) return r;
  g_smi_real[i].store(r, std::memory_order_release);
  if (handle != RTLD_DEFAULT && handle != RTLD_NEXT)
    g_smi_lib[i >= SMI_RSMI_MEM_TOTAL ? 1 : 0].store(handle, std::memory_order_release);
  return kSmiHooks[i];
}

struct HookEntry {
  const char* name;
  void* hook;
  void* (*real)();
};

#define HOOK(n) {#n, reinterpret_cast<void*>(static_cast<n##_fn>(&::n)), +[]() -> void* { return reinterpret_cast<void*>(real_##n()); }}
const HookEntry kHooks[] = {
    HOOK(hipMalloc), HOOK(hipExtMallocWithFlags), HOOK(hipMallocManaged), HOOK(hipMallocAsync),
    HOOK(hipMallocFromPoolAsync), HOOK(hipMallocPitch), HOOK(hipMemAllocPitch), HOOK(hipMalloc3D),
    HOOK(hipMallocArray), HOOK(hipMalloc3DArray), HOOK(hipArrayCreate), HOOK(hipArray3DCreate),
    HOOK(hipMallocMipmappedArray), HOOK(hipMipmappedArrayCreate), HOOK(hipFreeArray), HOOK(hipArrayDestroy),
    HOOK(hipFreeMipmappedArray), HOOK(hipMipmappedArrayDestroy), HOOK(hipModuleLoad), HOOK(hipModuleLoadData),
    HOOK(hipModuleLoadDataEx), HOOK(hipModuleUnload), HOOK(hipFree), HOOK(hipFreeAsync), HOOK(hipMemCreate),
    HOOK(hipMemRelease), HOOK(hipMemGetInfo), HOOK(hipDeviceTotalMem), HOOK(hipGetDevicePropertiesR0600),
    HOOK(hipGetDevicePropertiesR0000), HOOK(hipLaunchKernel), HOOK(hipLaunchKernel_spt),
    HOOK(hipModuleLaunchKernel), HOOK(hipExtModuleLaunchKernel), HOOK(hipHccModuleLaunchKernel),
    HOOK(hipLaunchCooperativeKernel), HOOK(hipModuleLaunchCooperativeKernel), HOOK(hipExtLaunchKernel),
    HOOK(hipGraphLaunch), HOOK(hipGraphLaunch_spt), HOOK(hipLaunchKernelExC), HOOK(hipDrvLaunchKernelEx),
    HOOK(hipLaunchCooperativeKernelMultiDevice), HOOK(hipExtLaunchMultiKernelMultiDevice),
    HOOK(hipStreamBeginCapture), HOOK(hipStreamBeginCapture_spt), HOOK(hipStreamBeginCaptureToGraph),
    HOOK(hipStreamEndCapture), HOOK(hipStreamEndCapture_spt), HOOK(hipStreamSynchronize),
    HOOK(hipStreamSynchronize_spt), HOOK(hipDeviceSynchronize), HOOK(hipGetProcAddress),
};
#undef HOOK

// (entries are null until this library's initialisers have run: a lookup
// made earlier, from another preloaded library's constructor, passes through)
MIVGPU_NO_SANITIZE const HookEntry* find_hook(const char* name) {
  if (!name || name[0] != 'h' || name[1] != 'i' || name[2] != 'p') return nullptr;
  for (const HookEntry& e : kHooks) {
    if (!e.name) continue;
    const char* a = e.name;
    const char* b = name;
    while (*a && *a == *b) ++a, ++b;
    if (*a == *b) return &e;
  }
  return nullptr;
}

const HookEntry* find_hook_by_real(void* p) {
  if (!p) return nullptr;
  for (const HookEntry& e : kHooks)
    if (e.name && e.real() == p) return &e;
  return nullptr;
}

bool in_hip_runtime(void* p) {
  Dl_info di;
  if (!dladdr(p, &di) || !di.dli_fname) return false;
  const char* slash = strrchr(di.dli_fname, '/');
  return strncmp(slash ? slash + 1 : di.dli_fname, "libamdhip64", 11) == 0;
}

// `r` is what the real lookup returned for hooked name `e`.
void* hooked_result(const HookEntry* e, void* handle, void* r) {
  if (!r || r == e->hook) return r;
  // a HIP runtime opened privately while none is global: the hooks forward to it
  if (handle != RTLD_DEFAULT && handle != RTLD_NEXT && in_hip_runtime(r) &&
      !libc_dlsym()(RTLD_NEXT, "hipMalloc")) {
    void* none = nullptr;
    g_hip_handle.compare_exchange_strong(none, handle, std::memory_order_acq_rel);
  }
  if (r == e->real()) return e->hook;
  static std::atomic<bool> warned{false};
  if (in_hip_runtime(r) && !warned.exchange(true))
    mlog(1, "a second HIP runtime is loaded in this process; its entry points (%s) are not governed", e->name);
  return r;
}

void* dlsym_hooked(void* handle, const char* name) {
  const HookEntry* e = find_hook(name);
  void* r = libc_dlsym()(handle, name);
  if (e) return hooked_result(e, handle, r);
  const int si = smi_index(name);
  return si >= 0 ? smi_result(si, handle, r) : r;
}

void* dlvsym_hooked(void* handle, const char* name, const char* version) {
  const HookEntry* e = find_hook(name);
  void* r = libc_dlvsym()(handle, name, version);
  if (e) return hooked_result(e, handle, r);
  const int si = smi_index(name);
  return si >= 0 ? smi_result(si, handle, r) : r;
}

}  // namespace

// Called from the dlsym / dlvsym entry stubs below with the caller's
// arguments: the address to jump to.  Non-HIP names go straight to libc's
// implementation as a tail jump, so glibc still sees the ORIGINAL caller's
// return address -- RTLD_NEXT keeps its meaning for every other interposer in
// the process (an exec or malloc wrapper resolving its next definition).
extern "C" __attribute__((visibility("hidden"))) MIVGPU_NO_SANITIZE void* mivgpu_dlsym_route(const char* name) {
  return find_hook(name) || smi_index(name) >= 0 ? reinterpret_cast<void*>(&dlsym_hooked)
                                                 : reinterpret_cast<void*>(libc_dlsym());
}
extern "C" __attribute__((visibility("hidden"))) MIVGPU_NO_SANITIZE void* mivgpu_dlvsym_route(const char* name) {
  return find_hook(name) || smi_index(name) >= 0 ? reinterpret_cast<void*>(&dlvsym_hooked)
                                                 : reinterpret_cast<void*>(libc_dlvsym());
}

// x86-64 SysV: save the argument registers, ask the router, restore, jump.
// Exported as dlsym/dlvsym under both glibc versions callers bind to
// (GLIBC_2.34 for current builds, GLIBC_2.2.5 for manylinux wheels such as
// PyTorch's ROCm libraries).
__asm__(
    ".text\n"
    ".p2align 4\n"
    ".globl __mivgpu_dlsym_entry\n"
    ".type __mivgpu_dlsym_entry,@function\n"
    ".globl __mivgpu_dlsym_compat\n"
    ".type __mivgpu_dlsym_compat,@function\n"
    "__mivgpu_dlsym_entry:\n"
    "__mivgpu_dlsym_compat:\n"
    "  push %rdi\n"
    "  push %rsi\n"
    "  sub $8, %rsp\n"
    "  mov %rsi, %rdi\n"
    "  call mivgpu_dlsym_route\n"
    "  add $8, %rsp\n"
    "  pop %rsi\n"
    "  pop %rdi\n"
    "  jmp *%rax\n"
    ".size __mivgpu_dlsym_entry, .-__mivgpu_dlsym_entry\n"
    ".size __mivgpu_dlsym_compat, .-__mivgpu_dlsym_compat\n"
    ".p2align 4\n"
    ".globl __mivgpu_dlvsym_entry\n"
    ".type __mivgpu_dlvsym_entry,@function\n"
    ".globl __mivgpu_dlvsym_compat\n"
    ".type __mivgpu_dlvsym_compat,@function\n"
    "__mivgpu_dlvsym_entry:\n"
    "__mivgpu_dlvsym_compat:\n"
    "  push %rdi\n"
    "  push %rsi\n"
    "  push %rdx\n"
    "  mov %rsi, %rdi\n"
    "  call mivgpu_dlvsym_route\n"
    "  pop %rdx\n"
    "  pop %rsi\n"
    "  pop %rdi\n"
    "  jmp *%rax\n"
    ".size __mivgpu_dlvsym_entry, .-__mivgpu_dlvsym_entry\n"
    ".size __mivgpu_dlvsym_compat, .-__mivgpu_dlvsym_compat\n"
    ".symver __mivgpu_dlsym_entry, dlsym@@GLIBC_2.34\n"
    ".symver __mivgpu_dlsym_compat, dlsym@GLIBC_2.2.5\n"
    ".symver __mivgpu_dlvsym_entry, dlvsym@@GLIBC_2.34\n"
    ".symver __mivgpu_dlvsym_compat, dlvsym@GLIBC_2.2.5\n");

MIVGPU_EXPORT hipError_t hipGetProcAddress(const char* symbol, void** pfn, int hip_version, uint64_t flags,
                                           hipDriverProcAddressQueryResult* status) {
  if (!real_hipGetProcAddress()) return hipErrorNotSupported;
  hipError_t rc = real_hipGetProcAddress()(symbol, pfn, hip_version, flags, status);
  if (rc != hipSuccess || !pfn || !*pfn) return rc;
  // the runtime may hand out the exported function or an internal one, and
  // version-dependent variants of one name (hipGetDeviceProperties ->
  // R0600 / R0000): match the pointer first, then the name
  const HookEntry* e = find_hook_by_real(*pfn);
  if (!e) e = find_hook(symbol);
  if (!e && symbol && !strcmp(symbol, "hipGetDeviceProperties"))
    e = find_hook(hip_version >= 600 ? "hipGetDevicePropertiesR0600" : "hipGetDevicePropertiesR0000");
  if (e) *pfn = e->hook;
  return rc;
}

// Runtime settings that are part of the grant and that the HIP runtime or
// ROCr read from the environment: with a grant file the granted value is what
// they read, whatever the tenant exported (GPU_MAX_HW_QUEUES is read by HIP
// before it initialises ROCr, so the hsa_init re-assert cannot cover it; the
// queue budget is what the per-GPU split count is sized for).
extern char** environ;

namespace {
__attribute__((tls_model("initial-exec"))) thread_local bool t_in_getenv = false;
bool enforced_env_key(const char* name) {
  return !strcmp(name, "GPU_MAX_HW_QUEUES") || !strcmp(name, "HSA_CU_MASK") || !strcmp(name, "ROCR_VISIBLE_DEVICES");
}
}  // namespace

// HIP's runtime does not only call getenv: ROCclr parses its flags
// (GPU_MAX_HW_QUEUES among them) straight out of `environ`.  So the granted
// values are also put INTO the environment -- once when the shim is loaded
// (before main, before any HIP library initialises) -- and setenv / putenv /
// unsetenv / clearenv cannot change them afterwards (a tenant's
// os.environ["GPU_MAX_HW_QUEUES"] = "8" before `import torch`).
namespace {
using setenv_fn = int (*)(const char*, const char*, int);
using unsetenv_fn = int (*)(const char*);
using putenv_fn = int (*)(char*);
using clearenv_fn = int (*)(void);

template <typename F>
F libc_env_fn(const char* name) {
  static_assert(sizeof(F) == sizeof(void*), "function pointer");
  return reinterpret_cast<F>(libc_sym(name));
}

// granted value of an enforced runtime key, or nullptr
const char* granted_env(const char* name, size_t len) {
  if (!name || t_in_getenv) return nullptr;
  char key[64];
  if (len == 0 || len >= sizeof(key)) return nullptr;
  memcpy(key, name, len);
  key[len] = 0;
  if (!enforced_env_key(key)) return nullptr;
  t_in_getenv = true;
  ensure_limits();
  t_in_getenv = false;
  if (!g_limits.loaded) return nullptr;
  for (int i = 0; i < g_limits.n; ++i)
    if (!strcmp(g_limits.keys[i], key)) return g_limits.vals[i];
  return nullptr;
}

void reassert_granted_env() {
  static const setenv_fn real = libc_env_fn<setenv_fn>("setenv");
  if (!real) return;
  for (const char* k : {"GPU_MAX_HW_QUEUES", "HSA_CU_MASK", "ROCR_VISIBLE_DEVICES"}) {
    const char* v = granted_env(k, strlen(k));
    if (v) real(k, v, 1);
  }
}

__attribute__((constructor)) void mivgpu_env_ctor() { reassert_granted_env(); }
}  // namespace

MIVGPU_EXPORT int setenv(const char* name, const char* value, int overwrite) {
  static const setenv_fn real = libc_env_fn<setenv_fn>("setenv");
  if (name && !strchr(name, '=')) {
    if (const char* g = granted_env(name, strlen(name))) return real ? real(name, g, 1) : 0;
  }
  if (!real) {
    errno = ENOSYS;
    return -1;
  }
  return real(name, value, overwrite);
}

MIVGPU_EXPORT int unsetenv(const char* name) {
  static const unsetenv_fn real = libc_env_fn<unsetenv_fn>("unsetenv");
  if (name && granted_env(name, strlen(name))) return 0;   // the grant stays
  if (!real) {
    errno = ENOSYS;
    return -1;
  }
  return real(name);
}

MIVGPU_EXPORT int putenv(char* string) {
  static const putenv_fn real = libc_env_fn<putenv_fn>("putenv");
  if (string) {
    const char* eq = strchr(string, '=');
    const size_t n = eq ? (size_t)(eq - string) : strlen(string);
    if (const char* g = granted_env(string, n)) {
      static const setenv_fn set = libc_env_fn<setenv_fn>("setenv");
      char key[64];
      memcpy(key, string, n);
      key[n] = 0;
      return set ? set(key, g, 1) : 0;
    }
  }
  if (!real) {
    errno = ENOSYS;
    return -1;
  }
  return real(string);
}

MIVGPU_EXPORT int clearenv(void) {
  static const clearenv_fn real = libc_env_fn<clearenv_fn>("clearenv");
  const int rc = real ? real() : -1;
  reassert_granted_env();
  return rc;
}

MIVGPU_EXPORT char* getenv(const char* name) {
  if (!name || !*name || strchr(name, '=')) return nullptr;
  if ((name[0] == 'G' || name[0] == 'H' || name[0] == 'R') && !t_in_getenv && enforced_env_key(name)) {
    t_in_getenv = true;
    ensure_limits();
    t_in_getenv = false;
    if (g_limits.loaded) {
      for (int i = 0; i < g_limits.n; ++i)
        if (!strcmp(g_limits.keys[i], name)) return g_limits.vals[i];
    }
  }
  const size_t n = strlen(name);
  for (char** e = environ; e && *e; ++e)
    if (!strncmp(*e, name, n) && (*e)[n] == '=') return *e + n + 1;
  return nullptr;
}

// ======================================================================
// Introspection ABI (MIVGPU_1.0) used by tests and the Python layer.
// ======================================================================

MIVGPU_EXPORT long mivgpu_abi_offsetof(int field) {
  switch (field) {
    case MIVGPU_F_MAGIC: return offsetof(mivgpu_shared_region_t, magic);
    case MIVGPU_F_LOCK: return offsetof(mivgpu_shared_region_t, lock);
    case MIVGPU_F_NUM_DEVICES: return offsetof(mivgpu_shared_region_t, num_devices);
    case MIVGPU_F_PROCNUM: return offsetof(mivgpu_shared_region_t, procnum);
    case MIVGPU_F_UTIL_SWITCH: return offsetof(mivgpu_shared_region_t, utilization_switch);
    case MIVGPU_F_RECENT_KERNEL: return offsetof(mivgpu_shared_region_t, recent_kernel);
    case MIVGPU_F_PRIORITY: return offsetof(mivgpu_shared_region_t, priority);
    case MIVGPU_F_LAST_KERNEL_TIME: return offsetof(mivgpu_shared_region_t, last_kernel_time);
    case MIVGPU_F_CORE_POLICY: return offsetof(mivgpu_shared_region_t, core_policy);
    case MIVGPU_F_UUIDS: return offsetof(mivgpu_shared_region_t, uuids);
    case MIVGPU_F_MEM_LIMIT: return offsetof(mivgpu_shared_region_t, mem_limit);
    case MIVGPU_F_CU_LIMIT: return offsetof(mivgpu_shared_region_t, cu_limit);
    case MIVGPU_F_CU_MASK_COUNT: return offsetof(mivgpu_shared_region_t, cu_mask_count);
    case MIVGPU_F_DEV_USED: return offsetof(mivgpu_shared_region_t, dev_used);
    case MIVGPU_F_PROCS: return offsetof(mivgpu_shared_region_t, procs);
    case MIVGPU_F_SIZEOF_REGION: return sizeof(mivgpu_shared_region_t);
    case MIVGPU_F_SIZEOF_SLOT: return sizeof(mivgpu_proc_slot_t);
    case MIVGPU_F_SLOT_USED: return offsetof(mivgpu_proc_slot_t, used);
    case MIVGPU_F_SLOT_UTIL: return offsetof(mivgpu_proc_slot_t, util);
    case MIVGPU_F_CTL_SEQ: return offsetof(mivgpu_control_t, seq);
    case MIVGPU_F_CTL_LEASE: return offsetof(mivgpu_control_t, lease_until_ns);
    case MIVGPU_F_CTL_BLOCK: return offsetof(mivgpu_control_t, block);
    case MIVGPU_F_CTL_SWITCH: return offsetof(mivgpu_control_t, utilization_switch);
    case MIVGPU_F_CTL_OVER: return offsetof(mivgpu_control_t, over_grant);
    case MIVGPU_F_CTL_EXCESS: return offsetof(mivgpu_control_t, host_excess);
    case MIVGPU_F_SIZEOF_CTL: return sizeof(mivgpu_control_t);
    case MIVGPU_F_BOARD_SEQ: return offsetof(mivgpu_board_t, seq);
    case MIVGPU_F_BOARD_BEAT: return offsetof(mivgpu_board_t, beat_ns);
    case MIVGPU_F_BOARD_SLOTS: return offsetof(mivgpu_board_t, slots);
    case MIVGPU_F_SIZEOF_BOARD: return sizeof(mivgpu_board_t);
    case MIVGPU_F_SIZEOF_BOARD_SLOT: return sizeof(mivgpu_board_slot_t);
    case MIVGPU_F_FLAGS_ENTRIES: return offsetof(mivgpu_board_flags_t, flags);
    case MIVGPU_F_SIZEOF_FLAGS: return sizeof(mivgpu_board_flags_t);
    default: return -1;
  }
}

MIVGPU_EXPORT int mivgpu_parse_cu_mask_count(const char* mask, int idx) {
  return parse_cu_mask_count(mask, idx);
}

MIVGPU_EXPORT unsigned long long mivgpu_parse_size(const char* s) { return parse_size(s); }
MIVGPU_EXPORT unsigned int mivgpu_parse_pct_ppm(const char* s) { return parse_pct_ppm(s); }
MIVGPU_EXPORT int mivgpu_pct_of_ppm(unsigned int ppm) { return pct_of_ppm(ppm); }

// Usage of this process on `dev` as seen by the shim (bytes); -1 if inactive.
MIVGPU_EXPORT long long mivgpu_process_usage(int dev) {
  ensure_init();
  if (!g_region || g_slot < 0 || dev < 0 || dev >= MIVGPU_MAX_DEVICES) return -1;
  return (long long)__atomic_load_n(&g_region->procs[g_slot].used[dev].total, __ATOMIC_RELAXED);
}

MIVGPU_EXPORT unsigned long long mivgpu_launch_count(void) {
  return g_launches_local.load(std::memory_order_relaxed);
}

// Governor counters for `dev`: GPU time charged, held, gates (ns, ns, count).
// Charged = what the bucket was debited: the sampler's share integral in the
// default host-bucket mode (the gate kernel keeps no busy clock there), the
// gates' measured busy wall time x share in device-bucket mode.
MIVGPU_EXPORT int mivgpu_gate_stats(int dev, unsigned long long* busy, unsigned long long* held,
                                    unsigned long long* gates) {
  if (dev < 0 || dev >= MIVGPU_MAX_DEVICES) return -1;
  DeviceGate& G = g_gates[dev];
  if (!G.ok_pub.load(std::memory_order_acquire) || !G.host_stats) return -1;
  const volatile unsigned long long* h = static_cast<const volatile unsigned long long*>(G.host_stats);
  const bool host_bucket = g_occ_live[dev].load(std::memory_order_acquire) && !g_cfg.gate_device_mode;
  if (busy)
    *busy = host_bucket && g_region && g_slot >= 0
                ? __atomic_load_n(&g_region->procs[g_slot].util[dev].share_ns, __ATOMIC_RELAXED)
                : h[0];
  if (held) *held = h[1];
  if (gates) *gates = h[2];
  return 0;
}

// Host-bucket balance of `dev` (ns of GPU time; negative = in debt) and the
// GPU time received so far (the share integral); -1 when the device has no
// host bucket (no gate yet, or no KFD view).
MIVGPU_EXPORT int mivgpu_gate_balance(int dev, long long* tokens, unsigned long long* received) {
  if (dev < 0 || dev >= MIVGPU_MAX_DEVICES) return -1;
  DeviceGate& G = g_gates[dev];
  const uint64_t* hs = static_cast<const uint64_t*>(G.hs_pub.load(std::memory_order_acquire));
  if (!hs || !g_occ_live[dev].load(std::memory_order_acquire)) return -1;
  if (tokens) *tokens = (long long)__atomic_load_n(&hs[kHsHostTokens], __ATOMIC_RELAXED);
  if (received && g_region && g_slot >= 0)
    *received = __atomic_load_n(&g_region->procs[g_slot].util[dev].share_ns, __ATOMIC_RELAXED);
  return 0;
}

// Sampler diagnostics of `dev`: wall ns spent in each sampling state (own
// waves resident / alone+busy with none resident / held by its own gate /
// only other tenants' waves / idle) and the number of samples.
MIVGPU_EXPORT int mivgpu_occ_states(int dev, double* ns5, unsigned long long* samples) {
  if (dev < 0 || dev >= MIVGPU_MAX_DEVICES || !g_occ_live[dev].load(std::memory_order_acquire)) return -1;
  std::lock_guard<std::mutex> pass(g_occ_pass_mu);
  for (int i = 0; i < 5; ++i) ns5[i] = g_occ[dev].state_ns[i];
  if (samples) *samples = g_occ[dev].samples;
  return 0;
}

// Sampler passes so far, their total and their longest duration (ns).
MIVGPU_EXPORT int mivgpu_occ_timing(unsigned long long* passes, unsigned long long* total_ns,
                                    unsigned long long* max_ns) {
  std::lock_guard<std::mutex> pass(g_occ_pass_mu);
  if (passes) *passes = g_occ_passes;
  if (total_ns) *total_ns = g_occ_pass_ns;
  if (max_ns) *max_ns = g_occ_pass_max_ns;
  return 0;
}

// The sampler's view of `dev` as one JSON object (NUL-terminated, at most n
// bytes; returns the length or -1): the share board (owner role, owner, the
// board's age, every process's integrals), the samples charged from the board
// or the local estimate, the local estimate's peers, the state split.  What a
// failed governor test prints so the record explains itself.
MIVGPU_EXPORT int mivgpu_sampler_info(int dev, char* buf, int n) {
  if (dev < 0 || dev >= MIVGPU_MAX_DEVICES || !buf || n < 64) return -1;
  std::lock_guard<std::mutex> pass(g_occ_pass_mu);
  const OccDev& o = g_occ[dev];
  int len = 0;
  auto put = [&](const char* fmt, ...) __attribute__((format(printf, 2, 3))) {
    if (len >= n - 1) return;
    va_list ap;
    va_start(ap, fmt);
    const int w = vsnprintf(buf + len, (size_t)(n - len), fmt, ap);
    va_end(ap);
    if (w > 0) len = len + w < n - 1 ? len + w : n - 1;
  };
  const uint64_t now = mono_ns();
  put("{\"live\":%d,\"gpu_id\":%d,\"pid\":%d,\"samples\":%llu,\"board_charged\":%llu,\"local_charged\":%llu,"
      "\"window_ms\":%.1f,\"share_avg\":%.4f,\"board_share\":%.4f,\"state_ms\":[%.1f,%.1f,%.1f,%.1f,%.1f],"
      "\"fair_samples\":%llu,\"fair_held_samples\":%llu,\"lead_ms\":%.3f,\"tokens_ms\":%.3f",
      o.live ? 1 : 0, o.gpu_id, o.own_pid, (unsigned long long)o.samples, (unsigned long long)o.board_charged,
      (unsigned long long)o.local_charged, o.window_ns / 1e6, o.share_avg, o.board_share, o.state_ns[0] / 1e6,
      o.state_ns[1] / 1e6, o.state_ns[2] / 1e6, o.state_ns[3] / 1e6, o.state_ns[4] / 1e6,
      (unsigned long long)o.fair_samples, (unsigned long long)o.fair_held_samples,
      o.last_lead_ns >= 0 ? o.last_lead_ns / 1e6 : -1.0, o.tokens_ns / 1e6);
  put(",\"nonfair\":[");
  {
    const uint64_t k = o.nonfair_n < 16 ? o.nonfair_n : 16;
    for (uint64_t i = 0; i < k; ++i) {
      const OccDev::NonFair& nf = o.nonfair[(o.nonfair_n - k + i) % 16];
      put("%s[%.3f,%.3f,%.3f,%.3f,%.3f,%d]", i ? "," : "", nf.t_ns / 1e6, nf.dt_ns / 1e6, nf.share, nf.run_ns / 1e6,
          nf.tokens_ns / 1e6, nf.prev_fair);
    }
  }
  put("],\"peers\":[");
  for (size_t i = 0; i < o.peers.size(); ++i) {
    const OccPeer& p = o.peers[i];
    put("%s{\"pid\":%d,\"v\":%d,\"avg\":%.2f,\"busy_age_ms\":%.1f}", i ? "," : "", p.pid, p.v, p.avg,
        p.busy_ns ? (now - p.busy_ns) / 1e6 : -1.0);
  }
  put("],\"board\":");
  const mivgpu_board_t* b = o.board.b;
  if (!b) {
    put("{\"dir\":\"%s\",\"open\":0}}", g_cfg.board_dir);
    return len;
  }
  put("{\"dir\":\"%s\",\"open\":1,\"writable\":%d,\"owner\":%d,\"owner_kind\":%d,\"owner_pid\":%d,"
      "\"beat_age_ms\":%.2f,\"passes\":%llu,\"sub_passes\":%llu,\"fair_passes\":%llu,\"period_us\":%.0f,"
      "\"busy_ms\":%.1f,\"slots\":[",
      g_cfg.board_dir, o.board.writable ? 1 : 0, o.board.owner ? 1 : 0, b->owner_kind, b->owner_pid,
      b->beat_ns ? ((double)now - (double)b->beat_ns) / 1e6 : -1.0, (unsigned long long)b->passes,
      (unsigned long long)b->sub_passes, (unsigned long long)b->fair_passes, b->period_ns / 1e3, b->busy_ns / 1e6);
  bool first = true;
  for (int k = 0; k < MIVGPU_BOARD_SLOTS; ++k) {
    const mivgpu_board_slot_t& s = b->slots[k];
    if (!s.pid) continue;
    put("%s{\"pid\":%d,\"occ\":%d,\"obs_ms\":%.1f,\"frac_ms\":%.1f,\"recv_ms\":%.1f,\"busy_ms\":%.1f,"
        "\"lead_ms\":%.3f}",
        first ? "" : ",", s.pid, s.occupancy, s.obs_ns / 1e6, s.frac_ns / 1e6, s.recv_ns / 1e6, s.busy_ns / 1e6,
        s.lead_ns >= 0 ? s.lead_ns / 1e6 : -1.0);
    first = false;
  }
  put("]}}");
  return len;
}

// Copy up to `n` most recent gate trace entries (8 x int64 each) into `out`;
// returns the number copied (0 unless MIVGPU_GATE_TRACE=1).
MIVGPU_EXPORT int mivgpu_gate_trace(int dev, long long* out, int n) {
  if (dev < 0 || dev >= MIVGPU_MAX_DEVICES || !out || n <= 0 || !g_cfg.gate_trace) return 0;
  DeviceGate& G = g_gates[dev];
  if (!G.ok_pub.load(std::memory_order_acquire) || !G.host_stats) return 0;
  const volatile long long* h = static_cast<const volatile long long*>(G.host_stats);
  const unsigned long long gates = static_cast<const volatile unsigned long long*>(G.host_stats)[2];
  int cnt = (int)(gates < 128 ? gates : 128);
  if (cnt > n) cnt = n;
  for (int i = 0; i < cnt; ++i) {
    unsigned long long g = gates - cnt + i;
    const volatile long long* e = h + 8 + (g % 128) * 8;
    for (int k = 0; k < 8; ++k) out[i * 8 + k] = e[k];
  }
  return cnt;
}

// How the process is charged: bit 0 device-bucket gate mode, bit 1 instant
// share estimator, bit 2 ratio estimator, bit 3 a grant file is loaded, bit 4
// a control file is mapped; *ctx_refresh_ns the context-VRAM refresh period.
MIVGPU_EXPORT int mivgpu_config_info(unsigned long long* ctx_refresh_ns) {
  ensure_init();
  if (ctx_refresh_ns) *ctx_refresh_ns = g_cfg.context_refresh_ns;
  return (g_cfg.gate_device_mode ? 1 : 0) | (g_cfg.share_instant ? 2 : 0) | (g_cfg.share_ratio ? 4 : 0) |
         (g_limits.loaded ? 8 : 0) | (g_ctl ? 16 : 0);
}

MIVGPU_EXPORT int mivgpu_active(void) {
  ensure_init();
  return g_region != nullptr && !g_cfg.disabled;
}
