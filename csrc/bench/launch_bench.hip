// Per-launch cost of the interposition layer (VERDICT r1 "per-launch hook cost").
//
// Launches an empty one-wave kernel N times through hipLaunchKernel (the
// <<<>>> stub), on one stream, and reports host ns per launch for the launch
// loop alone and for loop + drain.  Run natively, under libmivgpu.so with
// the governor off, and with it on: the difference is what the shim adds to
// a launch-bound eager workload.  Also times hipGraphLaunch of a captured
// graph of 32 empty kernels (replay path).  host_launch_ns: the same launches
// queued behind a held stream in rounds of 512 -- the host's enqueue cost
// alone (launch_ns is paced by the GPU's empty-kernel dispatch, ~2.9 us).
// hook_ns: the interposition's own cost, in one process -- hipLaunchKernel
// called through the dynamic symbol (the shim's hook when it is preloaded)
// against the runtime's own entry point (read from libamdhip64's .dynsym:
// dlsym would return the hook, by design), in alternating rounds behind a
// held stream; the median per-round difference (0 without the shim).
// Process-to-process variation of the runtime's ~2.5 us enqueue is +-200 ns,
// so comparing separate native and shim runs cannot resolve tens of ns.
// Prints one JSON line.
//
//   launch_bench [N=100000] [graph_replays=2000]
#include <dlfcn.h>
#include <elf.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <link.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef hipError_t (*launch_fn)(const void*, dim3, dim3, void**, size_t, hipStream_t);

// Address of `name` as defined by the loaded HIP runtime (its .dynsym, read
// from the file), bypassing every interposer; nullptr if not found.
static void* runtime_symbol(const char* name) {
  struct Ctx {
    uintptr_t base;
    char path[1024];
  } ctx{0, {0}};
  dl_iterate_phdr(
      [](dl_phdr_info* info, size_t, void* p) -> int {
        Ctx* c = static_cast<Ctx*>(p);
        if (info->dlpi_name && strstr(info->dlpi_name, "libamdhip64")) {
          c->base = info->dlpi_addr;
          strncpy(c->path, info->dlpi_name, sizeof(c->path) - 1);
          return 1;
        }
        return 0;
      },
      &ctx);
  if (!ctx.path[0]) return nullptr;
  const int fd = open(ctx.path, O_RDONLY);
  if (fd < 0) return nullptr;
  struct stat st;
  void* map = fstat(fd, &st) == 0 ? mmap(nullptr, st.st_size, PROT_READ, MAP_PRIVATE, fd, 0) : MAP_FAILED;
  close(fd);
  if (map == MAP_FAILED) return nullptr;
  void* out = nullptr;
  const char* b = static_cast<const char*>(map);
  const Elf64_Ehdr* eh = reinterpret_cast<const Elf64_Ehdr*>(b);
  const Elf64_Shdr* sh = reinterpret_cast<const Elf64_Shdr*>(b + eh->e_shoff);
  for (int i = 0; i < eh->e_shnum && !out; ++i) {
    if (sh[i].sh_type != SHT_DYNSYM) continue;
    const Elf64_Sym* sym = reinterpret_cast<const Elf64_Sym*>(b + sh[i].sh_offset);
    const char* str = b + sh[sh[i].sh_link].sh_offset;
    for (size_t k = 0; k < sh[i].sh_size / sizeof(Elf64_Sym); ++k)
      if (sym[k].st_shndx != SHN_UNDEF && sym[k].st_value && strcmp(str + sym[k].st_name, name) == 0) {
        out = reinterpret_cast<void*>(ctx.base + sym[k].st_value);
        break;
      }
  }
  munmap(map, st.st_size);
  return out;
}

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));          \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__global__ void __launch_bounds__(64) empty_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) *p = 1;  // never taken
}

// Holds the stream until the host raises *flag (or ~2 s pass: every wave
// exits on its own), so the launches queued behind it measure the host's
// enqueue cost alone -- no dispatch of the GPU paces the loop.
__global__ void __launch_bounds__(64) hold_until(int* flag) {
  if (threadIdx.x != 0) return;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
         (long long)__builtin_amdgcn_s_memrealtime() - t0 < 200000000ll)
    __builtin_amdgcn_s_sleep(32);
}

static double now_ns() {
  return (double)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 100000;
  const long replays = argc > 2 ? atol(argv[2]) : 2000;
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // warm up: code object load, queue creation, shim bootstrap
  for (int i = 0; i < 1000; ++i) empty_kernel<<<1, 64, 0, s>>>(nullptr);
  CHECK(hipStreamSynchronize(s));

  double t0 = now_ns();
  for (long i = 0; i < n; ++i) empty_kernel<<<1, 64, 0, s>>>(nullptr);
  double t1 = now_ns();
  CHECK(hipStreamSynchronize(s));
  double t2 = now_ns();
  CHECK(hipGetLastError());

  // Host-bound: rounds of `chunk` launches queued behind a held stream (far
  // below the queue's capacity, so no launch waits for a slot).
  const long chunk = 512, rounds = n / chunk > 0 ? (n / chunk < 200 ? n / chunk : 200) : 1;
  int* flag = nullptr;
  CHECK(hipHostMalloc((void**)&flag, sizeof(int), hipHostMallocCoherent | hipHostMallocMapped));
  double host_ns = 0;
  for (long r = 0; r < rounds; ++r) {
    __atomic_store_n(flag, 0, __ATOMIC_RELEASE);
    hold_until<<<1, 64, 0, s>>>(flag);
    double h0 = now_ns();
    for (long i = 0; i < chunk; ++i) empty_kernel<<<1, 64, 0, s>>>(nullptr);
    host_ns += now_ns() - h0;
    __atomic_store_n(flag, 1, __ATOMIC_RELEASE);
    CHECK(hipStreamSynchronize(s));
  }
  const double host_launch_ns = host_ns / (double)(rounds * chunk);

  // In-process A/B of the hook: rounds of `half` launches through the symbol
  // and `half` through the runtime's own entry, in alternating order, behind
  // one hold each round.
  const launch_fn direct = reinterpret_cast<launch_fn>(runtime_symbol("hipLaunchKernel"));
  double hook_ns = -1, plt_ns = -1, direct_ns = -1, hook_p25 = -1, hook_p75 = -1;
  if (direct) {
    int* nullp = nullptr;
    void* kargs[] = {&nullp};
    const void* fn = reinterpret_cast<const void*>(empty_kernel);
    // ABBA legs of `leg` launches per round behind one hold: a per-round
    // difference free of slow drifts (clock, queue depth); median of 400
    const long leg = 64, ab_rounds = 400;
    std::vector<double> diff;
    double sum_a = 0, sum_b = 0;
    for (long r = 0; r < ab_rounds; ++r) {
      __atomic_store_n(flag, 0, __ATOMIC_RELEASE);
      hold_until<<<1, 64, 0, s>>>(flag);
      double ta = 0, tb = 0;
      for (int l = 0; l < 4; ++l) {
        const bool via_sym = (l == 0 || l == 3) == (r % 2 == 0);
        const double h0 = now_ns();
        if (via_sym)
          for (long i = 0; i < leg; ++i) hipLaunchKernel(fn, dim3(1), dim3(64), kargs, 0, s);
        else
          for (long i = 0; i < leg; ++i) direct(fn, dim3(1), dim3(64), kargs, 0, s);
        (via_sym ? ta : tb) += (now_ns() - h0) / (double)(2 * leg);
      }
      __atomic_store_n(flag, 1, __ATOMIC_RELEASE);
      CHECK(hipStreamSynchronize(s));
      CHECK(hipGetLastError());
      diff.push_back(ta - tb);
      sum_a += ta;
      sum_b += tb;
    }
    std::sort(diff.begin(), diff.end());
    hook_ns = diff[diff.size() / 2];
    hook_p25 = diff[diff.size() / 4];
    hook_p75 = diff[3 * diff.size() / 4];
    plt_ns = sum_a / (double)ab_rounds;
    direct_ns = sum_b / (double)ab_rounds;
  }
  CHECK(hipHostFree(flag));

  if (getenv("LAUNCH_BENCH_NO_GRAPH")) {
    CHECK(hipStreamDestroy(s));
    printf("{\"launches\": %ld, \"launch_ns\": %.1f, \"launch_drain_ns\": %.1f, \"host_launch_ns\": %.1f, "
           "\"hook_ns\": %.1f, \"hook_p25_ns\": %.1f, \"hook_p75_ns\": %.1f, \"symbol_launch_ns\": %.1f, "
           "\"direct_launch_ns\": %.1f}\n",
           n, (t1 - t0) / n, (t2 - t0) / n, host_launch_ns, hook_ns, hook_p25, hook_p75, plt_ns, direct_ns);
    return 0;
  }
  // graph replay: 32 empty kernels per graph
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < 32; ++i) empty_kernel<<<1, 64, 0, s>>>(nullptr);
  CHECK(hipStreamEndCapture(s, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 50; ++i) CHECK(hipGraphLaunch(ge, s));
  CHECK(hipStreamSynchronize(s));
  double g0 = now_ns();
  for (long i = 0; i < replays; ++i) CHECK(hipGraphLaunch(ge, s));
  double g1 = now_ns();
  CHECK(hipStreamSynchronize(s));
  double g2 = now_ns();
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  CHECK(hipStreamDestroy(s));
  printf("{\"launches\": %ld, \"launch_ns\": %.1f, \"launch_drain_ns\": %.1f, \"host_launch_ns\": %.1f, "
         "\"hook_ns\": %.1f, \"hook_p25_ns\": %.1f, \"hook_p75_ns\": %.1f, \"symbol_launch_ns\": %.1f, "
         "\"direct_launch_ns\": %.1f, \"graph_replays\": %ld, \"graph_launch_ns\": %.1f, \"graph_drain_ns\": %.1f}\n",
         n, (t1 - t0) / n, (t2 - t0) / n, host_launch_ns, hook_ns, hook_p25, hook_p75, plt_ns, direct_ns, replays,
         (g1 - g0) / replays, (g2 - g0) / replays);
  return 0;
}
