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
// Prints one JSON line.
//
//   launch_bench [N=100000] [graph_replays=2000]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

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
  CHECK(hipHostFree(flag));
  const double host_launch_ns = host_ns / (double)(rounds * chunk);

  if (getenv("LAUNCH_BENCH_NO_GRAPH")) {
    CHECK(hipStreamDestroy(s));
    printf("{\"launches\": %ld, \"launch_ns\": %.1f, \"launch_drain_ns\": %.1f, \"host_launch_ns\": %.1f}\n", n,
           (t1 - t0) / n, (t2 - t0) / n, host_launch_ns);
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
         "\"graph_replays\": %ld, \"graph_launch_ns\": %.1f, \"graph_drain_ns\": %.1f}\n",
         n, (t1 - t0) / n, (t2 - t0) / n, host_launch_ns, replays, (g1 - g0) / replays, (g2 - g0) / replays);
  return 0;
}
