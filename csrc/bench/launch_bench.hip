// Per-launch cost of the interposition layer (VERDICT r1 "per-launch hook cost").
//
// Launches an empty one-wave kernel N times through hipLaunchKernel (the
// <<<>>> stub), on one stream, and reports host ns per launch for the launch
// loop alone and for loop + drain.  Run natively, under libmivgpu.so with
// the governor off, and with it on: the difference is what the shim adds to
// a launch-bound eager workload.  Also times hipGraphLaunch of a captured
// graph of 32 empty kernels (replay path).  Prints one JSON line.
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

  if (getenv("LAUNCH_BENCH_NO_GRAPH")) {
    CHECK(hipStreamDestroy(s));
    printf("{\"launches\": %ld, \"launch_ns\": %.1f, \"launch_drain_ns\": %.1f}\n", n, (t1 - t0) / n,
           (t2 - t0) / n);
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
  printf("{\"launches\": %ld, \"launch_ns\": %.1f, \"launch_drain_ns\": %.1f, \"graph_replays\": %ld, "
         "\"graph_launch_ns\": %.1f, \"graph_drain_ns\": %.1f}\n",
         n, (t1 - t0) / n, (t2 - t0) / n, replays, (g1 - g0) / replays, (g2 - g0) / replays);
  return 0;
}
