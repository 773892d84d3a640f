// mivgpu-rccl-check -- RCCL collective validator over xGMI, native (one
// process per GPU): the data plane a multi-GPU pod placed by the topology
// score runs on (the reference's counterpart is the NCCL
// data path its vGPU layer must not break, examples/nvidia/vllm_cross_vgpu.yaml:
// 99-102).  For each message size and collective it checks every element of
// the result exactly and times back-to-back calls on one HIP stream:
//   all_reduce (sum)   busBW = algBW x 2(n-1)/n
//   all_gather         busBW = algBW x (n-1)/n   (algBW over the gathered bytes)
//   reduce_scatter     busBW = algBW x (n-1)/n   (algBW over the input bytes)
//
//   mivgpu-rccl-check --rank R --nranks N --uid FILE [--device D]
//                     [--sizes 1048576,16777216,268435456] [--iters 20] [--warmup 5]
//
// Rank 0 creates the communicator id and publishes it in FILE (written under
// a private name, renamed into place); the other ranks wait for it (60 s).
// One JSON line per (collective, size) on stdout; exit status 0 only when
// every check passed.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <vector>

namespace {

#define HIPCHECK(x)                                                                      \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "mivgpu-rccl-check: %s: %s\n", #x, hipGetErrorString(e_));         \
      exit(3);                                                                           \
    }                                                                                    \
  } while (0)
#define NCCLCHECK(x)                                                                     \
  do {                                                                                   \
    ncclResult_t r_ = (x);                                                               \
    if (r_ != ncclSuccess) {                                                             \
      fprintf(stderr, "mivgpu-rccl-check: %s: %s\n", #x, ncclGetErrorString(r_));        \
      exit(4);                                                                           \
    }                                                                                    \
  } while (0)

// x[i] = rank + 1 + (i % 7): every all-reduce element is exact in fp32
__global__ void fill_kernel(float* x, size_t n, int rank) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    x[i] = (float)(rank + 1 + (int)(i % 7));
}

// counts the elements that differ from the expected value of `op`
__global__ void check_kernel(const float* y, size_t n, int nranks, int rank, int op, unsigned long long* bad) {
  unsigned long long local = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float want;
    if (op == 0) {            // all_reduce: sum over ranks of (r + 1 + i%7)
      want = (float)(nranks * (nranks + 1) / 2 + nranks * (int)(i % 7));
    } else if (op == 1) {     // all_gather: block j holds rank j's input
      const size_t per = n / (size_t)nranks;
      const int j = (int)(i / per);
      want = (float)(j + 1 + (int)((i % per) % 7));
    } else {                  // reduce_scatter: this rank's block of the sum
      const size_t gi = (size_t)rank * n + i;
      want = (float)(nranks * (nranks + 1) / 2 + nranks * (int)(gi % 7));
    }
    if (y[i] != want) ++local;
  }
  if (local) atomicAdd(bad, local);
}

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

bool publish_uid(const char* path, const ncclUniqueId& id) {
  std::string tmp = std::string(path) + ".tmp." + std::to_string(getpid());
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return false;
  const bool ok = fwrite(&id, sizeof(id), 1, f) == 1;
  fclose(f);
  return ok && rename(tmp.c_str(), path) == 0;
}

bool read_uid(const char* path, ncclUniqueId* id, double timeout_s) {
  const double t0 = now_s();
  while (now_s() - t0 < timeout_s) {
    FILE* f = fopen(path, "rb");
    if (f) {
      const bool ok = fread(id, sizeof(*id), 1, f) == 1;
      fclose(f);
      if (ok) return true;
    }
    usleep(20000);
  }
  return false;
}

}  // namespace

int main(int argc, char** argv) {
  int rank = -1, nranks = -1, device = -1, iters = 20, warmup = 5;
  const char* uid_path = nullptr;
  std::vector<size_t> sizes = {1u << 20, 16u << 20, 256u << 20};
  for (int i = 1; i + 1 < argc; i += 2) {
    const char* a = argv[i];
    const char* v = argv[i + 1];
    if (!strcmp(a, "--rank")) rank = atoi(v);
    else if (!strcmp(a, "--nranks")) nranks = atoi(v);
    else if (!strcmp(a, "--device")) device = atoi(v);
    else if (!strcmp(a, "--uid")) uid_path = v;
    else if (!strcmp(a, "--iters")) iters = atoi(v);
    else if (!strcmp(a, "--warmup")) warmup = atoi(v);
    else if (!strcmp(a, "--sizes")) {
      sizes.clear();
      for (const char* p = v; *p;) {
        char* end = nullptr;
        sizes.push_back(strtoull(p, &end, 10));
        p = *end == ',' ? end + 1 : end;
        if (end == p && *p) break;
      }
    }
  }
  if (rank < 0 || nranks < 1 || rank >= nranks || !uid_path || iters < 1) {
    fprintf(stderr, "usage: %s --rank R --nranks N --uid FILE [--device D] [--sizes a,b,c] [--iters K] [--warmup W]\n",
            argv[0]);
    return 2;
  }
  HIPCHECK(hipSetDevice(device >= 0 ? device : 0));
  ncclUniqueId id;
  if (rank == 0) {
    NCCLCHECK(ncclGetUniqueId(&id));
    if (!publish_uid(uid_path, id)) {
      fprintf(stderr, "mivgpu-rccl-check: cannot write %s\n", uid_path);
      return 5;
    }
  } else if (!read_uid(uid_path, &id, 60.0)) {
    fprintf(stderr, "mivgpu-rccl-check: no communicator id in %s after 60 s\n", uid_path);
    return 5;
  }
  ncclComm_t comm;
  NCCLCHECK(ncclCommInitRank(&comm, nranks, id, rank));
  {
    // what RCCL saw: its rank count and this rank's device, by PCI location
    int count = -1, urank = -1, dev = -1;
    NCCLCHECK(ncclCommCount(comm, &count));
    NCCLCHECK(ncclCommUserRank(comm, &urank));
    NCCLCHECK(ncclCommCuDevice(comm, &dev));
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) snprintf(bus, sizeof(bus), "?");
    char ver[32] = {0};
    int v = 0;
    if (ncclGetVersion(&v) == ncclSuccess) snprintf(ver, sizeof(ver), "%d", v);
    printf("{\"comm\":{\"rank\":%d,\"nranks\":%d,\"device\":%d,\"pci_bus_id\":\"%s\",\"rccl_version\":\"%s\"}}\n",
           urank, count, dev, bus, ver);
  }
  hipStream_t s;
  HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned long long* bad_d;
  HIPCHECK(hipMalloc(&bad_d, sizeof(unsigned long long)));
  int failures = 0;
  const char* names[3] = {"all_reduce", "all_gather", "reduce_scatter"};
  for (size_t bytes : sizes) {
    // element count divisible by the rank count (the gathered / scattered blocks)
    const size_t n = (bytes / sizeof(float)) / (size_t)nranks * (size_t)nranks;
    if (n == 0) continue;
    float *x, *y;
    HIPCHECK(hipMalloc(&x, n * sizeof(float)));
    HIPCHECK(hipMalloc(&y, n * sizeof(float)));
    for (int op = 0; op < 3; ++op) {
      const size_t in_n = op == 1 ? n / nranks : n;     // all_gather sends one block
      const size_t out_n = op == 2 ? n / nranks : n;    // reduce_scatter receives one block
      hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, s, x, in_n, rank);
      auto run = [&]() {
        if (op == 0) NCCLCHECK(ncclAllReduce(x, y, n, ncclFloat32, ncclSum, comm, s));
        else if (op == 1) NCCLCHECK(ncclAllGather(x, y, in_n, ncclFloat32, comm, s));
        else NCCLCHECK(ncclReduceScatter(x, y, out_n, ncclFloat32, ncclSum, comm, s));
      };
      for (int w = 0; w < warmup; ++w) run();
      HIPCHECK(hipStreamSynchronize(s));
      const double t0 = now_s();
      for (int it = 0; it < iters; ++it) run();
      HIPCHECK(hipStreamSynchronize(s));
      const double dt = (now_s() - t0) / iters;
      HIPCHECK(hipMemsetAsync(bad_d, 0, sizeof(unsigned long long), s));
      hipLaunchKernelGGL(check_kernel, dim3(1024), dim3(256), 0, s, y, out_n, nranks, rank, op, bad_d);
      unsigned long long bad = 0;
      HIPCHECK(hipMemcpyAsync(&bad, bad_d, sizeof(bad), hipMemcpyDeviceToHost, s));
      HIPCHECK(hipStreamSynchronize(s));
      const double algbw = (double)n * sizeof(float) / dt / 1e9;
      const double factor = op == 0 ? 2.0 * (nranks - 1) / nranks : (double)(nranks - 1) / nranks;
      failures += bad != 0;
      printf("{\"op\":\"%s\",\"rank\":%d,\"nranks\":%d,\"bytes\":%zu,\"ms\":%.4f,\"algbw_gbs\":%.2f,"
             "\"busbw_gbs\":%.2f,\"bad_elements\":%llu,\"ok\":%s}\n",
             names[op], rank, nranks, n * sizeof(float), dt * 1e3, algbw, algbw * factor, bad,
             bad ? "false" : "true");
      fflush(stdout);
    }
    HIPCHECK(hipFree(x));
    HIPCHECK(hipFree(y));
  }
  HIPCHECK(hipFree(bad_d));
  NCCLCHECK(ncclCommDestroy(comm));
  HIPCHECK(hipStreamDestroy(s));
  if (rank == 0) unlink(uid_path);
  return failures ? 1 : 0;
}
