// mivgpu-boardd -- the node's share-board owner: ONE wave-occupancy sampler
// per GPU for every tenant on it (board.h, ABI in mivgpu/shared_region.h).
//
// Started by the node monitor (cmd/monitor.py, hostPID, KFD sysfs of the
// host) on the host board directory that the device plugin mounts READ-ONLY
// into every vGPU container (deviceplugin/allocate.py): tenants read the
// shares they are charged and cannot write them.  Reference role: the
// utilisation sampling HAMi-core serialises through /tmp/vgpulock
// (pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:853-864).
//
//   mivgpu-boardd --dir DIR [--kfd-sysfs /sys/class/kfd/kfd] [--period-us 2000]
//                 [--idle-period-us 20000] [--dormant-period-us 50000]
//                 [--presence-window-us 20000] [--passes N] [--exit-with-parent]
//
// Every pass reads <kfd>/proc/<pid>/stats_<gpu_id>/cu_occupancy of every KFD
// process (~7 us per read on MI355X) and writes each GPU's board; the process
// list is re-scanned every 100 ms.  Fast passes while a tenant is governed
// (GATED flags within the last second) and waves were resident within the
// last second, idle passes while one is governed but the GPU is idle, and
// dormant (50 ms) passes while no tenant is governed (CU-masked tenants only).
// Tenant files are read with pread, never mapped, created or followed
// through a symlink; a pid's flags come only from the directory
// of the container the monitor attributes it to (<dir>/gpu-<id>.owners).
#include <dirent.h>
#include <signal.h>
#include <stdlib.h>
#include <sys/prctl.h>
#include <time.h>

#include <map>
#include <utility>
#include <vector>

#include "board.h"

namespace {

volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

int read_occ(int fd) {
  char buf[32];
  ssize_t n = pread(fd, buf, sizeof(buf) - 1, 0);
  if (n <= 0) return -1;
  buf[n] = 0;
  return atoi(buf);
}

std::vector<int> gpu_ids(const char* kfd) {
  std::vector<int> out;
  char dir[512];
  snprintf(dir, sizeof(dir), "%s/topology/nodes", kfd);
  DIR* d = opendir(dir);
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    char path[800];
    snprintf(path, sizeof(path), "%s/%s/gpu_id", dir, e->d_name);
    FILE* f = fopen(path, "r");
    if (!f) continue;
    int gid = 0;
    if (fscanf(f, "%d", &gid) == 1 && gid > 0) out.push_back(gid);
    fclose(f);
  }
  closedir(d);
  return out;
}

struct Gpu {
  int gpu_id;
  mivgpu_board::Handle h;
  std::map<int, int> fds;   // pid -> cu_occupancy fd
  std::vector<mivgpu_board::Reading> rd;
};

void rescan(const char* kfd, std::vector<Gpu>& gpus) {
  char dir[512];
  snprintf(dir, sizeof(dir), "%s/proc", kfd);
  std::vector<int> pids;
  if (DIR* d = opendir(dir)) {
    while (dirent* e = readdir(d)) {
      char* end = nullptr;
      long pid = strtol(e->d_name, &end, 10);
      if (end != e->d_name && !*end && pid > 0) pids.push_back((int)pid);
    }
    closedir(d);
  }
  for (Gpu& g : gpus) {
    std::map<int, int> next;
    for (int pid : pids) {
      auto it = g.fds.find(pid);
      if (it != g.fds.end()) {
        next.emplace(pid, it->second);
        g.fds.erase(it);
        continue;
      }
      char path[600];
      snprintf(path, sizeof(path), "%s/proc/%d/stats_%d/cu_occupancy", kfd, pid, g.gpu_id);
      int fd = open(path, O_RDONLY | O_CLOEXEC);   // no stats_<gpu_id>: not on this GPU
      if (fd >= 0) next.emplace(pid, fd);
    }
    for (auto& kv : g.fds) close(kv.second);
    g.fds.swap(next);
  }
}

}  // namespace

int main(int argc, char** argv) {
  const char* dir = nullptr;
  const char* kfd = "/sys/class/kfd/kfd";
  uint64_t period_ns = 2000000, idle_ns = 20000000, dormant_ns = 50000000, max_passes = 0;
  uint64_t presence_ns = mivgpu_board::kPresenceNs;
  int split = mivgpu_board::kSplitRatio;
  for (int i = 1; i < argc; ++i) {
    const char* a = argv[i];
    const char* v = i + 1 < argc ? argv[i + 1] : nullptr;
    if (!strcmp(a, "--dir") && v) { dir = v; ++i; }
    else if (!strcmp(a, "--kfd-sysfs") && v) { kfd = v; ++i; }
    else if (!strcmp(a, "--period-us") && v) { period_ns = strtoull(v, nullptr, 10) * 1000ull; ++i; }
    else if (!strcmp(a, "--idle-period-us") && v) { idle_ns = strtoull(v, nullptr, 10) * 1000ull; ++i; }
    else if (!strcmp(a, "--dormant-period-us") && v) { dormant_ns = strtoull(v, nullptr, 10) * 1000ull; ++i; }
    else if (!strcmp(a, "--passes") && v) { max_passes = strtoull(v, nullptr, 10); ++i; }
    else if (!strcmp(a, "--presence-window-us") && v) { presence_ns = strtoull(v, nullptr, 10) * 1000ull; ++i; }
    else if (!strcmp(a, "--split") && v) { split = !strcmp(v, "equal") ? mivgpu_board::kSplitEqual : split; ++i; }
    else if (!strcmp(a, "--exit-with-parent")) { prctl(PR_SET_PDEATHSIG, SIGTERM); }
    else {
      fprintf(stderr, "usage: %s --dir DIR [--kfd-sysfs PATH] [--period-us N] [--idle-period-us N] [--dormant-period-us N] [--presence-window-us N] [--passes N] "
              "[--split ratio|equal] [--exit-with-parent]\n", argv[0]);
      return 2;
    }
  }
  if (!dir) {
    fprintf(stderr, "mivgpu-boardd: --dir is required\n");
    return 2;
  }
  if (period_ns < 200000) period_ns = 200000;
  if (idle_ns < period_ns) idle_ns = period_ns;
  if (dormant_ns < idle_ns) dormant_ns = idle_ns;
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);
  std::vector<Gpu> gpus;
  for (int gid : gpu_ids(kfd)) {
    Gpu g;
    g.gpu_id = gid;
    if (!mivgpu_board::open_board(g.h, dir, gid, true) || !g.h.writable) {
      fprintf(stderr, "mivgpu-boardd: cannot map a writable board for KFD gpu %d in %s\n", gid, dir);
      continue;
    }
    g.h.owner = true;   // the node sampler owns unconditionally; shims yield to a live one
    g.h.node = true;    // tenant files: read only, never created, never through a symlink
    g.h.presence_ns = presence_ns;
    gpus.push_back(std::move(g));
  }
  if (gpus.empty()) {
    fprintf(stderr, "mivgpu-boardd: no GPU in %s/topology\n", kfd);
    return 1;
  }
  fprintf(stderr, "mivgpu-boardd: %zu GPU board(s) in %s, period %llu us\n", gpus.size(), dir,
          (unsigned long long)(period_ns / 1000));
  const int self = (int)getpid();
  uint64_t list_ns = 0, wave_ns = 0, passes = 0;
  while (!g_stop) {
    const uint64_t now = mono_ns();
    if (now - list_ns >= 100000000ull) {
      list_ns = now;
      rescan(kfd, gpus);
    }
    // fast passes only while a governed tenant asks for them (GATED flags
    // within the last second) and waves are resident; dormant without one:
    // CU-masked tenants are never charged from the board
    bool demand = false;
    for (const Gpu& g : gpus) demand |= g.h.demand_ns && now - g.h.demand_ns < 1000000000ull;
    const bool fast = demand && wave_ns && now - wave_ns < 1000000000ull;
    const uint64_t wait_ns = fast ? period_ns : (demand ? idle_ns : dormant_ns);
    for (Gpu& g : gpus) {
      const uint64_t t0 = mono_ns();
      g.rd.clear();
      for (auto& kv : g.fds) {
        const int v = read_occ(kv.second);
        g.rd.push_back(mivgpu_board::Reading{kv.first, v});
        if (v > mivgpu_board::kGateUnits) wave_ns = t0;
      }
      mivgpu_board::owner_pass(g.h, g.rd.data(), (int)g.rd.size(), t0, wait_ns, MIVGPU_BOARD_OWNER_NODE, self,
                               split, mono_ns() - t0);
    }
    if (max_passes && ++passes >= max_passes) break;
    const uint64_t sleep_ns = wait_ns;
    timespec ts{(time_t)(sleep_ns / 1000000000ull), (long)(sleep_ns % 1000000000ull)};
    nanosleep(&ts, nullptr);
  }
  for (Gpu& g : gpus) __atomic_store_n(&g.h.b->owner_kind, (int32_t)MIVGPU_BOARD_OWNER_NONE, __ATOMIC_RELEASE);
  return 0;
}
