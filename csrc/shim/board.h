// Share board: one wave-occupancy sampler per GPU (ABI in mivgpu/shared_region.h).
//
// Shared by the shim (libmivgpu.so: a tenant reads its share from the board
// and, on a writable board with no live node sampler, may hold the owner
// role) and the node sampler (mivgpu-boardd, started by the monitor).
//
// Reference behaviour replaced: HAMi-core serialises utilisation sampling of
// all containers on a node through the host lock directory /tmp/vgpulock
// (pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:853-864) so one
// process samples NVML for everyone.  Here the owner reads every KFD process's
// cu_occupancy on a GPU in the same pass (~7 us per read on MI355X) and
// integrates each one's share, so the shares every tenant is charged come from
// the same instants and sum to the GPU's busy time.
#ifndef MIVGPU_BOARD_H
#define MIVGPU_BOARD_H

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "mivgpu/shared_region.h"

namespace mivgpu_board {

// A process with at most this many CU units of waves resident is taken to sit
// in its governor gate (governor.hip: one 64-lane wave per held stream; KFD
// rounds waves up to whole CUs, so up to 32 held streams read as 1) or to run
// kernels too small to matter: not contending.
constexpr int kGateUnits = 1;
// A slot whose pid has not been listed for this long is freed.
constexpr uint64_t kSlotStaleNs = 1000000000ull;
// Passes longer apart than this do not invent history (a stalled owner).
constexpr uint64_t kMaxDtNs = 100000000ull;
// Fair-share mode (shared_region.h vt_ns / lead_ns): a process counts as
// backlogged while it was backlogged in at least half of the passes of the
// last ~10 ms (EWMA), so that one tenant's host gap does not break the
// subscription of eight; the mode is entered when the GPU has been fully
// subscribed -- those processes' core limits adding up to the whole GPU -- in
// most passes of the last ~10 ms (EWMA >= 0.8), left below 0.5.
constexpr uint64_t kSubTauNs = 10000000ull;
constexpr double kSubEnter = 0.8, kSubLeave = 0.5;
// ... and the subscription EWMA falls with this longer time constant (leaves
// the mode ~35 ms after the GPU stopped being full): symmetric tenants that
// finish a phase together do not hand the last runner straight to its token
// bucket -- alone it is charged the whole GPU, and eight pooled 12.5 %
// tenants measured the last one held 75 ms at the end of a 100-step window
// (round 6); a tenant left alone for longer is still capped by its bucket.
constexpr uint64_t kSubFallTauNs = 50000000ull;
// Fair-share mode: credit a process keeps while it is not backlogged (its
// virtual time trails the smallest running one by at most this much GPU
// time): a tenant returning from a short gap is still behind the ones that
// ran without it, one away for long has banked no more than this.
constexpr uint64_t kCreditNs = 5000000ull;
// Fair-share mode: a tenant whose flags went stale still counts as backlogged
// by its last fresh state for this long.
constexpr uint64_t kStateGraceNs = 100000000ull;
// Fair-share mode: a HELD or OWES flag counts while the process had waves of
// its own resident within this long (a held tenant runs a graph between its
// gates at least every ~25 ms hold; an idle one faked busy by a neighbour
// drops out after this).
constexpr uint64_t kEvidenceNs = 200000000ull;
// Fair-share mode: a tenant's lead over the furthest-behind contender is
// bounded here (virtual time beyond it is dropped: a tenant cannot bank an
// unbounded lead that holds it for seconds).
constexpr uint64_t kMaxLeadNs = 200000000ull;
// Fair-share mode: default presence window (Handle::presence_ns).
constexpr uint64_t kPresenceNs = 20000000ull;

struct Reading {
  int pid;
  int v;   // cu_occupancy, < 0 = unreadable this pass
};

// Node sampler: one container's flags (<dir>/flags/<key>/gpu-<id>.flags),
// read with pread into a private copy every pass -- never mapped, so a tenant
// truncating its file cannot fault the root sampler (SIGBUS), and never
// created or written.
struct KeyFlags {
  char key[MIVGPU_OWNER_KEY_MAX] = {0};
  int fd = -1;
  bool ok = false;                          // buf holds a valid copy this pass
  bool seen = false;                        // listed by the last directory scan
  mivgpu_board_flags_t* buf = nullptr;
};

struct Handle {
  mivgpu_board_t* b = nullptr;
  int fd = -1;
  int owner_fd = -1;
  bool writable = false;
  bool owner = false;
  bool node = false;           // the node sampler: reads tenant files only (pread, O_NOFOLLOW)
  int gpu_id = -1;
  uint64_t last_pass_ns = 0;   // owner: the previous pass
  char dir[256] = {0};
  char flags_dir[512] = {0};   // this tenant's flags directory ("" = <dir>/flags)
  mivgpu_board_flags_t* flags = nullptr;   // shim: <flags dir>/gpu-<id>.flags, mapped (tenant-written)
  int flag_slot = -1;                      // this tenant's entry
  // node sampler: the shared flags file (no per-container directories: hand-run
  // slices) and every container's own, plus host truth's pid -> container map
  KeyFlags shared;
  std::vector<KeyFlags> keys;
  std::vector<std::pair<int, int>> owners;   // (host pid, index into keys), sorted by pid
  uint64_t owners_ns = 0;
  uint64_t demand_ns = 0;                    // the last pass with a fresh GATED flag
  // node-written core limits (<dir>/gpu-<id>.limits), reloaded every 100 ms
  mivgpu_limit_entry_t* lims = nullptr;
  int nlims = 0;
  uint64_t lims_ns = 0;
  // owner-private fair-share state
  bool was_backlogged[MIVGPU_BOARD_SLOTS] = {};   // per board slot, the previous pass
  double bl_ewma[MIVGPU_BOARD_SLOTS] = {};        // per board slot, share of recent passes backlogged
  uint32_t last_lim[MIVGPU_BOARD_SLOTS] = {};     // per board slot, the weight of its last fresh flags
  int last_state[MIVGPU_BOARD_SLOTS] = {};        // ... their state, and when they were fresh
  uint64_t last_state_ns[MIVGPU_BOARD_SLOTS] = {};
  uint64_t wave_ns[MIVGPU_BOARD_SLOTS] = {};      // per board slot, the last pass with its waves resident
  uint64_t run_ns[MIVGPU_BOARD_SLOTS] = {};       // per board slot, the last pass with more than a gate's waves
  // fair-share presence window: a backlogged, unheld process counts as
  // present while it had more than a gate's waves resident within this long
  // (0 = at this pass's instant only, the round-5 rule).  A decode tenant's
  // stream of short kernels is caught between two of them in some passes and
  // not others; eight symmetric tenants were charged 12.0-13.8 % on the
  // instant.
  uint64_t presence_ns = kPresenceNs;
  double sub_ewma = 0;                            // share of recent passes fully subscribed
  bool fair = false;                              // fair-share mode
  uint64_t vmin = 0;                              // the previous pass's smallest running virtual time
};

// fstat under the shim's glibc floor (glibc_floor.h: fstat became a real
// symbol in GLIBC_2.33); plain fstat for the node sampler.
inline int board_fstat(int fd, struct stat* st) {
#ifdef MIVGPU_GLIBC_FLOOR_H
  return mivgpu_fstat(fd, st);
#else
  return fstat(fd, st);
#endif
}

inline void board_path(char* out, size_t n, const char* dir, int gpu_id, const char* ext) {
  snprintf(out, n, "%s/gpu-%d.%s", dir, gpu_id, ext);
}

// open(2) of an existing REGULAR file, never through a symlink in the last
// component, never blocking on a FIFO planted in its place (the
// node sampler runs as root next to tenant-writable directories).
inline int open_regular(const char* path, int flags) {
  const int fd = open(path, flags | O_NOFOLLOW | O_NONBLOCK | O_CLOEXEC);
  if (fd < 0) return -1;
  struct stat st;
  if (board_fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
    close(fd);
    errno = EINVAL;
    return -1;
  }
  return fd;
}

// Create a new private file <dir>/.<stem>.<pid>.<nonce> (O_EXCL: never an
// existing file or a planted symlink; the name is not predictable from the pid).
inline int create_private(const char* dir, const char* stem, char* out, size_t n) {
  for (int attempt = 0; attempt < 16; ++attempt) {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    const unsigned long nonce = (unsigned long)ts.tv_nsec ^ ((unsigned long)ts.tv_sec << 20) ^
                                ((unsigned long)attempt * 2654435761ul) ^ (unsigned long)(uintptr_t)out;
    snprintf(out, n, "%s/.%s.%d.%lx", dir, stem, (int)getpid(), nonce);
    const int fd = open(out, O_RDWR | O_CREAT | O_EXCL | O_NOFOLLOW | O_CLOEXEC, 0666);
    if (fd >= 0) return fd;
    if (errno != EEXIST) return -1;
  }
  return -1;
}

// Create <dir>/gpu-<id>.board if it does not exist: built under a private
// name and linked into place, so a reader never maps a half-initialised file.
inline bool create_board(const char* dir, int gpu_id) {
  if (mkdir(dir, 0777) == 0) (void)chmod(dir, 0777);   // tenants of other uids share it
  char path[512], tmp[600], stem[64];
  board_path(path, sizeof(path), dir, gpu_id, "board");
  snprintf(stem, sizeof(stem), "gpu-%d.board", gpu_id);
  int fd = create_private(dir, stem, tmp, sizeof(tmp));
  if (fd < 0) return false;
  (void)fchmod(fd, 0666);
  bool ok = ftruncate(fd, (off_t)sizeof(mivgpu_board_t)) == 0;
  if (ok) {
    mivgpu_board_t init;
    memset(&init, 0, sizeof(init));
    init.magic = MIVGPU_BOARD_MAGIC;
    init.version = MIVGPU_BOARD_VERSION;
    init.gpu_id = gpu_id;
    ok = pwrite(fd, &init, sizeof(init), 0) == (ssize_t)sizeof(init);
  }
  close(fd);
  if (ok && link(tmp, path) != 0 && errno != EEXIST) ok = false;
  unlink(tmp);
  return ok;
}

// Map the board of KFD GPU `gpu_id` in `dir`: read-write where the directory
// allows it (a shim may then become the owner), read-only otherwise (the
// production mount: only the node sampler writes).
inline bool open_board(Handle& h, const char* dir, int gpu_id, bool may_create) {
  if (!dir || !*dir || gpu_id < 0) return false;
  char path[512];
  board_path(path, sizeof(path), dir, gpu_id, "board");
  int fd = open_regular(path, O_RDWR);
  bool writable = fd >= 0;
  if (fd < 0 && errno == ENOENT && may_create && create_board(dir, gpu_id)) {
    fd = open_regular(path, O_RDWR);
    writable = fd >= 0;
  }
  if (fd < 0) {
    fd = open_regular(path, O_RDONLY);
    writable = false;
  }
  if (fd < 0) return false;
  struct stat st;
  if (board_fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(mivgpu_board_t)) {
    close(fd);
    return false;
  }
  void* m = mmap(nullptr, sizeof(mivgpu_board_t), PROT_READ | (writable ? PROT_WRITE : 0), MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) {
    close(fd);
    return false;
  }
  mivgpu_board_t* b = static_cast<mivgpu_board_t*>(m);
  if (b->magic != MIVGPU_BOARD_MAGIC || b->version != MIVGPU_BOARD_VERSION || b->gpu_id != gpu_id) {
    munmap(m, sizeof(mivgpu_board_t));
    close(fd);
    return false;
  }
  h.b = b;
  h.fd = fd;
  h.writable = writable;
  h.gpu_id = gpu_id;
  snprintf(h.dir, sizeof(h.dir), "%s", dir);
  return true;
}

// Shim side: map (creating it if needed) <flags dir>/gpu-<id>.flags
// read-write -- this tenant's own directory in production
// (MIVGPU_BOARD_FLAGS_DIR), <dir>/flags shared by hand-run slices.  False when
// it cannot be written (the owner then judges this process from its occupancy
// alone).  The node sampler never calls this (node_flags_refresh reads).
inline bool open_flags(Handle& h) {
  if (h.flags) return true;
  if (h.node) return false;
  char fdir[600], path[700];
  if (h.flags_dir[0]) snprintf(fdir, sizeof(fdir), "%s", h.flags_dir);
  else snprintf(fdir, sizeof(fdir), "%s/flags", h.dir);
  if (mkdir(fdir, 0777) == 0) (void)chmod(fdir, 0777);
  snprintf(path, sizeof(path), "%s/gpu-%d.flags", fdir, h.gpu_id);
  int fd = open_regular(path, O_RDWR);
  if (fd < 0 && errno == ENOENT) {
    char tmp[800], stem[64];
    snprintf(stem, sizeof(stem), "gpu-%d.flags", h.gpu_id);
    const int t = create_private(fdir, stem, tmp, sizeof(tmp));
    if (t >= 0) {
      (void)fchmod(t, 0666);
      mivgpu_board_flags_t init;
      memset(&init, 0, sizeof(init));
      init.magic = MIVGPU_FLAGS_MAGIC;
      init.version = MIVGPU_FLAGS_VERSION;
      init.gpu_id = h.gpu_id;
      const bool ok = pwrite(t, &init, sizeof(init), 0) == (ssize_t)sizeof(init);
      close(t);
      if (ok) (void)link(tmp, path);
      unlink(tmp);
    }
    fd = open_regular(path, O_RDWR);
  }
  if (fd < 0) return false;
  struct stat st;
  if (board_fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(mivgpu_board_flags_t)) {
    close(fd);
    return false;
  }
  void* m = mmap(nullptr, sizeof(mivgpu_board_flags_t), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return false;
  mivgpu_board_flags_t* f = static_cast<mivgpu_board_flags_t*>(m);
  if (f->magic != MIVGPU_FLAGS_MAGIC || f->version != MIVGPU_FLAGS_VERSION || f->gpu_id != h.gpu_id) {
    munmap(m, sizeof(mivgpu_board_flags_t));
    return false;
  }
  h.flags = f;
  return true;
}

// Node side: a container key as the monitor and the device plugin write it.
inline bool valid_key(const char* k) {
  const size_t n = strlen(k);
  if (n == 0 || n >= MIVGPU_OWNER_KEY_MAX || !strcmp(k, ".") || !strcmp(k, "..")) return false;
  for (size_t i = 0; i < n; ++i) {
    const char c = k[i];
    if (!((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_' || c == '-' ||
          c == '.'))
      return false;
  }
  return true;
}

inline void drop_key(KeyFlags& k) {
  if (k.fd >= 0) close(k.fd);
  k.fd = -1;
  k.ok = false;
  delete k.buf;
  k.buf = nullptr;
}

// Node side: open <dir>/flags/<key>/gpu-<id>.flags (key "" = the shared
// <dir>/flags/gpu-<id>.flags) read-only: the key directory and the file
// without following symlinks, a regular file only.
inline void open_key(Handle& h, KeyFlags& k) {
  if (k.fd >= 0) return;
  char d[700], name[64];
  if (k.key[0]) snprintf(d, sizeof(d), "%s/flags/%s", h.dir, k.key);
  else snprintf(d, sizeof(d), "%s/flags", h.dir);
  snprintf(name, sizeof(name), "gpu-%d.flags", h.gpu_id);
  const int dfd = open(d, O_RDONLY | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC);
  if (dfd < 0) return;
  const int fd = openat(dfd, name, O_RDONLY | O_NOFOLLOW | O_NONBLOCK | O_CLOEXEC);
  close(dfd);
  if (fd < 0) return;
  struct stat st;
  if (board_fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
    close(fd);
    return;
  }
  k.fd = fd;
  if (!k.buf) k.buf = new mivgpu_board_flags_t;
}

// Node side, every pass: re-read the containers' flags directories and host
// truth's owners (every 100 ms), then copy every open flags file (pread).
inline void node_flags_refresh(Handle& h, uint64_t now) {
  if (!h.owners_ns || now - h.owners_ns >= 100000000ull) {
    h.owners_ns = now;
    for (KeyFlags& k : h.keys) k.seen = false;
    char d[600];
    snprintf(d, sizeof(d), "%s/flags", h.dir);
    if (DIR* dir = opendir(d)) {
      while (dirent* e = readdir(dir)) {
        if (!valid_key(e->d_name) || !strncmp(e->d_name, "gpu-", 4)) continue;
        // a directory, not a symlink to one (open_key opens it O_DIRECTORY | O_NOFOLLOW too)
        if (e->d_type != DT_DIR && e->d_type != DT_UNKNOWN) continue;
        KeyFlags* hit = nullptr;
        for (KeyFlags& k : h.keys)
          if (!strcmp(k.key, e->d_name)) hit = &k;
        if (!hit) {
          if (h.keys.size() >= 4 * MIVGPU_BOARD_SLOTS) continue;
          h.keys.emplace_back();
          hit = &h.keys.back();
          snprintf(hit->key, sizeof(hit->key), "%s", e->d_name);
        }
        hit->seen = true;
      }
      closedir(dir);
    }
    for (size_t i = 0; i < h.keys.size();) {
      if (!h.keys[i].seen) {
        drop_key(h.keys[i]);
        h.keys.erase(h.keys.begin() + (long)i);
      } else {
        open_key(h, h.keys[i]);
        ++i;
      }
    }
    open_key(h, h.shared);
    // owners: "<pid> <key>" lines under a "MIVGPU-OWNERS 1 <gpu_id>" header
    h.owners.clear();
    char path[600];
    board_path(path, sizeof(path), h.dir, h.gpu_id, "owners");
    const int fd = open_regular(path, O_RDONLY);
    if (fd >= 0) {
      const size_t cap = MIVGPU_OWNERS_MAX * (MIVGPU_OWNER_KEY_MAX + 16) + 64;
      std::vector<char> buf(cap);
      char* text = buf.data();
      const ssize_t n = pread(fd, text, cap - 1, 0);
      close(fd);
      int ver = 0, gid = -1, off = 0;
      if (n > 0) {
        text[n] = 0;
        if (sscanf(text, "MIVGPU-OWNERS %d %d%n", &ver, &gid, &off) == 2 && ver == 1 && gid == h.gpu_id) {
          char* p = text + off;
          while (*p && h.owners.size() < MIVGPU_OWNERS_MAX) {
            while (*p == '\n' || *p == ' ') ++p;
            char key[MIVGPU_OWNER_KEY_MAX];
            int pid = 0, used = 0;
            if (sscanf(p, "%d %127s%n", &pid, key, &used) != 2) break;
            p += used;
            if (pid <= 0 || !valid_key(key)) continue;
            for (size_t i = 0; i < h.keys.size(); ++i)
              if (!strcmp(h.keys[i].key, key)) {
                h.owners.emplace_back(pid, (int)i);
                break;
              }
          }
        }
      }
      std::sort(h.owners.begin(), h.owners.end());
    }
  }
  auto copy = [&](KeyFlags& k) {
    k.ok = false;
    if (k.fd < 0 || !k.buf) return;
    if (pread(k.fd, k.buf, sizeof(*k.buf), 0) != (ssize_t)sizeof(*k.buf)) return;
    k.ok = k.buf->magic == MIVGPU_FLAGS_MAGIC && k.buf->version == MIVGPU_FLAGS_VERSION &&
           k.buf->gpu_id == h.gpu_id;
  };
  for (KeyFlags& k : h.keys) copy(k);
  copy(h.shared);
}

// Tenant side: publish this pass's state and its core limit (ppm, 0 = none)
// under its KFD pid (an entry claimed once, by CAS on a free or stale one).
inline void publish_flags(Handle& h, int pid, int state, uint32_t limit_ppm, uint64_t now) {
  if (!h.flags || pid <= 0) return;
  mivgpu_flag_t* e = h.flag_slot >= 0 ? &h.flags->flags[h.flag_slot] : nullptr;
  if (!e || __atomic_load_n(&e->pid, __ATOMIC_RELAXED) != pid) {
    h.flag_slot = -1;
    for (int k = 0; k < MIVGPU_FLAGS_SLOTS && h.flag_slot < 0; ++k) {
      mivgpu_flag_t* c = &h.flags->flags[k];
      int cur = __atomic_load_n(&c->pid, __ATOMIC_ACQUIRE);
      if (cur == pid) h.flag_slot = k;
    }
    for (int k = 0; k < MIVGPU_FLAGS_SLOTS && h.flag_slot < 0; ++k) {
      mivgpu_flag_t* c = &h.flags->flags[k];
      int cur = __atomic_load_n(&c->pid, __ATOMIC_ACQUIRE);
      const bool stale = cur != 0 && __atomic_load_n(&c->stamp_ns, __ATOMIC_RELAXED) + 2000000000ull < now;
      if ((cur == 0 || stale) &&
          __atomic_compare_exchange_n(&c->pid, &cur, pid, false, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED))
        h.flag_slot = k;
    }
    if (h.flag_slot < 0) return;
    e = &h.flags->flags[h.flag_slot];
  }
  __atomic_store_n(&e->state, state, __ATOMIC_RELAXED);
  __atomic_store_n(&e->limit_ppm, limit_ppm, __ATOMIC_RELAXED);
  __atomic_store_n(&e->stamp_ns, now, __ATOMIC_RELEASE);
}

// Owner side: (re)load the node-written core limits, at most every 100 ms.
inline void load_limits(Handle& h, uint64_t now) {
  if (h.lims_ns && now - h.lims_ns < 100000000ull) return;
  h.lims_ns = now;
  h.nlims = 0;
  char path[512];
  board_path(path, sizeof(path), h.dir, h.gpu_id, "limits");
  const int fd = open_regular(path, O_RDONLY);
  if (fd < 0) return;
  mivgpu_board_limits_t hdr;
  if (pread(fd, &hdr, sizeof(hdr), 0) == (ssize_t)sizeof(hdr) && hdr.magic == MIVGPU_LIMITS_MAGIC &&
      hdr.version == MIVGPU_LIMITS_VERSION && hdr.gpu_id == h.gpu_id && hdr.count > 0 &&
      hdr.count <= MIVGPU_LIMITS_MAX) {
    if (!h.lims) h.lims = new mivgpu_limit_entry_t[MIVGPU_LIMITS_MAX];
    const ssize_t want = (ssize_t)(hdr.count * sizeof(mivgpu_limit_entry_t));
    if (pread(fd, h.lims, (size_t)want, sizeof(hdr)) == want) h.nlims = hdr.count;
  }
  close(fd);
}

// The node-written core limit of `pid` (ppm), 0 when it has none.
inline uint32_t node_limit(const Handle& h, int pid) {
  for (int k = 0; k < h.nlims; ++k)
    if (h.lims[k].pid == pid) return h.lims[k].limit_ppm;
  return 0;
}

// Owner side: a process's published state, -1 when it has no fresh entry;
// `limit_ppm` gets its core limit (1e6 when it has none).
constexpr uint64_t kFlagFreshNs = 20000000ull;   // 20 ms: ten tenant passes
inline int read_flags(const mivgpu_board_flags_t* f, int pid, uint64_t now, uint32_t* limit_ppm = nullptr) {
  if (limit_ppm) *limit_ppm = 1000000u;
  if (!f || pid <= 0) return -1;
  for (int k = 0; k < MIVGPU_FLAGS_SLOTS; ++k) {
    const mivgpu_flag_t* e = &f->flags[k];
    if (__atomic_load_n(&e->pid, __ATOMIC_ACQUIRE) != pid) continue;
    const uint64_t st = __atomic_load_n(&e->stamp_ns, __ATOMIC_ACQUIRE);
    if (st + kFlagFreshNs < now) return -1;
    const uint32_t lim = __atomic_load_n(&e->limit_ppm, __ATOMIC_RELAXED);
    if (limit_ppm && lim > 0 && lim < 1000000u) *limit_ppm = lim;
    return __atomic_load_n(&e->state, __ATOMIC_RELAXED);
  }
  return -1;
}

// Owner side: the flags a process's state is read from.  The shim owner
// (hand-run slices): the shared file.  The node sampler: the file of the
// container host truth attributes the pid to -- nothing else, so a tenant
// cannot speak for a neighbour; a pid not attributed (yet) takes the one
// source that has a fresh entry for it, none when two disagree.
inline const mivgpu_board_flags_t* flags_of(const Handle& h, int pid, uint64_t now) {
  if (!h.node) return h.flags;
  auto it = std::lower_bound(h.owners.begin(), h.owners.end(), std::make_pair(pid, -1));
  if (it != h.owners.end() && it->first == pid) {
    const KeyFlags& k = h.keys[(size_t)it->second];
    return k.ok ? k.buf : nullptr;
  }
  const mivgpu_board_flags_t* hit = nullptr;
  int hits = 0;
  auto probe = [&](const KeyFlags& k) {
    if (!k.ok || hits > 1) return;
    if (read_flags(k.buf, pid, now) >= 0) {
      hit = k.buf;
      ++hits;
    }
  };
  probe(h.shared);
  for (const KeyFlags& k : h.keys) probe(k);
  return hits == 1 ? hit : nullptr;
}

inline bool node_owner_live(const mivgpu_board_t* b, int self_pid, uint64_t now) {
  const int kind = __atomic_load_n(&b->owner_kind, __ATOMIC_ACQUIRE);
  const uint64_t beat = __atomic_load_n(&b->beat_ns, __ATOMIC_ACQUIRE);
  return kind == MIVGPU_BOARD_OWNER_NODE && __atomic_load_n(&b->owner_pid, __ATOMIC_RELAXED) != self_pid &&
         beat + 1000000000ull > now;
}

// Shim side: take the owner role with a non-blocking flock on
// <dir>/gpu-<id>.owner (released by the kernel when the process dies).
inline bool try_own(Handle& h, int self_pid, uint64_t now) {
  if (!h.b || !h.writable || h.owner) return h.owner;
  if (node_owner_live(h.b, self_pid, now)) return false;
  if (h.owner_fd < 0) {
    char path[512];
    board_path(path, sizeof(path), h.dir, h.gpu_id, "owner");
    h.owner_fd = open(path, O_RDWR | O_CREAT | O_NOFOLLOW | O_NONBLOCK | O_CLOEXEC, 0666);
    if (h.owner_fd < 0) return false;
    (void)fchmod(h.owner_fd, 0666);
  }
  if (flock(h.owner_fd, LOCK_EX | LOCK_NB) != 0) return false;
  h.owner = true;
  h.last_pass_ns = 0;
  __atomic_store_n(&h.b->owner_pid, self_pid, __ATOMIC_RELAXED);
  __atomic_store_n(&h.b->owner_kind, (int32_t)MIVGPU_BOARD_OWNER_SHIM, __ATOMIC_RELEASE);
  return true;
}

inline void release_own(Handle& h) {
  if (!h.owner) return;
  h.owner = false;
  if (h.owner_fd >= 0) (void)flock(h.owner_fd, LOCK_UN);
}

// How a pass splits the GPU among the processes with waves resident: by
// their waves (default), or equally (A/B).
enum Split { kSplitRatio = 0, kSplitEqual = 1 };

// One owner pass over `n` readings (every KFD process on the GPU, this pass).
// Call with h.owner (or from the node sampler); `kind`/`owner_pid` go to the
// header.  Per process:
//   held   -- its flags say its streams sit in a governor gate, or (no fresh
//             flags) it shows exactly a gate's CU unit: not contending, and
//             the pass is not observed for it;
//   w      -- its resident CU units when not held (a running tenant's small
//             kernels count: a queued tenant is not charged the GPU while
//             they run);
//   f      -- w / W when any process has waves resident (W = all w); when
//             none has, the owing tenants (flags) split the pass equally (a
//             process without flags is charged it whole: it is alone between
//             its own kernels).
// Then the fair-share state (shared_region.h, vt_ns / lead_ns): a process is
// backlogged in a pass when it owes work or sits in a gate (flags; one
// without flags: waves resident), weighted by its core limit (flags; 100 %
// without; the monitor's node-written limit caps it).  In fair-share mode
// (the backlogged weights filling the GPU in most recent passes) each
// backlogged process's virtual time advances by its presence (an equal part
// of each pass among the processes with waves resident) / its weight; one not backlogged, or held while behind, keeps at most
// kCreditNs of credit below the smallest running virtual time (a short gap
// does not forgive the ones that ran without it, a long one banks nothing
// more), and every process's lead is (vt - the running processes' mean vt)
// x its weight.  Outside the mode lead_ns = -1: the tenants' own token buckets cap
// them.
inline void owner_pass(Handle& h, const Reading* r, int n, uint64_t now, uint64_t period_ns, int kind,
                       int owner_pid, int split, uint64_t pass_cost_ns) {
  mivgpu_board_t* b = h.b;
  if (!b || !h.writable) return;
  uint64_t dt = h.last_pass_ns && now > h.last_pass_ns ? now - h.last_pass_ns : 0;
  if (dt > kMaxDtNs) dt = kMaxDtNs;
  h.last_pass_ns = now;
  if (h.node) node_flags_refresh(h, now);
  else if (h.flags == nullptr) (void)open_flags(h);
  load_limits(h, now);
  constexpr int kMaxRead = 256;
  int st[kMaxRead], sl[kMaxRead];
  bool hd[kMaxRead];
  uint32_t lim[kMaxRead];
  long wv[kMaxRead];
  double use[kMaxRead];
  long W = 0;
  int resident = 0, owing = 0, present = 0;
  if (n > kMaxRead) n = kMaxRead;
  for (int i = 0; i < n; ++i) {
    st[i] = read_flags(flags_of(h, r[i].pid, now), r[i].pid, now, &lim[i]);
    if (st[i] >= 0 && (st[i] & MIVGPU_FLAG_GATED)) h.demand_ns = now;
    // the grant's, when the monitor knows the process: authoritative over
    // whatever the tenant-written flags say
    const uint32_t nl = node_limit(h, r[i].pid);
    if (nl > 0) lim[i] = nl;
    const int v = r[i].v;
    bool held;
    // HELD flags are up to one tenant pass old: a tenant already released
    // (more than a gate's waves resident) runs.  Trusting the flag charged
    // such tenants nothing while the owner's own flags, always fresh, charged
    // it in full -- the owner came out slowest (held 0.8 s of a 2.9 s run).
    if (st[i] >= 0) held = (st[i] & MIVGPU_FLAG_HELD) != 0 && v <= kGateUnits;
    else held = v > 0 && v <= kGateUnits;
    hd[i] = held;
    wv[i] = (!held && v > 0) ? v : 0;
    if (st[i] >= 0 && (st[i] & MIVGPU_FLAG_OWES) && !held) ++owing;
    if (wv[i] > 0) {
      W += wv[i];
      ++resident;
    }
    if (wv[i] > kGateUnits) ++present;   // more than a gate's (or a stale HELD flag's) one CU unit
  }
  const uint64_t s0 = __atomic_load_n(&b->seq, __ATOMIC_RELAXED);
  __atomic_store_n(&b->seq, s0 | 1ull, __ATOMIC_RELAXED);
  __atomic_thread_fence(__ATOMIC_RELEASE);
  int hi = __atomic_load_n(&b->nslots, __ATOMIC_RELAXED);
  if (hi < 0 || hi > MIVGPU_BOARD_SLOTS) hi = MIVGPU_BOARD_SLOTS;
  double sum_w = 0;   // backlogged processes' weights
  int backlogged = 0;
  bool bl[kMaxRead];
  for (int i = 0; i < n; ++i) {
    sl[i] = -1;
    use[i] = 0;
    bl[i] = false;
    if (r[i].pid <= 0 || r[i].v < 0) continue;
    int slot = -1, free_slot = -1;
    for (int k = 0; k < MIVGPU_BOARD_SLOTS; ++k) {
      const int p = b->slots[k].pid;
      if (p == r[i].pid) {
        slot = k;
        break;
      }
      if (free_slot < 0 && (p == 0 || b->slots[k].seen_ns + kSlotStaleNs < now)) free_slot = k;
    }
    if (slot < 0) {
      if (free_slot < 0) continue;   // more than 64 processes on one GPU: the rest go unboarded
      slot = free_slot;
      mivgpu_board_slot_t& s = b->slots[slot];
      memset(&s, 0, sizeof(s));
      s.pid = r[i].pid;
      s.lead_ns = -1;
      h.was_backlogged[slot] = false;
      h.bl_ewma[slot] = 0;
      h.last_lim[slot] = 0;
      h.last_state_ns[slot] = 0;
      h.wave_ns[slot] = 0;
      h.run_ns[slot] = 0;
      if (slot + 1 > hi) hi = slot + 1;
    }
    sl[i] = slot;
    mivgpu_board_slot_t& s = b->slots[slot];
    const int v = r[i].v;
    const long w = wv[i];
    const bool held = hd[i];
    const bool owes = st[i] >= 0 && (st[i] & MIVGPU_FLAG_OWES);
    s.occupancy = v;
    s.seen_ns = now;
    // a tenant whose flags went stale for a moment (its sampler thread
    // descheduled) keeps the weight of its last fresh ones
    if (st[i] >= 0) {
      h.last_lim[slot] = lim[i];
      h.last_state[slot] = st[i];
      h.last_state_ns[slot] = now;
    } else if (h.last_lim[slot] && !node_limit(h, r[i].pid)) {
      lim[i] = h.last_lim[slot];
    }
    // backlogged: by its flags; by the last fresh ones within kStateGraceNs
    // (measured: with eight tenants their samplers ran every ~5.5 ms, not 2,
    // and a stall past the 20 ms freshness dropped a queued tenant out of the
    // subscription half the time); without flags, waves resident
    // Flags are tenant-writable, so they only count with evidence in the
    // readings: the process had waves beyond a gate's resident, or its gate's
    // wave, within kEvidenceNs.  A tenant faking an idle neighbour's flags
    // could otherwise declare the GPU fully subscribed and escape its own cap
    // in the fair-share mode.  (Demanding the gate's wave at every pass of a
    // hold instead, a held 25 % tenant next to a 75 % one measured 28 %.)
    if (w > kGateUnits || (held && v > 0)) h.wave_ns[slot] = now;
    if (w > kGateUnits) h.run_ns[slot] = now;
    const bool evidence = h.wave_ns[slot] && now - h.wave_ns[slot] < kEvidenceNs;
    if (st[i] >= 0) bl[i] = (held || owes) && evidence;
    else if (h.last_state_ns[slot] && now - h.last_state_ns[slot] < kStateGraceNs)
      bl[i] = ((h.last_state[slot] & (MIVGPU_FLAG_HELD | MIVGPU_FLAG_OWES)) && evidence) || w > 0;
    else bl[i] = w > 0;
    if (dt) {
      const double a = (double)dt / (double)kSubTauNs < 1.0 ? (double)dt / (double)kSubTauNs : 1.0;
      h.bl_ewma[slot] += a * ((bl[i] ? 1.0 : 0.0) - h.bl_ewma[slot]);
    }
    if (h.bl_ewma[slot] >= 0.5) {
      sum_w += (double)lim[i] / 1e6;
      ++backlogged;
    }
    if (!dt) continue;
    double f, got;
    if (W > 0) {
      got = split == kSplitEqual ? (w > 0 ? 1.0 / (double)resident : 0.0) : (double)w / (double)W;
      f = got;
      // the fair-share virtual time advances by presence: an equal part of
      // the pass for each process with waves resident (the reference's
      // NVML per-process utilisation is time-sliced presence).  The wave
      // ratio charged below scatters with each kernel's shape: eight
      // identical decode tenants came out 0.87 apart in throughput after
      // being held on it, where the hardware alone gives 0.996 (half ratio,
      // half presence: 0.91, and a 25 % tenant next to a 75 % one at 30 %).
      use[i] = w > kGateUnits ? 1.0 / (double)present : 0.0;
    } else {
      got = 0.0;
      // nobody resident: the owing tenants split the pass; any other process
      // is charged it whole -- alone between its own kernels, a tenant's
      // flags can read "owes nothing" at the pass that falls in a dispatch
      // gap (round 6 tried charging those nothing: a lone tenant under a
      // 12.5 % limit then ran at 0.27 of unthrottled, a Triton loop under 25 %
      // at 0.48; a tenant only charges a sample in which it owes work, so an
      // idle one pays nothing anyway)
      f = st[i] < 0 ? 1.0 : (owes && owing > 0 ? 1.0 / (double)owing : 1.0);
      use[i] = owes && owing > 0 ? 1.0 / (double)owing : 0.0;
    }
    if (!held) {
      s.obs_ns += dt;
      s.frac_ns += (uint64_t)(f * (double)dt + 0.5);
    }
    s.recv_ns += (uint64_t)(got * (double)dt + 0.5);
    if (w > 0) s.busy_ns += dt;
  }
  // presence over a window: every backlogged, unheld process whose waves ran
  // within presence_ns shares the pass equally (a dispatch gap at the pass's
  // instant does not make it absent; a starved one drops out after the window)
  if (h.presence_ns && W > 0 && dt) {
    int npres = 0;
    for (int i = 0; i < n; ++i)
      if (sl[i] >= 0 && bl[i] && !hd[i] && h.run_ns[sl[i]] && now - h.run_ns[sl[i]] < h.presence_ns) ++npres;
    for (int i = 0; i < n; ++i) {
      if (sl[i] < 0) continue;
      const bool p = bl[i] && !hd[i] && h.run_ns[sl[i]] && now - h.run_ns[sl[i]] < h.presence_ns;
      use[i] = p && npres ? 1.0 / (double)npres : 0.0;
    }
  }
  // fair-share mode while the backlogged weights fill the GPU
  if (dt) {
    const double x = (backlogged >= 2 && sum_w >= 0.999) ? 1.0 : 0.0;
    const double tau = (double)(x >= h.sub_ewma ? kSubTauNs : kSubFallTauNs);
    const double a = (double)dt / tau < 1.0 ? (double)dt / tau : 1.0;
    h.sub_ewma += a * (x - h.sub_ewma);
  }
  if (backlogged >= 2 && sum_w >= 0.999) b->sub_passes += 1;
  const bool entering = !h.fair && h.sub_ewma >= kSubEnter;
  h.fair = h.fair ? h.sub_ewma >= kSubLeave : entering;
  auto running = [&](int i) { return bl[i] && !hd[i]; };
  if (h.fair) {
    if (entering) {
      // everyone starts level
      uint64_t top = 0;
      for (int i = 0; i < n; ++i)
        if (sl[i] >= 0 && b->slots[sl[i]].vt_ns > top) top = b->slots[sl[i]].vt_ns;
      for (int i = 0; i < n; ++i)
        if (sl[i] >= 0) b->slots[sl[i]].vt_ns = top;
      h.vmin = top;
    }
    for (int i = 0; i < n; ++i) {
      const int k = sl[i];
      if (k < 0 || !bl[i]) continue;
      mivgpu_board_slot_t& s = b->slots[k];
      // joins within its credit of the running minimum (a new process too)
      const uint64_t credit = (uint64_t)((double)kCreditNs * 1e6 / (double)lim[i]);
      if (!h.was_backlogged[k] && s.vt_ns + credit < h.vmin) s.vt_ns = h.vmin - credit;
      s.vt_ns += (uint64_t)(use[i] * (double)dt * 1e6 / (double)lim[i] + 0.5);
    }
    uint64_t vmin = UINT64_MAX;
    double vsum = 0;
    int nrun = 0;
    for (int i = 0; i < n; ++i)
      if (sl[i] >= 0 && running(i)) {
        const uint64_t vt = b->slots[sl[i]].vt_ns;
        if (vt < vmin) vmin = vt;
        vsum += (double)vt;
        ++nrun;
      }
    if (vmin == UINT64_MAX) vmin = h.vmin;
    for (int i = 0; i < n; ++i) {
      const int k = sl[i];
      if (k < 0) continue;
      mivgpu_board_slot_t& s = b->slots[k];
      if (running(i)) {
        if (s.vt_ns < vmin) s.vt_ns = vmin;
      } else {
        const uint64_t credit = (uint64_t)((double)kCreditNs * 1e6 / (double)lim[i]);
        if (s.vt_ns + credit < vmin) s.vt_ns = vmin - credit;
      }
      const uint64_t cap = vmin + (uint64_t)((double)kMaxLeadNs * 1e6 / (double)lim[i]);
      if (s.vt_ns > cap) s.vt_ns = cap;
      // the lead is taken over the running processes' mean virtual time:
      // against the minimum, the spread of eight tenants' noisy estimates
      // alone put every one but the last behind its gate a third of the time
      const double vmean = nrun ? vsum / nrun : (double)vmin;
      const double ahead = (double)s.vt_ns - vmean;
      s.lead_ns = ahead > 0 ? (int64_t)(ahead * (double)lim[i] / 1e6 + 0.5) : 0;
    }
    h.vmin = vmin;
    b->fair_passes += 1;
  } else {
    for (int i = 0; i < n; ++i)
      if (sl[i] >= 0) b->slots[sl[i]].lead_ns = -1;
  }
  for (int i = 0; i < n; ++i)
    if (sl[i] >= 0) h.was_backlogged[sl[i]] = bl[i];
  // slots of processes gone for a while are freed (a new process may get the pid)
  for (int k = 0; k < hi; ++k)
    if (b->slots[k].pid && b->slots[k].seen_ns + kSlotStaleNs < now) memset(&b->slots[k], 0, sizeof(b->slots[k]));
  while (hi > 0 && b->slots[hi - 1].pid == 0) --hi;
  b->nslots = hi;
  if (W > 0) b->busy_ns += dt;
  b->passes += 1;
  b->period_ns = period_ns;
  b->pass_ns = pass_cost_ns;
  b->owner_pid = owner_pid;
  b->owner_kind = kind;
  __atomic_store_n(&b->beat_ns, now, __ATOMIC_RELAXED);
  __atomic_store_n(&b->seq, (s0 | 1ull) + 1ull, __ATOMIC_RELEASE);
}

struct View {
  int owner_kind = 0;
  int owner_pid = 0;
  int occupancy = 0;
  uint64_t beat_ns = 0;
  uint64_t period_ns = 0;
  uint64_t passes = 0;
  uint64_t obs_ns = 0;
  uint64_t frac_ns = 0;
  uint64_t recv_ns = 0;
  uint64_t busy_ns = 0;
  uint64_t vt_ns = 0;
  int64_t lead_ns = -1;
};

// Seqlock read of `pid`'s slot; `hint` caches its index.  False when the pid
// has no slot or the owner kept writing.
inline bool read_slot(const mivgpu_board_t* b, int pid, int* hint, View* out) {
  if (!b || pid <= 0) return false;
  for (int attempt = 0; attempt < 8; ++attempt) {
    const uint64_t s1 = __atomic_load_n(&b->seq, __ATOMIC_ACQUIRE);
    if (s1 & 1ull) {
      usleep(1);
      continue;
    }
    int k = (hint && *hint >= 0 && *hint < MIVGPU_BOARD_SLOTS && b->slots[*hint].pid == pid) ? *hint : -1;
    if (k < 0)
      for (int i = 0; i < MIVGPU_BOARD_SLOTS; ++i)
        if (b->slots[i].pid == pid) {
          k = i;
          break;
        }
    View v;
    v.owner_kind = b->owner_kind;
    v.owner_pid = b->owner_pid;
    v.beat_ns = b->beat_ns;
    v.period_ns = b->period_ns;
    v.passes = b->passes;
    if (k >= 0) {
      const mivgpu_board_slot_t& s = b->slots[k];
      v.occupancy = s.occupancy;
      v.obs_ns = s.obs_ns;
      v.frac_ns = s.frac_ns;
      v.recv_ns = s.recv_ns;
      v.busy_ns = s.busy_ns;
      v.vt_ns = s.vt_ns;
      v.lead_ns = s.lead_ns;
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    if (__atomic_load_n(&b->seq, __ATOMIC_RELAXED) != s1) continue;
    if (k < 0) return false;
    if (hint) *hint = k;
    *out = v;
    return true;
  }
  return false;
}

}  // namespace mivgpu_board

#endif  // MIVGPU_BOARD_H
