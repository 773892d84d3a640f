// mivgpu shared-region ABI (version 1.1; 1.1 names two spare util fields).
//
// One file-backed region per container, mmap'd MAP_SHARED by every process of
// the container that loads libmivgpu.so and, from the host side, by the node's
// vgpu-monitor.  It is the AMD-native counterpart of HAMi-core's
// `shared_region_t` whose Go mirror lives in the reference at
// pkg/monitor/nvidia/v1/spec.go:24-87 (offsets pinned by v1/spec_test.go:40-70).
//
// Design choices that differ from the reference on purpose:
//   * an aggregate per-device usage counter (`dev_used`) so an allocation check
//     is O(1) instead of a sweep over 1024 process slots;
//   * the header is small and cache-line aligned, the process table sits at the
//     end, so the monitor's hot fields (limits, switches) share few lines;
//   * a robust, process-shared pthread mutex guards slot ownership (a crashed
//     holder is recovered with EOWNERDEAD instead of a semaphore leak);
//   * cu_limit is a percentage of the device's CUs; cu_mask_count records how
//     many CUs the device plugin gave the container through HSA_CU_MASK (0 = no
//     spatial mask), which decides whether the temporal governor has to run.
//
// Layout is pinned by tests/test_shim_cpu.py::test_abi_offsets_match_c_layout
// against k8s_vgpu_scheduler_amd/monitor/region.py (ctypes mirror) via the
// exported mivgpu_abi_offsetof() of libmivgpu.so.
#ifndef MIVGPU_SHARED_REGION_H
#define MIVGPU_SHARED_REGION_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIVGPU_MAGIC 0x4D495647u /* 'MIVG' */
#define MIVGPU_MAJOR 1
#define MIVGPU_MINOR 1
#define MIVGPU_MAX_DEVICES 16
#define MIVGPU_MAX_PROCS 1024
#define MIVGPU_UUID_LEN 96
#define MIVGPU_LOCK_BYTES 64

/* Process slot status. */
#define MIVGPU_SLOT_FREE 0
#define MIVGPU_SLOT_ACTIVE 1

typedef struct {
  uint64_t context;  /* HIP context / runtime-internal bytes (estimated)   */
  uint64_t module;   /* code objects                                       */
  uint64_t buffer;   /* hipMalloc & friends                                */
  uint64_t vmm;      /* hipMemCreate physical handles (expandable segments) */
  uint64_t total;    /* context+module+buffer+vmm                          */
  uint64_t peak;     /* high-water mark of total                           */
  uint64_t unused[2];
} mivgpu_mem_t; /* 64 B */

typedef struct {
  uint64_t launches;      /* kernel + graph launches seen by the shim       */
  uint64_t busy_ns;       /* GPU busy time measured by the governor gate    */
  uint64_t throttled_ns;  /* time gate kernels held the stream              */
  uint64_t gates;         /* gate kernels enqueued                          */
  uint64_t util_pct;      /* GPU share received over the last >= 0.5 s, %   */
  uint64_t share_ns;      /* GPU time received: integral of the process's   */
                          /* share of resident wavefronts (KFD occupancy)   */
  uint64_t occupancy;     /* last KFD cu_occupancy sample of the process    */
  uint64_t share_ppm;     /* governor's measured share while contending, ppm */
} mivgpu_util_t; /* 64 B */

typedef struct {
  int32_t pid;       /* pid inside the container's pid namespace           */
  int32_t hostpid;   /* pid on the host (filled by the monitor if known)    */
  int32_t status;    /* MIVGPU_SLOT_*                                      */
  int32_t priority;  /* HIP_TASK_PRIORITY of the process                    */
  uint64_t start_ns;
  uint64_t heartbeat_ns;
  uint64_t unused[5];
  mivgpu_mem_t used[MIVGPU_MAX_DEVICES];
  mivgpu_util_t util[MIVGPU_MAX_DEVICES];
} mivgpu_proc_slot_t; /* 2112 B */

typedef struct {
  uint32_t magic;
  int32_t major_version;
  int32_t minor_version;
  int32_t initialized;            /* 1 once the creator finished init          */
  uint64_t owner_pid;             /* pid that created the region               */
  uint8_t lock[MIVGPU_LOCK_BYTES];/* robust pshared pthread_mutex_t             */
  uint64_t num_devices;
  int32_t procnum;                /* slots in use (high-water index+1)         */
  int32_t utilization_switch;     /* monitor -> lib: 1 = enforce core limit    */
  int32_t recent_kernel;          /* lib sets >0 on launch; monitor -1 = block */
  int32_t priority;               /* container task priority                   */
  int64_t last_kernel_time;       /* unix seconds of the most recent launch     */
  int32_t core_policy;            /* 0 default, 1 force, 2 disable             */
  int32_t oversubscribe;          /* 1 = allow > limit (host-spill semantics)  */
  uint64_t unused0[2];
  char uuids[MIVGPU_MAX_DEVICES][MIVGPU_UUID_LEN];
  uint64_t mem_limit[MIVGPU_MAX_DEVICES];     /* bytes, 0 = unlimited          */
  uint64_t cu_limit[MIVGPU_MAX_DEVICES];      /* percent 1..100, 0 = unlimited */
  uint64_t cu_mask_count[MIVGPU_MAX_DEVICES]; /* CUs granted by HSA_CU_MASK    */
  uint64_t dev_used[MIVGPU_MAX_DEVICES];      /* aggregate bytes in use        */
  uint64_t unused1[16];
  mivgpu_proc_slot_t procs[MIVGPU_MAX_PROCS];
} mivgpu_shared_region_t;

/* Host-owned control file (version 1).
 *
 * The shared region above sits in a directory the container mounts
 * read-write, so a verdict the monitor writes there (recent_kernel = -1) is
 * one store away from being cleared by the tenant.  The control file is the
 * monitor's channel instead: created by the device plugin's Allocate under
 * $HOOK_PATH/vgpu/control/<pod>_<ctr>.ctl on the host, bind-mounted
 * READ-ONLY into the container (named by the grant key MIVGPU_CONTROL_FILE),
 * mapped PROT_READ by the shim, written in place by the monitor each pass.
 *
 * The verdicts hold only while the lease the monitor renews every pass is
 * live (CLOCK_REALTIME, shared by host and container): a dead monitor cannot
 * leave a tenant parked forever. */
#define MIVGPU_CTL_MAGIC 0x4D495643u /* 'MIVC' */
#define MIVGPU_CTL_VERSION 1

typedef struct {
  uint32_t magic;
  int32_t version;
  uint64_t seq;                   /* monitor passes that wrote the file          */
  int64_t lease_until_ns;         /* CLOCK_REALTIME; verdicts void after it      */
  int32_t block;                  /* 1 = park every launch                        */
  int32_t utilization_switch;     /* 1 = time-slice to the core limit under a mask */
  int32_t over_grant;             /* 1 = host truth found the container over its HBM grant */
  int32_t reserved0;
  uint64_t host_excess[MIVGPU_MAX_DEVICES]; /* bytes KFD holds beyond the region's usage counter,
                                               charged by the shim's quota check */
  uint64_t unused[43];
} mivgpu_control_t; /* 512 B */

/* Share board (version 1): ONE wave-occupancy sampler per GPU.
 *
 * The governor charges a tenant the GPU time it receives: its share of the
 * resident wavefronts KFD reports per process.  Sampled by every tenant on
 * its own clock, those shares are not comparable across tenants (each one's
 * samples land at times correlated with its own work).  The reference
 * serialises utilisation sampling across containers through the host lock
 * directory /tmp/vgpulock (pkg/device-plugin/nvidiadevice/nvinternal/plugin/
 * server.go:853-864); here one owner per GPU reads EVERY process's
 * cu_occupancy in the same pass and publishes, per KFD pid, the integrals the
 * tenants charge from:
 *   obs_ns  -- time over passes in which the process was not sitting in a
 *              governor gate (cu_occupancy 0 or > one CU unit),
 *   frac_ns -- over the same passes, the integral of its share of the GPU:
 *              w / W (w = its waves, W = all processes' waves), 1 when no
 *              process has waves resident (its dispatch gaps are its own),
 *   recv_ns -- the integral of w / W (GPU time received; utilisation),
 *   busy_ns -- time with its waves resident,
 *   vt_ns   -- its virtual time while the GPU is fully subscribed (below):
 *              the integral of its presence (1 / the processes with waves
 *              resident, while it has) / its core limit,
 *   lead_ns -- -1 while the GPU is not fully subscribed, else its GPU time
 *              received beyond its weighted fair share: (vt - the mean vt of
 *              the running contenders) x its limit, >= 0.
 * A tenant charges (delta frac_ns / delta obs_ns) x its own non-held time.
 * Fully subscribed: the core limits of the processes contending for the GPU
 * (owing work or held in a gate, within 20 ms; a process without flags counts
 * as 100 %) add up to the whole GPU.  Then every tenant's token bucket is at
 * equilibrium (the time they are charged sums to the time they accrue), so a
 * bucket balance -- and any debt carried in from a phase alone -- never
 * recovers and holds cascade; the tenants are held on their lead instead
 * (weighted fair sharing, work-conserving: the tenants behind always run).
 *
 * The owner is the node sampler (mivgpu-boardd, run by the monitor; the
 * board directory is mounted READ-ONLY into containers, so no tenant can
 * write its own share) or, where the directory is writable and no node
 * sampler is live, the shim that holds flock() on <dir>/gpu-<id>.owner.
 * File: <dir>/gpu-<kfd gpu_id>.board.  Writes are bracketed by `seq`
 * (odd while a pass writes: a seqlock). */
#define MIVGPU_BOARD_MAGIC 0x4D495642u /* 'MIVB' */
#define MIVGPU_BOARD_VERSION 2
#define MIVGPU_BOARD_SLOTS 64
#define MIVGPU_BOARD_OWNER_NONE 0
#define MIVGPU_BOARD_OWNER_NODE 1
#define MIVGPU_BOARD_OWNER_SHIM 2

typedef struct {
  int32_t pid;        /* KFD (host) pid, 0 = free slot                        */
  int32_t occupancy;  /* cu_occupancy at the last pass                        */
  uint64_t seen_ns;   /* CLOCK_MONOTONIC of the last pass that listed it      */
  uint64_t obs_ns;
  uint64_t frac_ns;
  uint64_t recv_ns;
  uint64_t busy_ns;
  uint64_t vt_ns;
  int64_t lead_ns;
} mivgpu_board_slot_t; /* 64 B */

typedef struct {
  uint32_t magic;
  int32_t version;
  int32_t gpu_id;         /* KFD gpu_id of the GPU                            */
  int32_t owner_kind;     /* MIVGPU_BOARD_OWNER_*                             */
  int32_t owner_pid;      /* pid of the owner (its own namespace)             */
  int32_t nslots;         /* slots in use (high-water index + 1)              */
  uint64_t seq;           /* seqlock                                          */
  uint64_t beat_ns;       /* CLOCK_MONOTONIC of the last completed pass       */
  uint64_t period_ns;     /* the owner's current sampling period              */
  uint64_t passes;
  uint64_t want_fast_ns;  /* writable boards: a governed tenant's latest ask for fast passes */
  uint64_t busy_ns;       /* time with any process's waves resident           */
  uint64_t pass_ns;       /* cost of the last pass                            */
  uint64_t sub_passes;    /* passes with the backlogged weights filling the GPU */
  uint64_t fair_passes;   /* passes in fair-share mode                        */
  uint64_t unused[4];
  mivgpu_board_slot_t slots[MIVGPU_BOARD_SLOTS];
} mivgpu_board_t; /* 128 + 4096 B */

/* Tenant flags (version 2): <dir>/flags/gpu-<kfd gpu_id>.flags, the one
 * file of the board directory the tenants write (a read-write mount nested in
 * the read-only board mount).  Each shim claims an entry for its KFD pid and
 * publishes, every sampler pass, whether its streams sit in a governor gate
 * (HELD: its one resident wave per held stream is not work), whether it
 * owes GPU work (OWES: split the time nobody has waves resident) and its core
 * limit (the weight of its fair share).  The owner
 * reads them in its pass; a process without a fresh entry is judged from its
 * occupancy alone (one CU unit = a gate).
 *
 * Production (a node sampler): every container has a flags
 * directory of its OWN -- host <dir>/flags/<pod uid>_<container>/, mounted
 * read-write at MIVGPU_BOARD_FLAGS_DIR -- and the monitor writes, next to the
 * node limits, <dir>/gpu-<id>.owners: which container each host pid belongs
 * to (host truth).  The node sampler reads a pid's flags only from the file
 * of the container that owns it, so a tenant cannot publish entries for a
 * neighbour's pid or fill the slots its neighbours publish in; a pid's
 * weight is the node-written limit whenever the monitor wrote one.  The node
 * sampler never creates, truncates or follows a symlink to any file under a
 * tenant-writable directory.  Without a node sampler (hand-run slices, the
 * bench) the tenants share <dir>/flags/gpu-<id>.flags as before.
 * GATED: the tenant's governor gated this device within the last second --
 * the node sampler runs its fast passes only while some tenant is gated. */
#define MIVGPU_FLAGS_MAGIC 0x4D495646u /* 'MIVF' */
#define MIVGPU_FLAGS_VERSION 2
#define MIVGPU_FLAGS_SLOTS 256
#define MIVGPU_FLAG_HELD 1
#define MIVGPU_FLAG_OWES 2
#define MIVGPU_FLAG_GATED 4

typedef struct {
  int32_t pid;        /* KFD pid, 0 = free                                   */
  int32_t state;      /* MIVGPU_FLAG_*                                       */
  uint64_t stamp_ns;  /* CLOCK_MONOTONIC of the last publish                 */
  uint32_t limit_ppm; /* core limit, ppm of the GPU (0 = none: 100 %)        */
  uint32_t reserved;
  uint64_t unused;
} mivgpu_flag_t; /* 32 B */

typedef struct {
  uint32_t magic;
  int32_t version;
  int32_t gpu_id;
  int32_t reserved;
  uint64_t unused[6];
  mivgpu_flag_t flags[MIVGPU_FLAGS_SLOTS];
} mivgpu_board_flags_t; /* 64 + 8192 B */

/* Node-written core limits (version 1): <dir>/gpu-<kfd gpu_id>.limits, in
 * the read-only board mount.  The monitor writes, every feedback pass, the
 * core limit of each host pid it attributes to a granted container on the GPU
 * (grant files x the pod's processes, host truth); the owner pass weighs a
 * process with this limit whenever there is one (its flags' limit only
 * otherwise), so a tenant cannot move its own or a neighbour's fair share by
 * publishing a limit.  Written under a private name and renamed into place.
 *
 * Owners (text, next to it): <dir>/gpu-<kfd gpu_id>.owners --
 *   "MIVGPU-OWNERS 1 <gpu_id>\n" then "<host pid> <pod uid>_<container>\n"
 * per process host truth attributes; the key names the container's flags
 * directory <dir>/flags/<key>/ (characters [A-Za-z0-9_.-], at most 127). */
#define MIVGPU_OWNERS_MAX 1024
#define MIVGPU_OWNER_KEY_MAX 128
#define MIVGPU_LIMITS_MAGIC 0x4D49564Cu /* 'MIVL' */
#define MIVGPU_LIMITS_VERSION 1
#define MIVGPU_LIMITS_MAX 1024

typedef struct {
  int32_t pid;        /* host (KFD) pid                                       */
  uint32_t limit_ppm; /* core limit of its container on this GPU              */
} mivgpu_limit_entry_t;

typedef struct {
  uint32_t magic;
  int32_t version;
  int32_t gpu_id;
  int32_t count;      /* entries that follow (<= MIVGPU_LIMITS_MAX)           */
  mivgpu_limit_entry_t entries[];
} mivgpu_board_limits_t;

/* Field ids understood by mivgpu_abi_offsetof() (exported by libmivgpu.so). */
enum {
  MIVGPU_F_MAGIC = 0,
  MIVGPU_F_LOCK,
  MIVGPU_F_NUM_DEVICES,
  MIVGPU_F_PROCNUM,
  MIVGPU_F_UTIL_SWITCH,
  MIVGPU_F_RECENT_KERNEL,
  MIVGPU_F_PRIORITY,
  MIVGPU_F_LAST_KERNEL_TIME,
  MIVGPU_F_CORE_POLICY,
  MIVGPU_F_UUIDS,
  MIVGPU_F_MEM_LIMIT,
  MIVGPU_F_CU_LIMIT,
  MIVGPU_F_CU_MASK_COUNT,
  MIVGPU_F_DEV_USED,
  MIVGPU_F_PROCS,
  MIVGPU_F_SIZEOF_REGION,
  MIVGPU_F_SIZEOF_SLOT,
  MIVGPU_F_SLOT_USED,
  MIVGPU_F_SLOT_UTIL,
  MIVGPU_F_CTL_SEQ,
  MIVGPU_F_CTL_LEASE,
  MIVGPU_F_CTL_BLOCK,
  MIVGPU_F_CTL_SWITCH,
  MIVGPU_F_CTL_OVER,
  MIVGPU_F_CTL_EXCESS,
  MIVGPU_F_SIZEOF_CTL,
  MIVGPU_F_BOARD_SEQ,
  MIVGPU_F_BOARD_BEAT,
  MIVGPU_F_BOARD_SLOTS,
  MIVGPU_F_SIZEOF_BOARD,
  MIVGPU_F_SIZEOF_BOARD_SLOT,
  MIVGPU_F_FLAGS_ENTRIES,
  MIVGPU_F_SIZEOF_FLAGS,
  MIVGPU_F_COUNT
};

#ifdef __cplusplus
}
#endif

#endif /* MIVGPU_SHARED_REGION_H */
