// mivgpu governor: device-side token-bucket gate for CU-time throttling (gfx950).
//
// Reference behaviour being replaced: HAMi-core throttles the SM share of a
// container by blocking the HOST thread inside cuLaunchKernel on a token bucket
// refilled from NVML utilisation samples (contract inferred in SURVEY.md §2.6
// from pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:837 and
// cmd/vGPUmonitor/feedback.go:74-134).
//
// MI355X-first design: the shim enqueues this one-wave kernel on the SAME
// stream, in front of a user launch, at most once per `min interval` of host
// submission.  With a KFD view of the GPU (the normal case) the bucket lives
// on the host and the gate only enforces it (host_bucket_gate below).
// Without one, the gate keeps the bucket itself (device-bucket mode): it
//   1. reads the 100 MHz constant clock (s_memrealtime -> 10 ns ticks),
//   2. debits the GPU time the process received since this stream's previous
//      gate from a bucket shared by all its streams on this device: the
//      stream's busy wall time (in-order stream => everything between
//      max(previous gate exit, first submission) and now was its work),
//      weighted by the process's share of the GPU while busy.  The share is
//      measured by the shim's sampler from KFD's per-process wave counts
//      (SPI_CSQ_WF_ACTIVE_COUNT): own / (own + every other process) averaged
//      over the samples in which the process was contending, published in
//      pinned host memory and read here at execution time.  A tenant alone is
//      charged its wall time, N tenants time-sliced or co-resident are each
//      charged ~1/N, a CU-masked tenant at most its CU fraction -- the
//      analogue of HAMi-core charging NVML per-process SM utilisation.
//      Without a KFD view the share is 1 (plain wall time),
//   3. refills the bucket at `rate_ppm` of wall time (the container's share),
//   4. if the bucket is in debt, holds the stream on-device (s_sleep loop)
//      until the debt is repaid -- other tenants' queues run meanwhile -- and
//      publishes the hold's end so the sampler does not count the gate's own
//      resident wave as consumption.
// No host thread ever blocks, launches stay asynchronous, and graph replays are
// gated by the same mechanism.  Every spin is bounded (max_hold_ns), so a gate
// can never wedge a queue.
//
// Memory model (MI355X_MICROARCH.md "Workgroup dispatch ... visibility"): gates
// of different streams can run on different XCDs, so every access to the
// shared state is an agent-scope atomic, the critical section is bracketed by
// acquire/release on the lock word, and only lane 0 of one wave touches it.
// Host memory (fine-grained, coherent) is read and written with system-scope
// atomics only.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MIVGPU_GATE_SLOTS 64

struct mivgpu_gate_state {
  unsigned long long lock;
  long long last_ns;       // device ns at which the bucket was last settled
  long long tokens_ns;     // balance in ns of GPU time (may go negative)
  unsigned long long busy_total_ns;
  unsigned long long held_total_ns;
  unsigned long long gates;
  unsigned long long pad[2];
  long long slot_exit_ns[MIVGPU_GATE_SLOTS];  // per-stream last gate exit
};

// Written with plain system-visible stores into fine-grained host memory so
// the shim's bookkeeping thread can read stats without synchronising a stream.
struct mivgpu_gate_trace_entry {
  long long now_ns, submit_ns, prev_exit_ns, busy_ns, hold_ns, tokens_ns;
  long long slot, pad;
};
#define MIVGPU_GATE_TRACE 128
struct mivgpu_gate_host_stats {
  unsigned long long busy_total_ns;
  unsigned long long held_total_ns;
  unsigned long long gates;
  long long last_now_ns;
  long long last_tokens_ns;
  long long last_hold_ns;
  unsigned long long share_ppm;  // HOST-written by the sampler: the process's measured GPU share, ppm
  long long host_tokens_ns;      // HOST-written by the sampler: the bucket balance (host-bucket mode)
  mivgpu_gate_trace_entry trace[MIVGPU_GATE_TRACE];  // ring, index = gates % N
  long long hold_end_ns[MIVGPU_GATE_SLOTS];          // device ns at which a slot's hold ends
  long long hold_start_ns[MIVGPU_GATE_SLOTS];        // device ns at which its latest hold began
  long long held_cum_ns[MIVGPU_GATE_SLOTS];          // its completed holds, total ns
};

__device__ __forceinline__ long long rt_ns() {
  return (long long)__builtin_amdgcn_s_memrealtime() * 10ll;
}

__device__ __forceinline__ long long aload(long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void astore(long long* p, long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long aloadu(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void astoreu(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bounded spin lock (acquire).  If it cannot be taken in ~0.5 s something is
// badly wrong (a gate died holding it); proceed unlocked rather than hang.
__device__ __forceinline__ bool gate_lock(mivgpu_gate_state* st) {
  for (unsigned int spins = 0; spins < (1u << 17); ++spins) {
    unsigned long long expected = 0ull;
    if (__hip_atomic_compare_exchange_strong(&st->lock, &expected, 1ull, __ATOMIC_ACQUIRE,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      return true;
    __builtin_amdgcn_s_sleep(8);
  }
  return false;
}

__device__ __forceinline__ long long host_load(long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Host-bucket mode (flags bit 1, used whenever the shim has a KFD view of the
// GPU): the shim's sampler integrates the share of the GPU this process
// actually receives -- own resident waves / all resident waves, every ~2 ms --
// against its entitlement (rate x wall time) and publishes the balance.  The
// gate only enforces it: in debt, it holds the stream until the balance is
// back to zero (the sampler refills it while the process has no waves
// resident), at most max_hold_ns per gate; larger debts are repaid over the
// following gates.  Time the process spends co-resident with other tenants is
// charged at the share it got, and time it spends queued or idle is not
// charged at all -- the sample-time bias of charging a whole batch at one
// share estimate is gone.  The gate publishes its holds
// (start, end, running total per slot) so that the sampler takes the exact
// held time out of each interval instead of classifying the interval by the
// state it sees at the sample: releases follow the sampler's refills, so a
// sample lands in the next hold far more often than in the batch between
// (measured: 0.31 of the GPU at a 25 % limit before, the batches uncharged).
__device__ void host_bucket_gate(mivgpu_gate_state* st, mivgpu_gate_host_stats* hs, int slot,
                                 long long max_hold_ns, unsigned int flags) {
  const long long t0 = rt_ns();
  long long tokens = host_load(&hs->host_tokens_ns);
  long long t = t0;
  if (tokens < 0) {
    // "holding since / until at most" markers: the sampler discounts the
    // gate's own resident wave while it sits here, and takes the exact held
    // time out of the interval it charges (start, then end: the sampler reads
    // end, then start)
    __hip_atomic_store(&hs->hold_start_ns[slot], t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&hs->hold_end_ns[slot], t0 + max_hold_ns, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    while (tokens < 0 && t < t0 + max_hold_ns) {
      for (int k = 0; k < 4; ++k) __builtin_amdgcn_s_sleep(127);   // ~14 us between host reads
      tokens = host_load(&hs->host_tokens_ns);
      t = rt_ns();
    }
    // end, then the running total (the sampler reads the total first: a race
    // can only delay a hold's count to its next sample, never count it twice)
    __hip_atomic_store(&hs->hold_end_ns[slot], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const long long cum = __hip_atomic_load(&hs->held_cum_ns[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&hs->held_cum_ns[slot], cum + (t - t0), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const long long hold = t - t0;
  const bool locked = gate_lock(st);
  astore(&st->slot_exit_ns[slot], t);
  const unsigned long long held_tot = aloadu(&st->held_total_ns) + (unsigned long long)hold;
  const unsigned long long gates = aloadu(&st->gates) + 1ull;
  astoreu(&st->held_total_ns, held_tot);
  astoreu(&st->gates, gates);
  if (locked) __hip_atomic_store(&st->lock, 0ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&hs->held_total_ns, held_tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&hs->gates, gates, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (flags & 1u) {
    mivgpu_gate_trace_entry* e = &hs->trace[(gates - 1) % MIVGPU_GATE_TRACE];
    e->now_ns = t0;
    e->submit_ns = -1;
    e->prev_exit_ns = -1;
    e->busy_ns = 0;
    e->hold_ns = hold;
    e->tokens_ns = tokens;
    e->slot = slot;
  }
}

extern "C" __global__ void __launch_bounds__(64)
mivgpu_gate(mivgpu_gate_state* st, mivgpu_gate_host_stats* hs, long long submit_ns,
            int slot, unsigned int rate_ppm, long long cap_ns, long long max_hold_ns, unsigned int use_share,
            unsigned int flags) {
  if (threadIdx.x != 0) return;
  if (slot < 0 || slot >= MIVGPU_GATE_SLOTS) slot = 0;
  if (rate_ppm == 0) rate_ppm = 1;
  if ((flags & 2u) && hs) {
    host_bucket_gate(st, hs, slot, max_hold_ns, flags);
    return;
  }

  // Device-bucket mode (no KFD view: the busy wall time is the charge).
  const bool locked = gate_lock(st);

  const long long now = rt_ns();
  long long last = aload(&st->last_ns);
  long long tokens = aload(&st->tokens_ns);
  if (last == 0) {  // first gate of the process on this device: an empty bucket (bursts are earned)
    last = now;
    tokens = 0;
  }
  long long elapsed = now - last;
  if (elapsed < 0) elapsed = 0;  // bucket already settled into the future by a hold
  tokens += (long long)(((__int128)elapsed * rate_ppm) / 1000000);
  if (tokens > cap_ns) tokens = cap_ns;

  // Busy wall time of this stream since its previous gate.
  // submit_ns < 0: nothing was submitted on this stream since its previous
  // gate, so the time since then was idle, not busy.
  const long long prev_exit = aload(&st->slot_exit_ns[slot]);
  long long begin = prev_exit > submit_ns ? prev_exit : submit_ns;
  if (submit_ns < 0 || begin <= 0 || begin > now) begin = now;
  long long busy = now - begin;
  // Weight by the measured share (ppm) as of NOW, read from host memory: the
  // host can run far ahead of a held stream (hundreds of queued graph
  // launches), so a share captured at enqueue time would be stale (measured:
  // 2 x 50 % tenants 0.86 of unthrottled, fairness 0.83, vs 1.01 / 0.999).
  // 0 = no sample yet (or no KFD view) -> plain wall time.
  if (use_share && hs) {
    const unsigned long long share =
        __hip_atomic_load(&hs->share_ppm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (share > 0 && share < 1000000ull) busy = (long long)(((__int128)busy * (long long)share) / 1000000);
  }
  tokens -= busy;
  // Bound the debt to one burst: a single mis-measured interval can never
  // stall a tenant for longer than cap / rate.
  if (tokens < -cap_ns) tokens = -cap_ns;

  long long hold = 0;
  if (tokens < 0) {
    hold = (long long)(((__int128)(-tokens) * 1000000) / rate_ppm);
    if (hold > max_hold_ns) hold = max_hold_ns;
    tokens += (long long)(((__int128)hold * rate_ppm) / 1000000);
  }
  const long long t_end = now + hold;
  astore(&st->last_ns, t_end);
  astore(&st->tokens_ns, tokens);
  astore(&st->slot_exit_ns[slot], t_end);
  const unsigned long long busy_tot = aloadu(&st->busy_total_ns) + (unsigned long long)busy;
  const unsigned long long held_tot = aloadu(&st->held_total_ns) + (unsigned long long)hold;
  const unsigned long long gates = aloadu(&st->gates) + 1ull;
  astoreu(&st->busy_total_ns, busy_tot);
  astoreu(&st->held_total_ns, held_tot);
  astoreu(&st->gates, gates);
  if (locked) __hip_atomic_store(&st->lock, 0ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);

  // Publish to host memory (system scope; the host only reads monotone
  // counters and hold ends): three counters, the hold end when holding (the
  // sampler discounts the gate's own resident wave), and -- only with
  // MIVGPU_GATE_TRACE (flags bit 0) -- the last-state fields and trace ring.
  // Each system-scope store is a fabric write the gate's completion waits for:
  // fewer of them = a cheaper gate (measured 6.3 -> see profiles §25).
  if (hs) {
    __hip_atomic_store(&hs->busy_total_ns, busy_tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&hs->held_total_ns, held_tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&hs->gates, gates, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (hold > 0)
      __hip_atomic_store(&hs->hold_end_ns[slot], t_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (flags & 1u) {
      __hip_atomic_store(&hs->last_now_ns, now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&hs->last_tokens_ns, tokens, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&hs->last_hold_ns, hold, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      mivgpu_gate_trace_entry* e = &hs->trace[(gates - 1) % MIVGPU_GATE_TRACE];
      e->now_ns = now;
      e->submit_ns = submit_ns;
      e->prev_exit_ns = prev_exit;
      e->busy_ns = busy;
      e->hold_ns = hold;
      e->tokens_ns = tokens;
      e->slot = slot;
    }
  }

  // Hold the stream on-device.  ~3.4 us per s_sleep(127) at 2.4 GHz; bounded
  // by max_hold_ns through t_end.
  while (rt_ns() < t_end) __builtin_amdgcn_s_sleep(127);
}

// Clock calibration: device realtime (ns) for the host<->device offset.
extern "C" __global__ void __launch_bounds__(64) mivgpu_clock(long long* out) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(out, rt_ns(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
