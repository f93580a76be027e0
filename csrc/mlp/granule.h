// Data-tagged granules: the in-launch hand-off form of MI355X_MICROARCH.md's price list row 'handoff-1to1'
// (cdna_hip_programming.md Guideline 16, R2).  A granule is 8 bytes {value (low 32), tag (high 32)} written by
// ONE sc1 store; the consumer polls the granules themselves until every tag is the launch's epoch, so the data
// is its own flag: no store drain, no counter add, no flag poll and no separate payload load.  Tags only grow
// (the callers derive the epoch from a monotonic per-tile counter), so granule buffers are never re-zeroed.
// Used by the all-gather forward + head launches: fha_body.h (H <= 128) and mlp_split.hip wide_head_ag.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../common/hip_common.h"

namespace cme {

using gran_t = unsigned long long;

// The launch-epoch add (one per workgroup at kernel entry; old / tm + 1 is the epoch), issued WITHOUT a wait.
// Written as __hip_atomic_fetch_add, hipcc's atomic optimizer turns the one-lane returning atomic into a wave
// reduction and waits for its result at once (s_waitcnt vmcnt(0) right after it): an L2 atomic round trip on
// the counter line that every workgroup of the column tile hits, before the wave issues a single K-loop load --
// and in the per-stage-barrier GEMM engines, on the critical path of every wave.  As inline asm the add is
// counted by the hardware in issue order like any load, so every later vmcnt wait covers it (waits only get
// stricter), and gran_epoch_wait names the result register so no use of it is scheduled above the wait.
__device__ __forceinline__ gran_t gran_epoch_add(gran_t* p, gran_t amount = 1) {
  gran_t old;
  asm volatile("global_atomic_add_x2 %0, %1, %2, off sc0" : "=v"(old) : "v"(p), "v"(amount) : "memory");
  return old;
}
__device__ __forceinline__ void gran_epoch_wait(gran_t& old) { asm volatile("s_waitcnt vmcnt(0)" : "+v"(old)::"memory"); }
__device__ __forceinline__ void gran_store(gran_t* p, float v, unsigned ep) {  // ONE 8-byte sc1 store
  __hip_atomic_store(p, ((gran_t)ep << 32) | __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ gran_t gran_load(const gran_t* p) {  // sc1 load (L2-served, never a stale L1 line)
  return __hip_atomic_load(const_cast<gran_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The same granules across GPUs (the xGMI owner-tile exchange, mlp_split.hip xp_*): ONE 8-byte system-scope
// store (sc0 sc1, write-through to the IPC-mapped fine-grained buffer of a peer, or of this rank) and a
// system-coherent load -- the peer's store reaches memory as one 8-byte write, so a load that sees the tag sees
// the value.
__device__ __forceinline__ void gran_store_sys(gran_t* p, float v, unsigned ep) {
  __hip_atomic_store(p, ((gran_t)ep << 32) | __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ gran_t gran_load_sys(const gran_t* p) {
  return __hip_atomic_load(const_cast<gran_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Poll the granules base[off + k * stride] (k < cnt <= N; lanes with !need take no part) until every tag is
// `ep`, then hand the values to f(k, value) in k order (0 for k >= cnt).  The N addresses are formed once,
// before the poll loop; a pass is N back-to-back global_load_dwordx2 sc1 and one wait.  Wave-uniform; false
// when the wave gave up after `limit_us` microseconds of wall time (s_memrealtime; f is then not called).
// A granule seen with the epoch is final for this launch (tags only grow), so later passes re-load only the
// granules still missing (the others' loads are masked off): every workgroup of the launch polls at once,
// and re-reading the already-arrived granules made the waiting workgroups' sc1 traffic compete with the
// stores and polls of the workgroups they wait for.  The first pass is unchanged: no added latency.
template <int N, class F>
__device__ __forceinline__ bool gran_poll(const gran_t* base, unsigned off, unsigned stride, int cnt, bool need,
                                          unsigned ep, uint32_t limit_us, F&& f) {
  static_assert(N <= 32, "ready mask");
  // the granule addresses, once: k >= cnt re-reads granule 0 (needed anyway, so its tag check is the same)
  const gran_t* p[N];
#pragma unroll
  for (int k = 0; k < N; ++k)
    p[k] = reinterpret_cast<const gran_t*>(reinterpret_cast<const char*>(base) +
                                           (off + (k < cnt ? (unsigned)k * stride : 0u)) * 8u);
  constexpr unsigned kAll = N == 32 ? ~0u : (1u << N) - 1u;
  bool done = !need;
  unsigned rdy = 0u;  // bit k: granule k carried the epoch in an earlier pass (x[k] is final)
  gran_t x[N];
  // The wall clock is read only once a pass has come back incomplete: s_memrealtime is a scalar-memory read, and
  // read up front its latency (~0.5 us, bench/stamps_push.py) sat in front of the first LDS access after a poll
  // that needed no second pass (lgkmcnt counts it with the LDS operations).
  uint64_t t0 = 0;
  const uint64_t limit = (uint64_t)limit_us * kTicksPerUs;
  for (uint32_t pass = 1;; ++pass) {
    if (!done) {
#pragma unroll
      for (int k = 0; k < N; ++k)
        if (!(rdy & (1u << k))) x[k] = gran_load(p[k]);
#pragma unroll
      for (int k = 0; k < N; ++k) rdy |= (unsigned)((unsigned)(x[k] >> 32) == ep) << k;
      done = rdy == kAll;
    }
    if (__all(done)) break;
    // (the clock -- a scalar-memory read and its wait -- every 8th pass only: the first passes, where a hand-off
    // normally completes, poll at full rate)
    if (pass == 1) t0 = wall_ticks();
    else if ((pass & 7) == 0 && wall_ticks() - t0 > limit) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  if (need) {
#pragma unroll
    for (int k = 0; k < N; ++k) f(k, k < cnt ? __builtin_bit_cast(float, (unsigned)x[k]) : 0.f);
  }
  return true;
}

// The same poll over an arbitrary set of granules base[off[k]], k < N, of which this lane needs those whose bit is
// set in `need` (the others take no load and count as arrived); f(k, value) for every needed k in k order.  One pass
// issues every missing granule's load back to back, so a lane gathering several items pays ONE memory round trip
// per pass, not one per item.  Wave-uniform; false after `limit_us` of wall time (f not called).
template <int N, class F>
__device__ __forceinline__ bool gran_poll_set(const gran_t* base, const unsigned (&off)[N], unsigned need, unsigned ep,
                                              uint32_t limit_us, F&& f) {
  static_assert(N <= 32, "ready mask");
  constexpr unsigned kAll = N == 32 ? ~0u : (1u << N) - 1u;
  unsigned rdy = ~need & kAll;
  gran_t x[N];
  uint64_t t0 = 0;  // (read once a pass comes back incomplete: gran_poll)
  const uint64_t limit = (uint64_t)limit_us * kTicksPerUs;
  for (uint32_t pass = 1;; ++pass) {
    if (rdy != kAll) {
#pragma unroll
      for (int k = 0; k < N; ++k)
        if (!(rdy & (1u << k))) x[k] = gran_load(base + off[k]);
#pragma unroll
      for (int k = 0; k < N; ++k)
        if (!(rdy & (1u << k))) rdy |= (unsigned)((unsigned)(x[k] >> 32) == ep) << k;
    }
    if (__all(rdy == kAll)) break;
    if (pass == 1) t0 = wall_ticks();
    else if ((pass & 7) == 0 && wall_ticks() - t0 > limit) return false;
    __builtin_amdgcn_s_sleep(2);
  }
#pragma unroll
  for (int k = 0; k < N; ++k)
    if (need & (1u << k)) f(k, __builtin_bit_cast(float, (unsigned)x[k]));
  return true;
}

}  // namespace cme
