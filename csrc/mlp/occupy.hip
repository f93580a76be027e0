// TEST SUPPORT: hold CUs for a bounded time, so the in-launch hand-offs (the all-gather forward + head launches,
// fha_body.h and mlp_split.hip wide_head_ag) can be run with only part of their grid resident -- the hazard their
// bounded polls and the "apply nothing" error path exist for (tests/test_gpu_handoff.py).  Each workgroup asks for
// `lds_bytes` of LDS (the whole 160 KB of a CU: one workgroup per CU), so `wgs` workgroups keep `wgs` CUs busy; one
// thread per workgroup sleeps until s_memrealtime (100 MHz) passes the deadline, and the loop is also bounded by an
// iteration count, so every wave exits whatever the clock does.
#include "../common/hip_common.h"
#include "mlp_kernels.h"

#include <algorithm>

namespace cme {

namespace {
__global__ __launch_bounds__(64) void occupy_kernel(unsigned long long ticks, unsigned iters, int* running) {
  extern __shared__ char lds_hold[];
  if (threadIdx.x != 0) return;
  // (host-visible "the holder is running" word: one system-scope vector store by the first workgroup)
  if (running && blockIdx.x == 0) __hip_atomic_store(running, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned i = 0; i < iters; ++i) {
    if (__builtin_amdgcn_s_memrealtime() - t0 >= ticks) break;
    __builtin_amdgcn_s_sleep(127);
  }
  if (ticks == ~0ull) lds_hold[0] = 0;  // (never: keeps the LDS request honest)
}
}  // namespace

void occupy_cus(int wgs, int lds_bytes, int64_t ns, hipStream_t s, int* running) {
  CME_REQUIRE(wgs > 0 && lds_bytes >= 0 && lds_bytes <= 160 * 1024 && ns > 0 && ns <= 2000000000LL,
              "occupy_cus: 0 < wgs, 0 <= lds_bytes <= 160 KiB, 0 < ns <= 2 s");
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(occupy_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
  // s_sleep 127 is ~8 k cycles (~3.4 us at 2.4 GHz): the iteration bound is ~4x the requested time at that rate
  const unsigned iters = (unsigned)std::min<int64_t>(4 * (ns / 3000 + 1), 4000000);
  occupy_kernel<<<wgs, 64, lds_bytes, s>>>((unsigned long long)(ns / 10), iters, running);
  CME_LAUNCH_CHECK(s);
}

}  // namespace cme
