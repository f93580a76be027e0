// Pulling bytes into this XCD's L2 from a workgroup that computes nothing (the prefetch workgroups of the H <= 128
// step launches, SplitStepArgs::pf_wgs): LDS-DMA of 16 bytes per lane into a slot nobody reads -- no VGPRs, no
// data dependence -- then one wait, because the slot must outlive the DMAs.  Its value is the cache state it leaves:
// the workgroups that read the same lines next on this XCD then hit L2 instead of the MALL (a first-touch miss on
// the critical path of every K loop).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mma_tile.h"

namespace cme {

// `rows` segments of `len` bytes, `ld` bytes apart, from byte `off` of `base` (32-bit offsets); this workgroup
// takes part `part` of `parts` of the 16-byte chunks.  512 threads; `slot`: 8 KB of LDS (1 KB per wave).
__device__ __forceinline__ void l2_touch(const void* base, int64_t off, int rows, int64_t ld, int64_t len, int part,
                                         int parts, char* slot) {
  const __amdgpu_buffer_rsrc_t r = make_rsrc(base);
  const int64_t a0 = off & ~int64_t(15), nch = (off + len - a0 + 15) >> 4, total = rows * nch;
  const int64_t per = (total + parts - 1) / parts, begin = part * per, end = begin + per < total ? begin + per : total;
  auto* ws = (__attribute__((address_space(3))) void*)(slot + (threadIdx.x >> 6) * 1024);
  for (int64_t i = begin + threadIdx.x; i < end; i += 512) {
    const int64_t row = i / nch, c = i - row * nch;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, ws, 16, (int)(row * ld + a0 + c * 16), 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The same pull with NO wait at the end: the caller's later vmcnt waits cover the DMAs (they count in issue order),
// and `slot` must be LDS nobody else writes or reads for the rest of the launch.
__device__ __forceinline__ void l2_touch_nowait(const void* base, int64_t off, int rows, int64_t ld, int64_t len,
                                                int part, int parts, char* slot) {
  const __amdgpu_buffer_rsrc_t r = make_rsrc(base);
  const int64_t a0 = off & ~int64_t(15), nch = (off + len - a0 + 15) >> 4, total = rows * nch;
  const int64_t per = (total + parts - 1) / parts, begin = part * per, end = begin + per < total ? begin + per : total;
  auto* ws = (__attribute__((address_space(3))) void*)(slot + (threadIdx.x >> 6) * 1024);
  for (int64_t i = begin + threadIdx.x; i < end; i += blockDim.x) {
    const int64_t row = i / nch, c = i - row * nch;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, ws, 16, (int)(row * ld + a0 + c * 16), 0, 0, 0);
  }
}

}  // namespace cme
