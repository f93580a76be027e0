// Shared HIP helpers for every gfx950 kernel in this repository.
//
// Replaces the reference's per-kernel `check_launch` (device-wide sync + error
// poll after EVERY kernel, fpcode/inc/gpu_func.h:13-22) with an asynchronous
// launch check.  A debug-only full sync is available through the env flag
// CME_SYNC_CHECK=1 (read once), mirroring SURVEY §2.1 F2.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace cme {

[[noreturn]] inline void hip_fail(hipError_t e, const char* what, const char* file, int line) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "HIP error %d (%s) in %s at %s:%d", (int)e,
                hipGetErrorString(e), what, file, line);
  throw std::runtime_error(buf);
}

inline bool sync_check_enabled() {
  static int v = [] {
    const char* s = std::getenv("CME_SYNC_CHECK");
    return (s && s[0] == '1') ? 1 : 0;
  }();
  return v != 0;
}

}  // namespace cme

#define HIP_CHECK(expr)                                                  \
  do {                                                                   \
    hipError_t _e = (expr);                                              \
    if (_e != hipSuccess) ::cme::hip_fail(_e, #expr, __FILE__, __LINE__); \
  } while (0)

// Post-launch check: catches launch-configuration errors without a sync.
#define CME_LAUNCH_CHECK(stream)                                          \
  do {                                                                    \
    hipError_t _e = hipGetLastError();                                    \
    if (_e != hipSuccess) ::cme::hip_fail(_e, "kernel launch", __FILE__, __LINE__); \
    if (::cme::sync_check_enabled()) HIP_CHECK(hipStreamSynchronize(stream)); \
  } while (0)

#define CME_REQUIRE(cond, msg)                                  \
  do {                                                          \
    if (!(cond)) throw std::invalid_argument(std::string(msg)); \
  } while (0)

namespace cme {

constexpr int kWave = 64;  // CDNA wavefront width (gfx950): never 32.

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Wall-clock bounds for every wait on another workgroup or another GPU (a peer's flag, an in-launch hand-off):
// s_memrealtime is the constant 100 MHz counter, so a bound is a duration, not a poll count whose real length
// depends on the sleep, the poll's memory latency and how loaded the fabric is.  A wait that outlasts its bound
// sets an error word and the kernel applies nothing (never a hang).
constexpr uint64_t kTicksPerUs = 100;
constexpr uint64_t kPeerWaitUs = 2'000'000;  // xGMI peer waits: 2 s (a stalled or dead rank)
constexpr uint64_t kHandoffWaitUs = 50'000;  // in-launch hand-offs between co-resident workgroups: 50 ms
__device__ __forceinline__ uint64_t wall_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md
// §5 "XCD swizzle must be bijective"): consecutive logical tiles land on the
// same XCD so neighbouring tiles share that XCD's L2.  Speed only.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  if (nwg <= 8) return orig;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

inline int device_cu_count() {  // CUs of the current device, cached per device
  static int cached[64] = {0};
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return 0;
  if (!cached[dev]) HIP_CHECK(hipDeviceGetAttribute(&cached[dev], hipDeviceAttributeMultiprocessorCount, dev));
  return cached[dev];
}

}  // namespace cme
