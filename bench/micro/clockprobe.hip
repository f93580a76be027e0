// Shader clock seen by a kernel: one wave per workgroup spins for ~spin_us of wall time and records
// (s_memtime delta, s_memrealtime delta); s_memtime counts shader-clock cycles, s_memrealtime the 100 MHz
// constant clock, so 100 * dclk / dreal is the shader clock in MHz over the spin.  Loaded with ctypes by
// bench/cold_start.py (a plain C entry point on the caller's stream; shares torch's HIP runtime).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -o bench/micro/libclockprobe.so bench/micro/clockprobe.hip
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(64) void k_clock(unsigned long long* __restrict__ out, unsigned spin_ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = r0, c1 = c0;
  while (r1 - r0 < spin_ticks) {
    r1 = __builtin_amdgcn_s_memrealtime();
    c1 = __builtin_amdgcn_s_memtime();
  }
  out[2 * blockIdx.x] = c1 - c0;
  out[2 * blockIdx.x + 1] = r1 - r0;
}

// out: 2 * wgs uint64 device words; returns the hipError_t of the launch
extern "C" int clock_probe(void* stream, unsigned long long* out, int wgs, int spin_us) {
  hipLaunchKernelGGL(k_clock, dim3(wgs), dim3(64), 0, static_cast<hipStream_t>(stream), out,
                     (unsigned)(spin_us * 100));
  return (int)hipGetLastError();
}
