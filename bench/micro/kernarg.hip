// What does a kernel's argument block cost on the critical path of a launch?  The headline step's two launches
// pass ~0.6 KB of arguments by value (SplitStepArgs + HeadArgs); a stream launch writes them into a fresh slot of
// the runtime's kernarg pool every time, so the first scalar loads of every workgroup miss in the XCD's L2, while a
// replayed graph reuses the same argument memory launch after launch.  Back-to-back launches of a trivial kernel
// (256 workgroups x 512 threads; thread 0 reads one word from each of the block's 64-byte lines):
//   kA  -- 512 B by value, stream launches;       kB -- one pointer to the same 512 B kept in device memory;
//   kA in a captured graph (the same nodes replayed).
// Per-launch time = event time / launches.  Built twice: SPIN_TICKS=0 (host-bound: the enqueue rate) and
// SPIN_TICKS=1000 (every workgroup waits 10 us after reading its arguments: GPU-bound).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bench/micro/kernarg bench/micro/kernarg.hip
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DSPIN_TICKS=1000 -o bench/micro/kernarg_spin bench/micro/kernarg.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#ifndef SPIN_TICKS
#define SPIN_TICKS 0
#endif

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

struct Big {
  unsigned w[128];  // 512 B: 8 lines of 64 B
};

// after the argument reads, every workgroup waits ~kSpinTicks x 10 ns so the GPU, not the host's enqueue rate, bounds
// the loop (the launch-to-launch time is then spin + the GPU-side gap + the argument fetch)
constexpr unsigned long long kSpinTicks = SPIN_TICKS;

__device__ __forceinline__ void sink(unsigned* out, unsigned v) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < kSpinTicks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(v, r, blockIdx.x * 4, 0, 0);
  }
}

__global__ __launch_bounds__(512) void kA(Big a, unsigned* out) {
  unsigned s = 0;
#pragma unroll
  for (int l = 0; l < 8; ++l) s += a.w[16 * l + (l & 3)];
  sink(out, s);
}

__global__ __launch_bounds__(512) void kB(const Big* __restrict__ a, unsigned* out) {
  unsigned s = 0;
#pragma unroll
  for (int l = 0; l < 8; ++l) s += a->w[16 * l + (l & 3)];
  sink(out, s);
}

__global__ __launch_bounds__(512) void kC(unsigned x, unsigned* out) { sink(out, x); }  // 12 B of arguments

int main() {
  const int blocks = 256, launches = 2000, glaunch = 200;
  unsigned* out;
  Big* dbig;
  Big hb;
  for (int i = 0; i < 128; ++i) hb.w[i] = i;
  CK(hipMalloc(&out, blocks * 4));
  CK(hipMalloc(&dbig, sizeof(Big)));
  CK(hipMemcpy(dbig, &hb, sizeof(Big), hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](const char* name, auto&& body, int n) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      body();  // warm
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      body();
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("{\"case\": \"%s\", \"spin_us\": %.1f, \"us_per_launch\": %.3f}\n", name, kSpinTicks / 100.0,
           best * 1e3f / n);
  };
  timed("512 B by value, stream", [&] { for (int i = 0; i < launches; ++i) kA<<<blocks, 512, 0, s>>>(hb, out); },
        launches);
  timed("pointer to 512 B in device memory, stream",
        [&] { for (int i = 0; i < launches; ++i) kB<<<blocks, 512, 0, s>>>(dbig, out); }, launches);
  timed("12 B by value, stream", [&] { for (int i = 0; i < launches; ++i) kC<<<blocks, 512, 0, s>>>(7u, out); },
        launches);
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < glaunch; ++i) kA<<<blocks, 512, 0, s>>>(hb, out);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  timed("512 B by value, graph replay", [&] { CK(hipGraphLaunch(ge, s)); }, glaunch);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < glaunch; ++i) kB<<<blocks, 512, 0, s>>>(dbig, out);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  timed("pointer to 512 B in device memory, graph replay", [&] { CK(hipGraphLaunch(ge, s)); }, glaunch);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipFree(out));
  CK(hipFree(dbig));
  return 0;
}
