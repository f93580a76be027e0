// Does a kernel launch start with a cold instruction cache?  Each wave runs the same straight-line block of
// N one-cycle instructions (s_nop: 4 bytes each) twice in a loop and stamps s_memrealtime (100 MHz) around each
// pass: pass 1 fetches the block's lines unless an earlier launch left them in the SQC's instruction cache, pass 2
// finds them there.  Launches repeat back to back; the last one is reported.  If pass 1 costs ~N / 16 line fetches
// on every launch, not just the first, the instruction cache is invalidated at each kernel start and a kernel's
// executed code size is a per-launch latency (the headline forward's K loop: same time at a quarter of its K,
// profiles/stamps_ksplit_r4.jsonl).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bench/micro/icache bench/micro/icache.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

#define BLOCK(n) asm volatile(".rept " #n "\n s_nop 0\n .endr" ::: "memory")

// out[(block * 8 + wave) * 2 + p] = pass p's duration in 10 ns ticks (vector buffer stores from lane 0)
#define KERNEL(name, n)                                                                                 \
  __global__ __launch_bounds__(512) void name(unsigned* __restrict__ out) {                             \
    unsigned d[2];                                                                                       \
    _Pragma("clang loop unroll(disable)") for (int p = 0; p < 2; ++p) {                                  \
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();                                   \
      BLOCK(n);                                                                                          \
      const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();                                   \
      d[p] = (unsigned)(t1 - t0);                                                                        \
    }                                                                                                    \
    const int w = blockIdx.x * 8 + (threadIdx.x >> 6);                                                   \
    if ((threadIdx.x & 63) == 0) {                                                                       \
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000); \
      __builtin_amdgcn_raw_buffer_store_b32(d[0], r, w * 8, 0, 0);                                      \
      __builtin_amdgcn_raw_buffer_store_b32(d[1], r, w * 8 + 4, 0, 0);                                  \
    }                                                                                                    \
  }

KERNEL(k_256, 256)
KERNEL(k_1024, 1024)
KERNEL(k_4096, 4096)

static void run(const char* name, void (*k)(unsigned*), int blocks, unsigned* dout) {
  std::vector<unsigned> h(blocks * 8 * 2);
  float ms = 0.f;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 20; ++rep) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, dout);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
  }
  CK(hipMemcpy(h.data(), dout, h.size() * 4, hipMemcpyDeviceToHost));
  std::vector<double> p1, p2;
  for (int i = 0; i < blocks * 8; ++i) {
    p1.push_back(h[2 * i] * 10.0 / 1000.0);
    p2.push_back(h[2 * i + 1] * 10.0 / 1000.0);
  }
  auto pct = [](std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(q * (v.size() - 1))];
  };
  printf("{\"kernel\": \"%s\", \"blocks\": %d, \"pass1_us\": [%.3f, %.3f, %.3f], \"pass2_us\": [%.3f, %.3f, %.3f], "
         "\"launch_ms\": %.4f}\n",
         name, blocks, pct(p1, 0.1), pct(p1, 0.5), pct(p1, 0.9), pct(p2, 0.1), pct(p2, 0.5), pct(p2, 0.9), ms);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main() {
  unsigned* dout;
  const int kMaxBlocks = 256;
  CK(hipMalloc(&dout, kMaxBlocks * 8 * 2 * 4));
  for (int blocks : {8, 256}) {
    run("s_nop x256 (1 KB)", k_256, blocks, dout);
    run("s_nop x1024 (4 KB)", k_1024, blocks, dout);
    run("s_nop x4096 (16 KB)", k_4096, blocks, dout);
  }
  CK(hipFree(dout));
  return 0;
}
