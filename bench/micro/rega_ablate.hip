// Ablation of the A-in-registers GEMM engine (csrc/mlp/rega_gemm.h) at the 784-4096-10 forward shape
// (C[4096 x 800] = W1[4096 x 784] . X[800 x 784]^T, fp32 W1 split into 3 bf16 planes, bf16 X): the full
// K loop vs the same loop without MFMA (operand traffic + fragment reads + split only) vs without loads
// (MFMA + fragment reads only).  No epilogue beyond one store per lane.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc -o bench/micro/rega_ablate bench/micro/rega_ablate.hip
#include <cstdio>
#include <cstdlib>

#include "mlp/rega_gemm.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

using bf16 = __hip_bfloat16;

template <typename AT, int WC, int ABLATE>
__global__ __launch_bounds__(512) void k_ablate(const AT* A, const bf16* B, float* C, int M, int N, int K, int tn) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int id = cme::xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (id / tn) * 128, n0 = (id % tn) * 128;
  using G = cme::RegaGeom<128, WC>;
  cme::f32x4 acc[G::MB][G::NB];
  cme::rega_gemm_mainloop<AT, 128, WC, 25, ABLATE>(A, K, B, K, M, N, K, m0, n0, lds, acc);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < G::MB; ++i)
#pragma unroll
    for (int j = 0; j < G::NB; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  C[blockIdx.x * 512 + threadIdx.x] = s;
}

template <typename AT, int WC, int ABLATE>
void run(const char* name, const AT* A, const bf16* B, float* C) {
  const int M = 4096, N = 800, K = 784, tn = 7, nwg = 32 * 7;
  const int lds = cme::ra::lds_bytes<128>();
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ablate<AT, WC, ABLATE>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  for (int w = 0; w < 3; ++w) k_ablate<AT, WC, ABLATE><<<nwg, 512, lds>>>(A, B, C, M, N, K, tn);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 50;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) k_ablate<AT, WC, ABLATE><<<nwg, 512, lds>>>(A, B, C, M, N, K, tn);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("{\"variant\": \"%s\", \"us\": %.2f}\n", name, 1e3 * ms / reps);
  fflush(stdout);
}

int main() {
  float* A;
  bf16 *Ab, *B;
  float* C;
  CK(hipMalloc(&A, 4096 * 784 * 4));
  CK(hipMalloc(&Ab, 4096 * 784 * 2));
  CK(hipMalloc(&B, 800 * 784 * 2));
  CK(hipMalloc(&C, 224 * 512 * 4));
  CK(hipMemset(A, 0x3c, 4096 * 784 * 4));  // ~0.01, non-zero random-ish bits
  CK(hipMemset(Ab, 0x3c, 4096 * 784 * 2));
  CK(hipMemset(B, 0x3f, 800 * 784 * 2));
  for (int r = 0; r < 2; ++r) {
    run<float, 1, 0>("f32_wc1_full", A, B, C);
    run<float, 2, 0>("f32_wc2_full", A, B, C);
    run<float, 2, 1>("f32_wc2_no_mfma", A, B, C);
    run<float, 2, 2>("f32_wc2_no_loads", A, B, C);
    run<bf16, 1, 0>("bf16_wc1_full", Ab, B, C);
    run<bf16, 2, 0>("bf16_wc2_full", Ab, B, C);
    run<bf16, 2, 1>("bf16_wc2_no_mfma", Ab, B, C);
    run<bf16, 2, 2>("bf16_wc2_no_loads", Ab, B, C);
  }
  return 0;
}
