// Microbenchmark: per-CU global -> LDS fill rate of the LDS-DMA buffer load (buffer_load_dwordx4 ... lds)
// in the access pattern of the wide GEMM engine (csrc/mlp/glds_gemm.h), without any MFMA work.
//
// Every workgroup streams NSTAGE stages of ROWS rows x ROWB bytes (a K-slab of a row-major operand with a
// row pitch of `pitch` bytes) into a ring of NBUF LDS buffers, NBUF-1 stages in flight, one counted vmcnt
// + s_barrier per stage -- exactly the engine's pipeline.  Variants: row segment 64 B (BK = 32 bf16) vs
// 128 B (BK = 64), 4 vs 8 issuing waves, a hot (L2-resident, every workgroup reads the same slab) vs a
// streaming source (every workgroup its own rows, as the GEMM's A operand per row tile).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/glds_fill bench/micro/glds_fill.hip && /tmp/glds_fill
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int kOOB = 0x7FFFFFF0;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, kOOB, 0x00020000);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_base, 16, voff, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ROWS rows x ROWB bytes per stage, NT threads, NBUF buffers
template <int ROWB, int ROWS, int NT, int NBUF>
__global__ __launch_bounds__(NT) void fill_kernel(const char* __restrict__ src, int pitch, int nstage, int rows_per_wg,
                                           int hot, float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int SB = ROWS * ROWB;            // bytes per stage
  constexpr int NW = NT / 64;
  constexpr int INSTR = SB / 1024;           // 1 KB per DMA instruction
  static_assert(INSTR % NW == 0, "instructions per wave");
  constexpr int L = INSTR / NW;
  constexpr int RPI = 1024 / ROWB;           // rows per instruction
  constexpr int LPR = ROWB / 16;             // lanes per row
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t r = rsrc(src);
  // the GEMM's operand rows of this workgroup (hot: every workgroup the first rows_per_wg rows): the
  // first 3/4 are 3 planes x rows/4 A rows of row tile id / 7, the last 1/4 the B rows of column tile id % 7
  int id = blockIdx.x;
  {
    const int n = gridDim.x, q = n / 8, rr = n % 8, x = id % 8;  // bijective XCD remap (as the engine)
    id = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + id / 8;
  }
  const int rt = id / 7, ct = id % 7, qr = rows_per_wg / 4;
  int off[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const int ins = wave + NW * j;
    const int i = (ins * RPI + lane / LPR) % rows_per_wg;
    int row = i;
    if (!hot) row = i < 3 * qr ? (i / qr) * 4096 + rt * qr + i % qr : 3 * 4096 + ct * qr + (i - 3 * qr);
    off[j] = row * pitch + (lane % LPR) * 16;
  }
  auto issue = [&](int kt) {
    char* base = lds + (kt % NBUF) * SB;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int ins = wave + NW * j;
      dma16(r, base + ins * 1024, off[j] + kt * ROWB);
    }
  };
  for (int s = 0; s < NBUF - 1; ++s)
    if (s < nstage) issue(s);
  float acc = 0.f;
  for (int kt = 0; kt < nstage; ++kt) {
    const int younger = min(NBUF - 2, nstage - 1 - kt);
    if (younger >= 3) wait_vm<3 * L>();
    else if (younger == 2) wait_vm<2 * L>();
    else if (younger == 1) wait_vm<L>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NBUF - 1 < nstage) issue(kt + NBUF - 1);
    acc += reinterpret_cast<const float*>(lds + (kt % NBUF) * SB)[threadIdx.x];
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;
}

template <int ROWB, int ROWS, int NT, int NBUF>
void run(const char* name, const char* src, int pitch, int K_bytes, int nwg, int rows_per_wg, int hot, float* out) {
  const int nstage = K_bytes / ROWB;
  const int lds = NBUF * ROWS * ROWB;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fill_kernel<ROWB, ROWS, NT, NBUF>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) fill_kernel<ROWB, ROWS, NT, NBUF><<<nwg, NT, lds>>>(src, pitch, nstage, rows_per_wg, hot, out);
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) fill_kernel<ROWB, ROWS, NT, NBUF><<<nwg, NT, lds>>>(src, pitch, nstage, rows_per_wg, hot, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = 1e3 * ms / reps;
  const double bytes_wg = (double)nstage * ROWS * ROWB;
  printf("{\"variant\": \"%s\", \"row_bytes\": %d, \"rows_per_stage\": %d, \"waves\": %d, \"buffers\": %d, \"hot\": %d, "
         "\"wg\": %d, \"stages\": %d, \"us\": %.2f, \"GBps_per_wg\": %.1f, \"TBps_total\": %.2f}\n",
         name, ROWB, ROWS, NT / 64, NBUF, hot, nwg, nstage, us, bytes_wg / us / 1e3, bytes_wg * nwg / us / 1e6);
  fflush(stdout);
}


// A-in-registers variant: every wave streams its own 16 A rows x 128 B per stage (fp32 k32: two
// dwordx4 per lane, straight into registers, a DEPTH-stage register ring), while the B operand (BROWS
// rows x 64 B per stage) goes to LDS by LDS-DMA (4 buffers) -- the split-on-the-fly engine's traffic.
template <int DEPTH, int BROWS>
__global__ __launch_bounds__(512) void regA_kernel(const char* __restrict__ src, int pitch, int nstage, float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int NW = 8, SB = BROWS * 64, LB = SB / 1024 / NW;  // B DMA instructions per wave per stage
  static_assert(LB >= 1, "B rows");
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t r = rsrc(src);
  int id = blockIdx.x;
  {
    const int n = gridDim.x, q = n / 8, rr = n % 8, x = id % 8;
    id = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + id / 8;
  }
  const int rt = id / 7, ct = id % 7;
  // A: rows rt*128 + wave*16 + (lane & 15), 32 B at k-offset 32 * (lane >> 4) of the 128-B stage slab
  const int aoff = (rt * 128 + wave * 16 + (lane & 15)) * pitch * 2 + (lane >> 4) * 32;  // pitch*2: fp32 rows
  int boff[LB];
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    const int ins = wave + NW * j;
    boff[j] = (12288 + ct * BROWS + ins * 16 + (lane >> 2)) * pitch + (lane & 3) * 16;
  }
  uint4 ring[DEPTH][2];
  auto issueA = [&](int kt, uint4 (&dst)[2]) {
    dst[0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, aoff + kt * 128, 0, 0));
    dst[1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, aoff + kt * 128 + 16, 0, 0));
  };
  auto issueB = [&](int kt) {
#pragma unroll
    for (int j = 0; j < LB; ++j) dma16(r, lds + (kt % 4) * SB + (wave + NW * j) * 1024, boff[j] + kt * 64);
  };
  float acc = 0.f;
#pragma unroll
  for (int s = 0; s < DEPTH; ++s) {
    issueB(s);
    issueA(s, ring[s]);
  }
  for (int kt = 0; kt < nstage; kt += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      // stage kt+d (its A pair and B DMA) is the oldest group in flight: (DEPTH-1) younger groups of (LB+2)
      wait_vm<(DEPTH - 1) * (LB + 2)>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      acc += __builtin_bit_cast(float, ring[d][0].x) + __builtin_bit_cast(float, ring[d][1].w);
      acc += reinterpret_cast<const float*>(lds + ((kt + d) % 4) * SB)[threadIdx.x];
      issueB(kt + d + DEPTH);
      issueA(kt + d + DEPTH, ring[d]);
    }
  }
  wait_vm<0>();
  if (acc == 12345.f) out[blockIdx.x] = acc;
}

template <int DEPTH, int BROWS>
void run_regA(const char* name, const char* src, int pitch, int nstage, int nwg, float* out) {
  const int lds = 4 * BROWS * 64;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&regA_kernel<DEPTH, BROWS>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) regA_kernel<DEPTH, BROWS><<<nwg, 512, lds>>>(src, pitch, nstage, out);
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) regA_kernel<DEPTH, BROWS><<<nwg, 512, lds>>>(src, pitch, nstage, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = 1e3 * ms / reps;
  const double bytes_wg = (double)nstage * (128 * 128 + BROWS * 64);
  printf("{\"variant\": \"%s\", \"depth\": %d, \"wg\": %d, \"stages\": %d, \"us\": %.2f, \"GBps_per_wg\": %.1f, "
         "\"TBps_total\": %.2f}\n", name, DEPTH, nwg, nstage, us, bytes_wg / us / 1e3, bytes_wg * nwg / us / 1e6);
  fflush(stdout);
}

int main() {
  // a 3 x 4096-row x 784-col bf16 operand (the split3 W1 planes): pitch 1568 B, K = 1568 B per row
  const int rows = 3 * 4096 + 2048, pitch = 1568, K = 1536;  // 1536 B = 24 stages of 64 B / 12 of 128 B
  char* src;
  float* out;
  CK(hipMalloc(&src, (size_t)rows * pitch + 4096));
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  CK(hipMemset(src, 1, (size_t)rows * pitch));
  const int nwg = 224, rpw = 512;  // each workgroup: 512 rows (384 A rows + 128 B rows in the GEMM)
  for (int hot = 0; hot < 2; ++hot) {
    // the engine today: 64-B row segments, 512 rows per stage (32 KB), 8 waves, 4 buffers
    run<64, 512, 512, 4>("seg64_8w_4buf", src, pitch, K, nwg, rpw, hot, out);
    run<64, 512, 256, 4>("seg64_4w_4buf", src, pitch, K, nwg, rpw, hot, out);
    run<64, 512, 512, 3>("seg64_8w_3buf", src, pitch, K, nwg, rpw, hot, out);
    run<64, 512, 512, 5>("seg64_8w_5buf", src, pitch, K, nwg, rpw, hot, out);
    // 128-B row segments (BK = 64): the same 32 KB per stage = 256 rows, or the 64 KB stage of 512 rows
    run<128, 256, 512, 4>("seg128_8w_4buf_32K", src, pitch, K, nwg, 256, hot, out);
    run<128, 512, 512, 2>("seg128_8w_2buf_64K", src, pitch, K, nwg, rpw, hot, out);
    run<128, 256, 256, 4>("seg128_4w_4buf_32K", src, pitch, K, nwg, 256, hot, out);
  }
  // A fp32 in registers (4096 rows x 3136 B; pitch*2), B bf16 by DMA: 24 stages of k32
  run_regA<2, 128>("regA_d2", src, pitch, 24, nwg, out);
  run_regA<3, 128>("regA_d3", src, pitch, 24, nwg, out);
  run_regA<4, 128>("regA_d4", src, pitch, 24, nwg, out);
  CK(hipFree(src));
  CK(hipFree(out));
  return 0;
}
