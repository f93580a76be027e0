// Homework kernel suite on gfx950 -- the capabilities of CME213 hw1-hw4,
// re-designed for MI355X (no Thrust, no CUDA idioms):
//   hw1  even/odd sum (wave reductions) and LSD radix sort (LDS histograms,
//        scanned digit offsets, stable wave-ballot ranking)
//   hw2  byte-shift cipher streaming at 1/4/8/16 bytes per lane; CSR PageRank
//   hw3  2-D heat-diffusion stencil, orders 2/4/8: global, register-blocked
//        ("loop"), and LDS-tiled (the variant the reference left empty)
//   hw4  Vigenere: sanitise (stream compaction), shift, LDS-privatised
//        histograms, batched index-of-coincidence, per-residue frequency
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace cme::suite {

// ---------------------------------------------------------------- hw2 shift
// out[i] = in[i] + shift (byte-wise, wrap mod 256) using `width`-byte lanes
// (1, 4, 8, 16).  Wide lanes add shift*0x0101.. per byte WITH carry isolation,
// so the result equals the byte loop for every byte value (the reference's
// packed add was only correct while byte+shift < 256, hw2code/shift.cu:24-42).
void shift_bytes(const uint8_t* in, uint8_t* out, int64_t n, uint8_t shift, int width, int block, int grid_cap,
                 hipStream_t s);

// ------------------------------------------------------------- hw2 pagerank
// out[i] = 0.5/N + 0.5 * sum_{j in adj(i)} in[e_j] * inv_deg[e_j]   (CSR pull)
// variant 0: thread per node, 1: wave per node (long rows), 2: auto by avg degree
void pagerank_propagate(const uint32_t* indptr, const uint32_t* edges, const float* in, float* out,
                        const float* inv_deg, int n, int variant, hipStream_t s);
// the pre-multiplied form: w = in .* inv_deg once (pagerank_premul), then every propagation gathers w alone and
// writes out[i] = 0.5/N + 0.5 * sum_j w_in[e_j] and w_out[i] = out[i] * inv_deg[i] for the next one; lpn lanes per
// node (1, 2, 4, 8)
void pagerank_premul(const float* in, const float* inv_deg, float* w, int n, hipStream_t s);
void pagerank_propagate_w(const uint32_t* indptr, const uint32_t* edges, const float* w_in, float* out, float* w_out,
                          const float* inv_deg, int n, int lpn, hipStream_t s);

// ------------------------------------------------------------- hw3 stencil
// next(interior) = Stencil<order>(curr); variant 0 global, 1 register-blocked loop, 2 LDS tile
void stencil_step(float* next, const float* curr, int gx, int gy, int order, float xcfl, float ycfl,
                  int variant, hipStream_t s);
// one launch per time step: interior stencil AND next(border) = curr(border) * scale (with_bc)
void stencil_step_bc(float* next, const float* curr, int gx, int gy, int order, float xcfl, float ycfl, int variant,
                     float scale, bool with_bc, hipStream_t s);
// the LDS variant at order 8 with its knobs exposed (rows per wave 32/64/128, rows loaded ahead 4/8, non-temporal
// streamed loads), interior only: bench/stencil_tune.py
void stencil_lds_tune(float* next, const float* curr, int gx, int gy, float xcfl, float ycfl, int rows, int ahead,
                      int nt, hipStream_t s);
// next(border) = curr(border) * scale  (border width b)
void stencil_bc(float* next, const float* curr, int gx, int gy, int b, float scale, hipStream_t s);
// TWO time steps (each: interior stencil + border * scale) in one sweep of the grid: the LDS walk with temporal
// blocking (order 8); bitwise two stencil_step_bc launches
// (rows, ahead <= 0: the production walk -- 64 rows per wave, 4 rows of loads ahead; others: tuning)
void stencil_step2_bc(float* next, const float* curr, int gx, int gy, int order, float xcfl, float ycfl, float scale,
                      hipStream_t s, int rows = 0, int ahead = 0);

// -------------------------------------------------------------- hw1 sums
// sums[0] = sum of even values, sums[1] = sum of odd values (64-bit, device)
void sum_even_odd(const uint32_t* v, int64_t n, unsigned long long* sums, hipStream_t s);

// -------------------------------------------------------------- hw1 radix
int64_t radix_workspace_bytes(int64_t n);
// stable LSD sort of n uint32 keys in place (tmp: n keys scratch), 8-bit digits
void radix_sort_u32(uint32_t* keys, uint32_t* tmp, int64_t n, void* workspace, hipStream_t s);
// one stable pass on bits [start_bit, start_bit+8): out = stable partition of in by digit
void radix_pass_u32(const uint32_t* in, uint32_t* out, int64_t n, int start_bit, void* workspace, hipStream_t s);

// -------------------------------------------------------------- hw4 cipher
// lower-case letters of `in` (A-Z folded to a-z) compacted in order into out;
// returns the count through *count (device int64).  workspace: cipher_workspace_bytes(n)
int64_t cipher_workspace_bytes(int64_t n);
void sanitize_lower(const uint8_t* in, int64_t n, uint8_t* out, int64_t* count, void* workspace, hipStream_t s);
// out[i] = in[i] + sign*shifts[i % period]; wrap: within 'a'..'z' (mod 26), else raw byte add
void vigenere_apply(const uint8_t* in, uint8_t* out, int64_t n, const int* shifts, int period, int sign, int wrap,
                    hipStream_t s);
// 256-bin byte histogram (LDS-privatised, one global merge per block)
void byte_histogram(const uint8_t* in, int64_t n, uint32_t* hist, hipStream_t s);
// counts[s - lo] = #{i : t[i] == t[i+s]} for s in [lo, hi)   (batched kappa IoC)
void shifted_matches(const uint8_t* t, int64_t n, int lo, int hi, unsigned long long* counts, hipStream_t s);
// hist[r][c] = #{i : i % period == r, t[i] == c}  ([period][256])
void residue_histogram(const uint8_t* t, int64_t n, int period, uint32_t* hist, hipStream_t s);

}  // namespace cme::suite
