// Block one-sided Jacobi step on MFMA (the performance path).
//
// The reference rotates one column pair at a time with a memory-bound Givens
// kernel (reference main.cu:139-147) driven by host dot products
// (main.cu:698-707).  On CDNA4 the same sweep is re-blocked so every byte of
// A and V moved through HBM feeds matrix-core work:
//
//   columns are grouped in blocks of W; a step processes P disjoint block
//   pairs (bi, bj) with X = [A_bi A_bj] (m x 2W):
//     gram  : C = A_bi^T A_bj (cross) or G = X^T X (full), MFMA, split over
//             rows into partial slabs (deterministic, no float atomics);
//     evd   : G = [[D_bi, C], [C^T, D_bj]] -> Q^T G Q = Lambda by cyclic
//             parallel Jacobi held entirely in LDS (one 1024-thread WG per
//             pair); the convergence value max|g_pq|/sqrt(g_pp g_qq) of the
//             reference (main.cu:710) becomes the stop test;
//     apply : X <- X Q and [V_bi V_bj] <- [..] Q in place, MFMA, computed
//             transposed (Out^T = Q^T X^T) so loads AND stores are
//             128-byte coalesced column segments.
//
// Blocks are kept internally orthogonal (every step fully diagonalises its
// pair), so only the W x W cross Gram is needed per step; the diagonal blocks
// are the tracked squared column norms D.  The first step of a sweep uses the
// full Gram, which re-measures every within-block angle from the data.
#include "common.hpp"
#include "evd_deal_tables.hpp"
#include "svdj_debug.h"
#include "svdj_hip.h"
#include "svdj_stop.h"

#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

namespace svdj {

constexpr int kGramThreads = 256;
constexpr int kApplyThreads = 256;

__host__ __device__ constexpr int round_up(int a, int b) { return (a + b - 1) / b * b; }

// ------------------------------------------------------------------- gram
// MODE: GRAM_CROSS  C = A_bi^T A_bj (W x W slab per pair and row chunk);
//       GRAM_FULL   G = [A_bi A_bj]^T [..] (2W x 2W slab), one launch;
//       GRAM_SPLIT  the same 2W x 2W slab in three regions (A_bi^T A_bi,
//                   A_bj^T A_bj, A_bi^T A_bj), one per blockIdx.z: the
//                   one-launch form keeps 2W(2W+1)/2 tile accumulators, which
//                   for fp64 W = 64 exceed the register file.
// (The cross Grams of a quad step: gram_quad_kernel.)
// For fp64 W = 64 the cross products are also split over blockIdx.z in XS = 2
// row halves (x tiles), so accumulators plus the double-buffered loads fit in
// registers without spilling.
enum { GRAM_CROSS = 0, GRAM_FULL = 1, GRAM_SPLIT = 2 };

// (bi, bj) of Gram slab `pair`.
template <int MODE>
__device__ __forceinline__ void gram_pair(const int32_t* __restrict__ pairs, int pair, int& pi,
                                          int& pj) {
  pi = pairs[2 * pair];
  pj = pairs[2 * pair + 1];
}
template <typename T, int W>
__host__ __device__ constexpr int gram_xsplit() { return (sizeof(T) == 8 && W == 64) ? 2 : 1; }

// Rows per lane per slab of the fp32 W=64 cross Gram (16 = 64 bytes).  8 or
// 4 cut registers (208 -> 172) but measured slower end to end (16384^2 1 GPU
// 5.76 -> 6.08 s, 8-GPU rank plan 63.8 -> 73 ms; round 2).
constexpr int kGramLpl64 = 16;
// NV consecutive elements of one column with 16-byte vector loads.
template <typename T, int NV>
__device__ __forceinline__ void load_col16B(const T* __restrict__ p, T (&v)[NV]) {
  constexpr int PER = 16 / (int)sizeof(T);
  static_assert(NV % PER == 0, "whole 16-byte vectors");
  const f32x4* q = reinterpret_cast<const f32x4*>(p);
#pragma unroll
  for (int i = 0; i < NV / PER; ++i) {
    f32x4 x = q[i];
    const T* xs = reinterpret_cast<const T*>(&x);
#pragma unroll
    for (int j = 0; j < PER; ++j) v[i * PER + j] = xs[j];
  }
}

template <typename T, int W, int MODE>
__global__ __launch_bounds__(kGramThreads) void gram_kernel(
    const T* __restrict__ A, int lda, int m_pad, const int32_t* __restrict__ pairs,
    int rows_per_chunk, T* __restrict__ slabs) {
  using M = Mfma<T>;
  constexpr bool FULL = MODE == GRAM_FULL;
  constexpr int TL = M::TILE;
  constexpr int HT = W / TL;                             // column tiles per block
  constexpr int XS = FULL ? 1 : gram_xsplit<T, W>();     // row halves over blockIdx.z
  constexpr int HTX = HT / XS;                           // x tiles of this workgroup
  constexpr int NCT = FULL ? 2 * HT : HTX + HT;          // column tiles loaded
  constexpr int NTP = FULL ? NCT * (NCT + 1) / 2 : HTX * HT;
  // rows per lane per slab: 64 bytes
  constexpr int LPL = (sizeof(T) == 4 && W == 64 && !FULL) ? kGramLpl64 : M::LPL;
  constexpr int SR = M::KG * LPL;  // rows per wave per slab
  constexpr int SLAB = FULL ? 4 * W * W : HTX * TL * W;  // this workgroup's reduction
  constexpr int WAVES = kGramThreads / SVDJ_WAVE;
  static_assert(HT % XS == 0, "x tiles split evenly");

  const int pair = blockIdx.x, chunk = blockIdx.y, nchunk = gridDim.y;
  const int region = MODE == GRAM_SPLIT ? (int)blockIdx.z / XS : 2;
  const int xpart = FULL ? 0 : (int)blockIdx.z % XS;
  int pi, pj;
  gram_pair<MODE>(pairs, pair, pi, pj);
  const int bi = region == 1 ? pj : pi, bj = region == 0 ? pi : pj;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r_begin = chunk * rows_per_chunk;
  const int r_end = min(m_pad, r_begin + rows_per_chunk);

  // tile-pair list (compile-time)
  typename M::acc_t acc[NTP];
#pragma unroll
  for (int i = 0; i < NTP; ++i) acc[i] = M::zero();

  const T* colp[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    int blk, tile;
    if constexpr (FULL) {
      blk = ct < HT ? bi : bj;
      tile = ct % HT;
    } else {
      blk = ct < HTX ? bi : bj;
      tile = ct < HTX ? xpart * HTX + ct : ct - HTX;
    }
    const int col = blk * W + tile * TL + M::lane_col(lane);
    colp[ct] = A + (size_t)col * lda + M::lane_kg(lane) * LPL;
  }

  // Software pipeline: the next 32-row slab's loads are issued before this
  // slab's MFMAs, so HBM latency overlaps matrix-core work (without it the
  // kernel ran at ~2 TB/s, latency-bound, measured on MI355X at n=16384).
  int r0 = r_begin + wave * SR;
  T v[NCT][LPL];
  if (r0 < r_end) {
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) load_col16B<T, LPL>(colp[ct] + r0, v[ct]);
  }
  for (; r0 < r_end; r0 += WAVES * SR) {
    const int rn = r0 + WAVES * SR;
    T vn[NCT][LPL];
    if (rn < r_end) {
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) load_col16B<T, LPL>(colp[ct] + rn, vn[ct]);
    }
#pragma unroll
    for (int t = 0; t < LPL; ++t) {
      int idx = 0;
      if constexpr (FULL) {
#pragma unroll
        for (int a = 0; a < NCT; ++a)
#pragma unroll
          for (int b = a; b < NCT; ++b) {
            acc[idx] = M::mfma(v[a][t], v[b][t], acc[idx]);
            ++idx;
          }
      } else {
#pragma unroll
        for (int a = 0; a < HTX; ++a)
#pragma unroll
          for (int b = 0; b < HT; ++b) {
            acc[idx] = M::mfma(v[a][t], v[HTX + b][t], acc[idx]);
            ++idx;
          }
      }
    }
    if (rn < r_end) {
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int t = 0; t < LPL; ++t) v[ct][t] = vn[ct][t];
    }
  }

  // Combine the waves' partial tiles in LDS (sequentially, deterministic).
  __shared__ T red[SLAB];
  for (int i = threadIdx.x; i < SLAB; i += kGramThreads) red[i] = T(0);
  __syncthreads();
  for (int w = 0; w < WAVES; ++w) {
    if (wave == w) {
      int idx = 0;
      if constexpr (FULL) {
        constexpr int N = 2 * W;
#pragma unroll
        for (int a = 0; a < NCT; ++a)
#pragma unroll
          for (int b = a; b < NCT; ++b) {
#pragma unroll
            for (int e = 0; e < M::NACC; ++e) {
              const int r = a * TL + M::acc_row(e, lane);
              const int c = b * TL + M::lane_col(lane);
              red[r * N + c] += acc[idx][e];
              if (a != b) red[c * N + r] += acc[idx][e];
            }
            ++idx;
          }
      } else {
#pragma unroll
        for (int a = 0; a < HTX; ++a)
#pragma unroll
          for (int b = 0; b < HT; ++b) {
#pragma unroll
            for (int e = 0; e < M::NACC; ++e) {
              const int r = a * TL + M::acc_row(e, lane);
              const int c = b * TL + M::lane_col(lane);
              red[r * W + c] += acc[idx][e];
            }
            ++idx;
          }
      }
    }
    __syncthreads();
  }
  const int xoff = xpart * HTX * TL;  // first row of this workgroup's part
  if constexpr (MODE == GRAM_SPLIT) {  // this region's quadrant(s) of the 2W x 2W slab
    constexpr int N = 2 * W;
    T* out = slabs + ((size_t)pair * nchunk + chunk) * 4 * W * W;
    for (int i = threadIdx.x; i < SLAB; i += kGramThreads) {
      const int a = xoff + i / W, b = i % W;
      const T v = red[i];
      if (region == 0) out[a * N + b] = v;
      if (region == 1) out[(W + a) * N + W + b] = v;
      if (region == 2) {
        out[a * N + W + b] = v;
        out[(W + b) * N + a] = v;
      }
    }
  } else if constexpr (FULL) {
    T* out = slabs + ((size_t)pair * nchunk + chunk) * SLAB;
    for (int i = threadIdx.x; i < SLAB; i += kGramThreads) out[i] = red[i];
  } else {
    T* out = slabs + ((size_t)pair * nchunk + chunk) * (W * W) + xoff * W;
    for (int i = threadIdx.x; i < SLAB; i += kGramThreads) out[i] = red[i];
  }
}

// fp32 W = 64 cross Gram (GRAM_CROSS) with coalesced loads.
// gram_kernel's operand loads follow the MFMA lane map (lane = column): every
// 16-byte load instruction touches 64 columns, i.e. 64 cache lines.  Here a
// wave loads its 32-row slab of the pair's 128 columns with lanes along the
// rows (8 lanes x 16 B = one 128-byte column segment, 8 columns per
// instruction), keeps the next slab in flight in registers, and transposes
// through a wave-private LDS image [column][32 rows + 4 pad] (144-byte
// stride: conflict-free ds_read_b128 of 4 rows of a column per lane).  The
// MFMAs and the reduction are gram_kernel's; no barrier inside the row loop.
constexpr int kGlStride = 36;  // floats per column in the LDS image
template <int MODE>
__global__ __launch_bounds__(kGramThreads) void gram_cross_f32_kernel(
    const float* __restrict__ A, int lda, int m_pad, const int32_t* __restrict__ pairs,
    int rows_per_chunk, float* __restrict__ slabs, int rev) {
  static_assert(MODE == GRAM_CROSS, "cross Grams only");
  constexpr int W = 64, SR = 32, WAVES = kGramThreads / SVDJ_WAVE;
  using M = Mfma<float>;
  __shared__ float img[WAVES][2 * W * kGlStride];  // 4 x 18 KB; reused for the reduction
  // rev: row chunks dispatched last-first (the most recently written rows
  // of the previous apply first, while they may still sit in the Infinity Cache)
  const int pair = blockIdx.x, nchunk = gridDim.y,
            chunk = rev ? nchunk - 1 - (int)blockIdx.y : (int)blockIdx.y;
  int pi, pj;
  gram_pair<MODE>(pairs, pair, pi, pj);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r_begin = chunk * rows_per_chunk;
  const int r_end = min(m_pad, r_begin + rows_per_chunk);
  // loads: instruction j covers columns 8j .. 8j+7 (lane >> 3), rows 4 (lane & 7) ..
  const int lc = lane >> 3, lr = (lane & 7) * 4;
  const float* src[2] = {A + (size_t)pi * W * lda, A + (size_t)pj * W * lda};
  float* im = img[wave];
  f32x4 ld[16];
  auto gload = [&](int r0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int col = 8 * j + lc;  // 0..127: x block then y block
      ld[j] = *reinterpret_cast<const f32x4*>(src[col >> 6] + (size_t)(col & 63) * lda + r0 + lr);
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      *reinterpret_cast<f32x4*>(im + (8 * j + lc) * kGlStride + lr) = ld[j];
  };
  M::acc_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = M::zero();
  const int c = lane & 31, kg = lane >> 5;
  int r0 = r_begin + wave * SR;
  if (r0 < r_end) {
    gload(r0);
    lstore();
  }
  for (; r0 < r_end; r0 += WAVES * SR) {
    const int rn = r0 + WAVES * SR;
    if (rn < r_end) gload(rn);
    // rows kg*16 + t of column tile ct: 4 x ds_read_b128 per tile
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      f32x4 v[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        v[ct] = *reinterpret_cast<const f32x4*>(im + (ct * 32 + c) * kGlStride + kg * 16 + q4 * 4);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) acc[a][b] = M::mfma(v[a][t], v[2 + b][t], acc[a][b]);
    }
    if (rn < r_end) lstore();  // after this wave's reads of the image (in-order LDS)
  }
  // combine the waves' partial tiles (sequentially, deterministic)
  __syncthreads();
  float* red = &img[0][0];
  for (int i = threadIdx.x; i < W * W; i += kGramThreads) red[i] = 0.0f;
  __syncthreads();
  for (int w = 0; w < WAVES; ++w) {
    if (wave == w) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int e = 0; e < M::NACC; ++e)
            red[(a * 32 + M::acc_row(e, lane)) * W + b * 32 + c] += acc[a][b][e];
    }
    __syncthreads();
  }
  float* out = slabs + ((size_t)pair * nchunk + chunk) * (W * W);
  for (int i = threadIdx.x; i < W * W; i += kGramThreads) out[i] = red[i];
}

// -------------------------------------------------------------------- evd
// The EVD of the 2W x 2W pair Gram runs in ONE workgroup per pair, as a
// cyclic parallel Jacobi (circle-method round robin: W disjoint rotations per
// step, 2W-1 steps per sweep):
//   * G lives in LDS in POSITION space (see pos_next below): every
//     off-diagonal slot-pair block (a < b) of a step is owned by one thread
//     for the whole kernel and its LDS addresses are static;
//   * ONE barrier per step.  The rotations of step st+1 are solved inside
//     step st's update phase: the coupling of a next-step pair lies in exactly
//     one off-diagonal block of step st, always the same one, so its owner
//     computes the new coupling, takes the post-step diagonals from the
//     step-st rotation records, solves step st+1's rotation right away and
//     publishes it (c, s, fp64 c/s and the post-rotation diagonals) into the
//     other half of a double-buffered record array.  The reference solves
//     every 2x2 on the host between two kernel launches (main.cu:698-725);
//   * the rotation accumulator Q lives in REGISTERS in fp64, in "slot layout":
//     lane (slot a, row group g) holds Q[k][first(a)] and Q[k][second(a)] for
//     its rows k.  The circle-method movement is a one-lane DPP shift per step
//     (wave_shr:1 / wave_shl:1); fp64 keeps Q orthogonal to ~1e-16 before it
//     is rounded to the data type, so V stays orthogonal over hundreds of
//     block steps;
//   * the diagonal never lives in G: it travels in the rotation records (a
//     rotation of slot a changes only d_first and d_second).
// Two values of one type, aligned to their combined size (one LDS access).
template <typename T>
struct alignas(2 * sizeof(T)) Pair2 {
  T x, y;
};

// Split-K slab loads in flight per thread while the EVD assembles G (with
// many GPUs a pair has up to 64 slabs of its Gram to sum, 1 MB for one
// workgroup).  8, 16 and 32 measured the same (8-GPU rank plan 59.5 / 60.0 /
// 59.9 ms per sweep): the slab sum is not what the EVD's latency is made of.
#define SVDJ_EVD_SLAB_UNROLL 8
__host__ __device__ constexpr int evd_threads(int) { return 1024; }

// Lane i <- lane i-1 / i+1 across the wave (DPP wave_shr:1 / wave_shl:1).
// The edge lane receives 0 (bound_ctrl); every caller overwrites the edge
// slots by select, so no "old" value (and no register copy) is needed.
__device__ __forceinline__ int dpp_shr1(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ int dpp_shl1(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true);
}
__device__ __forceinline__ float dpp_shr1(float v) {
  return __int_as_float(dpp_shr1(__float_as_int(v)));
}
__device__ __forceinline__ float dpp_shl1(float v) {
  return __int_as_float(dpp_shl1(__float_as_int(v)));
}
__device__ __forceinline__ double dpp_shr1(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = dpp_shr1((int)(x & 0xffffffff)), hi = dpp_shr1((int)(x >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double dpp_shl1(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = dpp_shl1((int)(x & 0xffffffff)), hi = dpp_shl1((int)(x >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Rotation test, shared by the solve and the "nothing to do" pre-pass so the
// two decide identically: relative |g_pq| > tol sqrt(g_pp g_qq) (fp32: raw
// v_sqrt, ~1 ulp), or the reference's absolute |g_pq| > tol (TOLERANCE,
// reference lib/global.cuh:9, main.cu:714) when absmode.
//
// Underflowing columns: in the relative mode a pair is rotated only if both
// squared norms exceed `floor` = m realmin / eps (metric[2..3], set once per
// solve, svdj_set_norm_floor).  Below it the squared norms and dot products
// of a column lose their precision to underflow (the entries' products
// approach realmin), so the relative coupling is noise and the pair would be
// rotated forever.  LAPACK's xGESVJ likewise skips columns below its safe
// minimum.  The reference's own input (upper-triangular U(0,1)) has
// sigma_min / sigma_max ~ 2^-n: at n = 5000 most columns end far below
// fp64's range, and without the floor the solve did not converge in 60
// sweeps (profiles/r3_refshape); columns above it keep one-sided Jacobi's
// relative accuracy (n = 300: U orthogonal to 1e-12).  0 = off.
__device__ __forceinline__ bool needs_rotation(float gpp, float gqq, float gpq, float tol,
                                               int absmode, float floor = 0.0f) {
  if (absmode) return fabsf(gpq) > tol;
  const float nrm = __builtin_amdgcn_sqrtf(gpp) * __builtin_amdgcn_sqrtf(gqq);
  return nrm > 0.0f && fabsf(gpq) > tol * nrm && fminf(gpp, gqq) > floor;
}
__device__ __forceinline__ bool needs_rotation(double gpp, double gqq, double gpq, double tol,
                                               int absmode, double floor = 0.0) {
  if (absmode) return fabs(gpq) > tol;
  const double nrm = sqrt(gpp) * sqrt(gqq);
  return nrm > 0.0 && fabs(gpq) > tol * nrm && fmin(gpp, gqq) > floor;
}
// Effective sine of a rotation for the second-order stop test
// (svdj_stop.h): |s| times the larger ratio of the two columns' norms after
// it (d = squared norms); 0 for no rotation.  Hardware rcp / sqrt (~1 ulp:
// a stop-test statistic; the IEEE division and square root were ~30
// instructions on the EVD solver lane's step).
template <typename T>
__device__ __forceinline__ float eff_sine(T s, T dp, T dq) {
  if (s == T(0)) return 0.0f;
  const float a = (float)fabs(dp), b = (float)fabs(dq);
  const float lo = fminf(a, b), hi = fmaxf(a, b);
  return lo > 0.0f ? fabsf((float)s) * __builtin_amdgcn_sqrtf(hi * __builtin_amdgcn_rcpf(lo)) : 1.0f;
}
// The negligible-column floor of this solve (metric[2..3], a double).
template <typename T>
__device__ __forceinline__ T norm_floor(const uint32_t* metric) {
  return (T)*reinterpret_cast<const double*>(metric + 2);
}

// Rotation of one slot, branch-free (the solve sits on the EVD's critical
// path; the selects avoid exec-mask branches): c = 1, s = t = 0 when the
// test fails.  fp32: raw v_sqrt/v_rcp/v_rsq (~1 ulp) -- (c, s) only steer G;
// the fp64 Q is built from t.
__device__ __forceinline__ bool rotation_fast(float gpp, float gqq, float gpq, float tol,
                                              int absmode, float floor, float& c, float& s,
                                              float& t) {
  const bool rot = needs_rotation(gpp, gqq, gpq, tol, absmode, floor);
  // not `rot ? gpq : 1`: the rotation does not wait for the test (two
  // independent chains; a non-rotation is selected away below)
  const float g = gpq != 0.0f ? gpq : 1.0f;
  const float tau = (gqq - gpp) * __builtin_amdgcn_rcpf(2.0f * g);
  const float at = fabsf(tau);
  const float t_big = 0.5f * __builtin_amdgcn_rcpf(at);
  const float t_reg = __builtin_amdgcn_rcpf(at + __builtin_amdgcn_sqrtf(fmaf(tau, tau, 1.0f)));
  const float tt = at > 1e18f ? t_big : t_reg;
  t = rot ? (tau < 0.0f ? -tt : tt) : 0.0f;
  c = __builtin_amdgcn_rsqf(fmaf(t, t, 1.0f));
  s = t * c;
  return rot;
}
__device__ __forceinline__ bool rotation_fast(double gpp, double gqq, double gpq, double tol,
                                              int absmode, double floor, double& c, double& s,
                                              double& t) {
  const bool rot = needs_rotation(gpp, gqq, gpq, tol, absmode, floor);
  const double g = gpq != 0.0 ? gpq : 1.0;
  const double tau = (gqq - gpp) / (2.0 * g);
  const double at = fabs(tau);
  const double tt = at > 1e150 ? 0.5 / at : 1.0 / (at + sqrt(fma(tau, tau, 1.0)));
  t = rot ? (tau < 0.0 ? -tt : tt) : 0.0;
  c = 1.0 / sqrt(fma(t, t, 1.0));
  s = t * c;
  return rot;
}
// fp64 1/sqrt(x) for x in [1, 2^60]: fp32 hardware estimate (~2^-22) and two
// Newton steps in fp64 (quadratic: 2^-44, then below fp64 rounding).
__device__ __forceinline__ double rsqrt64(double x) {
  double y = (double)__builtin_amdgcn_rsqf((float)x);
  const double hx = 0.5 * x;
  y = y * (1.5 - hx * y * y);
  y = y * (1.5 - hx * y * y);
  return y;
}

// Circle-method players of slot a at step st (the same movement as the DPP
// shifts of the register Q: firsts move right, seconds left, player N-1 fixed
// in slot 0).  Ring of R = N-1 positions; slot a >= 1 has its first at
// position a-1 and its second at 2W-2-a; the player at position x after st
// steps is ((x - st) mod R + 1) mod R.  Checked against the DPP movement by
// tests/test_schedule.py::test_evd_ring_matches_dpp_movement.
template <int W>
__device__ __forceinline__ int ring_player(int pos, int st) {
  constexpr int R = 2 * W - 1;
  int x = pos - st;
  x += x < 0 ? R : 0;
  return x + 1 == R ? 0 : x + 1;
}
template <int W>
__device__ __forceinline__ void ring_slot(int a, int st, int& p, int& q) {
  p = a == 0 ? 2 * W - 1 : ring_player<W>(a - 1, st);
  q = ring_player<W>(2 * W - 2 - a, st);
}
// ---- position space.  The circle method fixes WHERE things happen and moves
// the players: ring positions 0..R-1 (R = 2W-1) plus the fixed position R of
// player N-1; slot a >= 1 owns positions (a-1, 2W-2-a), slot 0 owns (R, R-1).
// Every step each ring player advances one position, so an off-diagonal G
// entry at positions (P1, P2) moves to (P1+1, P2+1) (mod R; R stays R).
// Storing G by POSITION pair -- double-buffered, the update phase reads step
// st's buffer at the block's positions and writes the moved entries into the
// other buffer -- makes every thread's LDS addresses static for the whole
// kernel: no per-step index arithmetic.  Which entries of a block hold the
// next step's pairs is static as well (next_meeting).
template <int W>
__host__ __device__ constexpr int pos_next(int P) {
  return P == 2 * W - 1 ? P : (P + 1 == 2 * W - 1 ? 0 : P + 1);
}
template <int W>
__host__ __device__ constexpr int ring_slot_of(int pos) {  // slot of a ring position
  return pos == 2 * W - 1 ? 0 : (pos <= W - 2 ? pos + 1 : 2 * W - 2 - pos);
}
// Where the players now at positions (P1, P2) meet at the NEXT step: returns
// 2*slot + (the player at P1 is that slot's first), or -1 if they do not.
template <int W>
__host__ __device__ constexpr int next_meeting(int P1, int P2) {
  constexpr int R = 2 * W - 1;
  if (P1 == R || P2 == R) {
    const int o = P1 == R ? P2 : P1;
    if (pos_next<W>(o) != R - 1) return -1;  // N-1 meets the second of slot 0
    return P1 == R ? 1 : 0;
  }
  const int n1 = pos_next<W>(P1), n2 = pos_next<W>(P2);
  if (ring_slot_of<W>(n1) != ring_slot_of<W>(n2)) return -1;
  return 2 * ring_slot_of<W>(n1) + (n1 <= W - 2 ? 1 : 0);
}
// Packed strict upper triangle of an N x N position-pair matrix.
template <int N>
__host__ __device__ constexpr int tri_idx(int i, int j) {
  const int a = i < j ? i : j, b = i < j ? j : i;
  return a * N - a * (a + 1) / 2 + (b - a - 1);
}
// Position of player x at step 0 (inverse of ring_slot at st = 0).
template <int W>
__host__ __device__ constexpr int pos0(int x) {
  return x == 2 * W - 1 ? 2 * W - 1 : (x == 0 ? 2 * W - 2 : x - 1);
}
template <int W>
__host__ __device__ constexpr int slot_first_pos(int a) { return a == 0 ? 2 * W - 1 : a - 1; }
template <int W>
__host__ __device__ constexpr int slot_second_pos(int a) { return 2 * W - 2 - a; }
template <int W>
__host__ __device__ constexpr int block_duty(int a, int b) {  // 256*e + meeting, or -1
  for (int e = 0; e < 4; ++e) {
    const int x = (e >> 1) ? slot_second_pos<W>(a) : slot_first_pos<W>(a);
    const int y = (e & 1) ? slot_second_pos<W>(b) : slot_first_pos<W>(b);
    const int mt = next_meeting<W>(x, y);
    if (mt >= 0) return 256 * e + mt;
  }
  return -1;
}

// ---- inner orderings.  The kernel below is written against an ordering
// policy: where slot a's two players sit (first_pos / second_pos), how
// positions move per step (pos_next, prev_pos), which position pairs meet at
// the next step (next_meeting), the players of a slot at step st, and the
// register-Q movement (move).
//   EVD_CYCLIC: the circle-method round robin over all 2W players, 2W-1
//               steps per sweep (every pair of the 2W x 2W Gram);
//   EVD_BIP   : the bipartite ordering of the cross pairs only, W steps per
//               sweep: X players (block i) fixed at positions 0..W-1, the Y
//               player at Y-position p (position W+p) moves to p-1 (mod W);
//               slot a pairs positions (a, W+a).  Cross steps of a block
//               sweep use it (mode 2): the blocks' own columns are mutually
//               orthogonal when a cross step starts and the full-Gram step
//               at the start of every sweep rotates the within-block pairs,
//               so every column pair is still rotated once per sweep at half
//               the EVD steps (tests/test_schedule.py: bipartite data-flow
//               emulation; CPU block sweeps: same sweep count +-1).
enum { EVD_CYCLIC = 0, EVD_BIP = 1 };
template <int W, int ORD>
struct Ord;
template <int W>
struct Ord<W, EVD_CYCLIC> {
  static constexpr int R = 2 * W - 1;
  __host__ __device__ static constexpr int pos_next(int P) { return svdj::pos_next<W>(P); }
  __host__ __device__ static constexpr int prev_pos(int P) {
    return P == 2 * W - 1 ? P : (P == 0 ? 2 * W - 2 : P - 1);
  }
  __host__ __device__ static constexpr int slot_of(int pos) { return ring_slot_of<W>(pos); }
  __host__ __device__ static constexpr int next_meeting(int P1, int P2) {
    return svdj::next_meeting<W>(P1, P2);
  }
  __host__ __device__ static constexpr int pos0(int x) { return svdj::pos0<W>(x); }
  __host__ __device__ static constexpr int first_pos(int a) { return slot_first_pos<W>(a); }
  __host__ __device__ static constexpr int second_pos(int a) { return slot_second_pos<W>(a); }
  __host__ __device__ static constexpr int first0(int a) { return a == 0 ? 2 * W - 1 : a; }
  __host__ __device__ static constexpr int second0(int a) { return a == 0 ? 0 : 2 * W - 1 - a; }
  __device__ static void players(int a, int st, int& p, int& q) { ring_slot<W>(a, st, p, q); }
  // firsts shift right, seconds shift left; slot 0's first (player 2W-1)
  // stays, slot 1 takes slot 0's second, slot W-1's second is its own first
  template <typename V>
  __device__ static void move(V& f, V& s, int slot) {
    const V f_r = dpp_shr1(f), s_r = dpp_shr1(s), s_l = dpp_shl1(s);
    const V nf = slot == 0 ? f : (slot == 1 ? s_r : f_r);
    const V ns = slot == W - 1 ? f : s_l;
    f = nf;
    s = ns;
  }
};
// Lane i <- lane i+1 with wrap (DPP wave_rol:1).
__device__ __forceinline__ int dpp_rol1(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0x134, 0xf, 0xf, false);
}
// Lane i <- lane i ^ 32 (v_permlane32_swap of a value with itself).
__device__ __forceinline__ int half_swap(int v) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (threadIdx.x & 32) ? (int)r[0] : (int)r[1];
}
template <int W>
__device__ __forceinline__ int bip_shift(int v, int slot) {  // slot a <- slot a+1 (mod W)
  const int r = dpp_rol1(v);
  if constexpr (W == 32) return slot == W - 1 ? half_swap(r) : r;  // two slot groups per wave
  return r;
}
template <int W>
__device__ __forceinline__ float bip_shift(float v, int slot) {
  return __int_as_float(bip_shift<W>(__float_as_int(v), slot));
}
template <int W>
__device__ __forceinline__ double bip_shift(double v, int slot) {
  const long long x = __double_as_longlong(v);
  const int lo = bip_shift<W>((int)(x & 0xffffffff), slot), hi = bip_shift<W>((int)(x >> 32), slot);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int W>
struct Ord<W, EVD_BIP> {
  static_assert(W == 32 || W == 64 || W <= 16, "bipartite Q movement: one or two slot groups per wave");
  static constexpr int R = W;
  __host__ __device__ static constexpr int pos_next(int P) {
    return P < W ? P : (P == W ? 2 * W - 1 : P - 1);
  }
  __host__ __device__ static constexpr int prev_pos(int P) {
    return P < W ? P : (P == 2 * W - 1 ? W : P + 1);
  }
  __host__ __device__ static constexpr int slot_of(int pos) { return pos < W ? pos : pos - W; }
  __host__ __device__ static constexpr int next_meeting(int P1, int P2) {
    const int n1 = pos_next(P1), n2 = pos_next(P2);
    if ((n1 < W) == (n2 < W) || slot_of(n1) != slot_of(n2)) return -1;
    return 2 * slot_of(n1) + (n1 < W ? 1 : 0);
  }
  __host__ __device__ static constexpr int pos0(int x) { return x; }
  __host__ __device__ static constexpr int first_pos(int a) { return a; }
  __host__ __device__ static constexpr int second_pos(int a) { return W + a; }
  __host__ __device__ static constexpr int first0(int a) { return a; }
  __host__ __device__ static constexpr int second0(int a) { return W + a; }
  __device__ static void players(int a, int st, int& p, int& q) {
    p = a;
    q = W + (a + st) % W;
  }
  template <typename V>
  __device__ static void move(V& f, V& s, int slot) {
    (void)f;
    s = bip_shift<W>(s, slot);
  }
};
template <int W, int ORD>
__host__ __device__ constexpr int block_duty_o(int a, int b) {  // 256*e + meeting, or -1
  using O = Ord<W, ORD>;
  for (int e = 0; e < 4; ++e) {
    const int x = (e >> 1) ? O::second_pos(a) : O::first_pos(a);
    const int y = (e & 1) ? O::second_pos(b) : O::first_pos(b);
    const int mt = O::next_meeting(x, y);
    if (mt >= 0) return 256 * e + mt;
  }
  return -1;
}

// Which slot-pair blocks (a < b) each thread owns, computed at compile time.
// Thread roles: the W blocks holding the next step's pairs ("duty" blocks:
// their owners solve the rotations, W = 32 / 64 of them) go to the first W
// lanes of wave 0 -- the only lanes that solve, so only wave 0 carries the
// solve latency and it does no Q work; the other blocks follow in rows taken
// in complementary pairs 0, W-2, 1, W-3, ... (two paired rows hold W blocks,
// so a wave's lanes share few slots and the record reads broadcast).
// blk[j * NT + t] = (a << 8) | b of thread t's j-th block, 0xffff if none.
// OPT (fp32, bipartite, 1024 threads): the table of tools/evd_deal_opt.py
// instead -- the same duty blocks, the other blocks placed so the 32 lanes of
// each LDS lane group hit distinct banks where possible (modelled LDS cycles
// per step W=64: 1144 -> 812, conflict share 45 -> 22 %).
template <int W, int NT, int ORD = EVD_CYCLIC, bool OPT = false>
struct EvdDeal {
  static constexpr int NOFF = W * (W - 1) / 2;
  static constexpr int MAXOFF = (NOFF + NT - 1) / NT;
  unsigned short blk[MAXOFF * NT];
  constexpr EvdDeal() : blk{} {
    if constexpr (OPT) {
      static_assert(ORD == EVD_BIP && NT == 1024 && (W == 32 || W == 64), "optimised dealing tables");
      const unsigned short* t = W == 64 ? kEvdDealF32_W64_bip : kEvdDealF32_W32_bip;
      for (int g = 0; g < MAXOFF * NT; ++g) blk[g] = t[g];
      return;
    }
    using O = Ord<W, ORD>;
    int g = 0;
    // duty block of each next-step slot s: the positions that slot's players
    // occupy NOW are one behind its own positions
    for (int s = 0; s < W; ++s) {
      int a = O::slot_of(O::prev_pos(O::first_pos(s))), b = O::slot_of(O::prev_pos(O::second_pos(s)));
      if (a > b) {
        const int x = a;
        a = b;
        b = x;
      }
      blk[g++] = (unsigned short)((a << 8) | b);
    }
    for (int i = 0; i < W - 1; ++i) {
      const int a = (i & 1) ? W - 2 - (i >> 1) : (i >> 1);
      for (int b = a + 1; b < W; ++b)
        if (block_duty_o<W, ORD>(a, b) < 0) blk[g++] = (unsigned short)((a << 8) | b);
    }
    for (; g < MAXOFF * NT; ++g) blk[g] = 0xffff;
  }
};

// Compile-time check of the dealing: the first W entries are the duty blocks
// of next-step slots 0..W-1, and every block is dealt exactly once.
template <int W, int NT, int ORD, bool OPT = false>
constexpr bool evd_deal_ok() {
  constexpr EvdDeal<W, NT, ORD, OPT> d{};
  int seen[W * W] = {};
  int dealt = 0;
  for (int g = 0; g < EvdDeal<W, NT, ORD, OPT>::MAXOFF * NT; ++g) {
    if (d.blk[g] == 0xffff) continue;
    const int a = d.blk[g] >> 8, b = d.blk[g] & 255;
    if (!(a < b && b < W) || seen[a * W + b]++) return false;
    ++dealt;
    const int duty = block_duty_o<W, ORD>(a, b);
    if (g < W && (duty < 0 || ((duty & 255) >> 1) != g)) return false;
    if (g >= W && duty >= 0) return false;
  }
  return dealt == EvdDeal<W, NT, ORD, OPT>::NOFF;
}
static_assert(evd_deal_ok<32, evd_threads(32), EVD_CYCLIC>(), "EVD block dealing");
static_assert(evd_deal_ok<64, evd_threads(64), EVD_CYCLIC>(), "EVD block dealing");
static_assert(evd_deal_ok<32, evd_threads(32), EVD_BIP>(), "EVD block dealing");
static_assert(evd_deal_ok<64, evd_threads(64), EVD_BIP>(), "EVD block dealing");
static_assert(evd_deal_ok<64, 1024, EVD_BIP, true>(), "optimised EVD block dealing");
static_assert(evd_deal_ok<32, 1024, EVD_BIP, true>(), "optimised EVD block dealing");
// which dealing a kernel uses
template <typename T, int W, int NT, int ORD>
__host__ __device__ constexpr bool evd_deal_opt() {
  return sizeof(T) == 4 && ORD == EVD_BIP && NT == 1024 && (W == 32 || W == 64);
}

template <typename T, int W, int ORD>
__global__ __launch_bounds__(evd_threads(W)) void evd_kernel(
    const int32_t* __restrict__ pairs, int full, const T* __restrict__ slabs, int nchunk,
    T* __restrict__ D, T* __restrict__ Qout, int32_t* __restrict__ skip, T tol, int absmode,
    int max_inner, uint32_t* __restrict__ metric) {
  constexpr int NT = evd_threads(W);
  constexpr int NWAVE = NT / SVDJ_WAVE;
  constexpr int N = 2 * W;
  using O = Ord<W, ORD>;
  constexpr int R = O::R;               // steps per sweep
  constexpr int NTRI = N * (N - 1) / 2;
  constexpr int GPW = SVDJ_WAVE / W;    // Q row groups per wave
  // Q row groups: waves 1..NWAVE-1 (wave 0 solves).  Giving the solver wave
  // Q rows as well measured neutral (round 2, profiles/r2_evd_unroll): the
  // step is bound by the G update's LDS traffic, not by the Q rows.
  constexpr int QW0 = 1;  // first Q wave
  constexpr int NGRP = (NWAVE - QW0) * GPW;
  constexpr int RPL = (N + NGRP - 1) / NGRP;  // Q rows per lane (the last group may idle)
  constexpr bool DOPT = evd_deal_opt<T, W, NT, ORD>();
  constexpr int MAXOFF = EvdDeal<W, NT, ORD, DOPT>::MAXOFF;
  static_assert(W >= 4 && W <= 64 && NWAVE >= 2, "EVD geometry");
  using QT = double;  // fp32 Q measured 8 % faster with 10x worse V orthogonality
  static constexpr EvdDeal<W, NT, ORD, DOPT> deal{};

  __shared__ T Gb[2][NTRI + 1];  // off-diagonal G by position pair, double-buffered;
                                 // element NTRI takes the writes that go nowhere
  __shared__ T dg[N];        // assembled diagonal (player order)
  // rotation records by global step parity (structure of arrays): (c, s) in
  // the data precision steer G, (cq, sq) in the Q precision rotate Q (fp64
  // for fp32 data: normalised once, by the solver), (dp, dq) are the slot's
  // diagonals after its rotation
  // records as pairs: one 8/16-byte LDS access per (c, s), (dp, dq), (cq, sq)
  using T2 = Pair2<T>;
  using QT2 = Pair2<QT>;
  __shared__ T2 rcs[2][W], rdd[2][W];
  __shared__ QT2 rq[2][W];
  __shared__ int rot_flag[2];  // any rotation in sweep (parity), written by wave 0
  __shared__ float wmax[NWAVE];
  __shared__ int wneed[NWAVE];
  __shared__ int need_any;

  const int pair = blockIdx.x;
  const int bi = pairs[2 * pair], bj = pairs[2 * pair + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T nfloor = norm_floor<T>(metric);

  // ---- assemble G: diagonal first (player order), then every off-diagonal
  // entry into position space for step 0; split-K slabs summed in fp64
  if (full) {
    const T* s0 = slabs + (size_t)pair * nchunk * (4 * W * W);
    for (int a = tid; a < N; a += NT) {
      double acc = 0;
      for (int c = 0; c < nchunk; ++c) acc += (double)s0[(size_t)c * 4 * W * W + a * N + a];
      dg[a] = (T)acc;
    }
  } else {
    for (int a = tid; a < N; a += NT) dg[a] = D[a < W ? bi * W + a : bj * W + (a - W)];
  }
  __syncthreads();
  {
    float mx = 0.0f;
    int need = 0;
    // store an entry at its step-0 position; fold it into the convergence
    // value and the "anything to rotate" test
    auto visit = [&](int r, int c, T g) {
      Gb[0][tri_idx<N>(O::pos0(r), O::pos0(c))] = g;
      const T grr = dg[r], gcc = dg[c];
      const T d = sqrt(grr) * sqrt(gcc);
      if (d > T(0) && (absmode || (grr > nfloor && gcc > nfloor))) {
        const float v = (float)(fabs(g) / d);
        mx = v > mx ? v : mx;
      }
      need |= needs_rotation(grr, gcc, g, tol, absmode, nfloor) ? 1 : 0;
    };
    // Slab sums with 16-byte loads, all chunks of a group in flight at once
    // (one dependent global load per entry and chunk was ~12 us per kernel).
    constexpr int EV = 16 / (int)sizeof(T);
    if (full) {
      const T* s0 = slabs + (size_t)pair * nchunk * (4 * W * W);
      for (int gi = tid; gi < N * N / EV; gi += NT) {
        double acc[EV];
#pragma unroll
        for (int u = 0; u < EV; ++u) acc[u] = 0.0;
#pragma unroll SVDJ_EVD_SLAB_UNROLL
        for (int k = 0; k < nchunk; ++k) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(s0 + (size_t)k * 4 * W * W + gi * EV);
          const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
          for (int u = 0; u < EV; ++u) acc[u] += (double)e[u];
        }
#pragma unroll
        for (int u = 0; u < EV; ++u) {
          const int i = gi * EV + u, r = i / N, c = i % N;
          if (r < c) visit(r, c, (T)acc[u]);
        }
      }
    } else {
      // couplings inside a block are zero (blocks are kept internally orthogonal)
      for (int i = tid; i < N * N; i += NT) {
        const int r = i / N, c = i % N;
        if (r < c && (c < W || r >= W)) Gb[0][tri_idx<N>(O::pos0(r), O::pos0(c))] = T(0);
      }
      const T* s0 = slabs + (size_t)pair * nchunk * (W * W);
      for (int gi = tid; gi < W * W / EV; gi += NT) {
        double acc[EV];
#pragma unroll
        for (int u = 0; u < EV; ++u) acc[u] = 0.0;
#pragma unroll SVDJ_EVD_SLAB_UNROLL
        for (int k = 0; k < nchunk; ++k) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(s0 + (size_t)k * W * W + gi * EV);
          const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
          for (int u = 0; u < EV; ++u) acc[u] += (double)e[u];
        }
#pragma unroll
        for (int u = 0; u < EV; ++u) {
          const int i = gi * EV + u;
          visit(i / W, W + i % W, (T)acc[u]);
        }
      }
    }
    mx = wave_max(mx);
    need = __any(need) ? 1 : 0;
    if (lane == 0) {
      wmax[wave] = mx;
      wneed[wave] = need;
    }
    __syncthreads();
    if (tid == 0) {
      float m2 = 0.0f;
      int n2 = 0;
      for (int w = 0; w < NWAVE; ++w) {
        m2 = wmax[w] > m2 ? wmax[w] : m2;
        n2 |= wneed[w];
      }
      atomic_max_pos(&metric[0], m2);
      need_any = n2;
    }
    __syncthreads();
  }
  // If no pair passes the rotation test, the first pass would rotate nothing
  // (G never changes): it is skipped exactly.
  const bool run = need_any != 0;

  // ---- this thread's blocks and their static addresses
  int ba[MAXOFF], bb[MAXOFF];
  int rd[MAXOFF][4], wr[MAXOFF][4];  // read / write BYTE offsets into a G buffer (NTRI: no write)
  int pw = (int)sizeof(T) * NTRI, sv = -1;  // solve duty (256*e + meeting; j = 0 only), pending byte offset
#pragma unroll
  for (int j = 0; j < MAXOFF; ++j) {
    const int code = deal.blk[j * NT + tid];
    ba[j] = bb[j] = -1;
#pragma unroll
    for (int e = 0; e < 4; ++e) rd[j][e] = wr[j][e] = 0;
    if (code != 0xffff) {
      const int a = code >> 8, b = code & 255;
      ba[j] = a;
      bb[j] = b;
      const int pa[2] = {O::first_pos(a), O::second_pos(a)};
      const int pb[2] = {O::first_pos(b), O::second_pos(b)};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int x = pa[e >> 1], y = pb[e & 1];
        rd[j][e] = (int)sizeof(T) * tri_idx<N>(x, y);
        wr[j][e] = (int)sizeof(T) * tri_idx<N>(O::pos_next(x), O::pos_next(y));
        if (j == 0 && tid < W) {
          const int mt = O::next_meeting(x, y);
          if (mt >= 0) {
            wr[j][e] = (int)sizeof(T) * NTRI;  // within-slot entry next step: written one phase later
            pw = (int)sizeof(T) * tri_idx<N>(O::pos_next(O::pos_next(x)), O::pos_next(O::pos_next(y)));
            sv = 256 * e + mt;
          }
        }
      }
    }
  }
  T pend = T(0);

  // ---- slot layout state of the register Q (waves 1..NWAVE-1)
  const bool qlane = wave >= QW0;
  const int slot = lane % W;
  const int grp = (wave - QW0) * GPW + lane / W;
  int pf = O::first0(slot);   // first player of this slot
  int ps = O::second0(slot);  // second player
  QT qf[RPL], qs[RPL];
#pragma unroll
  for (int i = 0; i < RPL; ++i) {
    const int k = grp * RPL + i;
    qf[i] = (k == pf) ? QT(1) : QT(0);
    qs[i] = (k == ps) ? QT(1) : QT(0);
  }

  // ---- prologue: step 0's rotations from the assembled G
  // second-order stop test (svdj_stop.h): largest effective sine and count
  // of the rotations this solver lane solved (the final look-ahead rotation
  // included: conservative)
  float smax = 0.0f;
  uint32_t rcount = 0;
  auto publish = [&](int b, int ns, T c, T sn, T t, T dfp, T dsp) {
    smax = fmaxf(smax, eff_sine(sn, dfp, dsp));
    rcount += sn != T(0) ? 1u : 0u;
    rcs[b][ns] = T2{c, sn};
    rdd[b][ns] = T2{dfp, dsp};
    if constexpr (sizeof(QT) == sizeof(T)) {
      rq[b][ns] = QT2{c, sn};
    } else {  // fp64 (c, s) of the fp32 t, normalised in fp64
      const double td = (double)t, c64 = rsqrt64(fma(td, td, 1.0));
      rq[b][ns] = QT2{c64, td * c64};
    }
  };
  // rotations seen by this solver lane in the current / next inner sweep
  // (OR-reduced over wave 0 once per sweep: no per-step flag store)
  int racc = 0, racc_next = 0;
  if (run && tid < W) {
    const int fa = O::first_pos(tid), sa = O::second_pos(tid);
    int p, q;
    O::players(tid, 0, p, q);
    const T gpp = dg[p], gqq = dg[q];
    const T gpq = Gb[0][tri_idx<N>(fa, sa)];
    T c, s, t;
    const bool rot = rotation_fast(gpp, gqq, gpq, tol, absmode, nfloor, c, s, t);
    racc = rot;
    // thread tid's duty block holds next-step slot tid (EvdDeal), so phase 0's
    // pending write moves this coupling to its step-1 position
    pend = rot ? T(0) : gpq;
    publish(0, tid, c, s, t, gpp - t * gpq, gqq + t * gpq);
  }
  __syncthreads();

  // One block's update J^T G J (entries moved to their next-step positions)
  // and, for a duty block, the next step's rotation of its slot.
  // One block's update J^T G J (entries moved to their next-step positions)
  // and, for a duty block, the next step's rotation of its slot.  Split in a
  // read half and a compute/write half so a thread issues the LDS reads of
  // ALL its blocks before any write: Gb[b] and Gb[nb] are disjoint but the
  // compiler cannot prove it, so a fused per-block read-compute-write
  // serialises the read latency of every block.
  // G entry at byte offset `off` of buffer b (b is a compile-time constant in
  // the unrolled step loop, so the buffer base folds into the ds offset)
  auto gat = [&](int b, int off) -> T& {
    return *reinterpret_cast<T*>(reinterpret_cast<char*>(&Gb[b][0]) + off);
  };
  struct BlkIn {
    T g00, g01, g10, g11, ca, sa, cb, sb, dx, dy;
  };
  auto load_block = [&](int j, int b, bool duty, BlkIn& k) {
    k.g00 = gat(b, rd[j][0]);
    k.g01 = gat(b, rd[j][1]);
    k.g10 = gat(b, rd[j][2]);
    k.g11 = gat(b, rd[j][3]);
    const T2 ra = rcs[b][ba[j]], rb = rcs[b][bb[j]];
    k.ca = ra.x;
    k.sa = ra.y;
    k.cb = rb.x;
    k.sb = rb.y;
    k.dx = k.dy = T(0);
    if (duty) {
      const int e = sv >> 8;
      const T2 da = rdd[b][ba[j]], db = rdd[b][bb[j]];
      k.dx = (e >> 1) ? da.y : da.x;
      k.dy = (e & 1) ? db.y : db.x;
    }
  };
  auto finish_block = [&](int j, int nb, bool duty, bool last, const BlkIn& k) {
    const T h00 = k.ca * k.g00 - k.sa * k.g10, h01 = k.ca * k.g01 - k.sa * k.g11;
    const T h10 = k.sa * k.g00 + k.ca * k.g10, h11 = k.sa * k.g01 + k.ca * k.g11;
    const T h[4] = {k.cb * h00 - k.sb * h01, k.sb * h00 + k.cb * h01, k.cb * h10 - k.sb * h11,
                    k.sb * h10 + k.cb * h11};
    if (duty) {
      const int e = sv >> 8;
      const int ns = (sv & 255) >> 1;
      const bool x_first = sv & 1;
      const T g = e == 0 ? h[0] : e == 1 ? h[1] : e == 2 ? h[2] : h[3];
      const T df = x_first ? k.dx : k.dy, ds = x_first ? k.dy : k.dx;
      T c, sn, t;
      const bool rot = rotation_fast(df, ds, g, tol, absmode, nfloor, c, sn, t);
      if (last) racc_next |= rot; else racc |= rot;
      pend = rot ? T(0) : g;
      publish(nb, ns, c, sn, t, df - t * g, ds + t * g);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) gat(nb, wr[j][q]) = h[q];
  };
  auto update_blocks = [&](int b, int nb, bool solver, bool last) {
    BlkIn k[MAXOFF];
#pragma unroll
    for (int j = 0; j < MAXOFF; ++j)
      if (ba[j] >= 0) load_block(j, b, solver && j == 0 && sv >= 0, k[j]);
    // the coupling of this step's pair, solved last phase (or in the
    // prologue), moved on to its next-step position (dummy if no duty)
    gat(nb, pw) = pend;
#pragma unroll
    for (int j = 0; j < MAXOFF; ++j)
      if (ba[j] >= 0) finish_block(j, nb, solver && j == 0 && sv >= 0, last, k[j]);
  };

  bool any = false;
  int gs = 0;  // global step counter: step gs reads buffer gs & 1, records gs & 1
  int sw = 0, st = 0;
  // One step with the buffer parity as a compile-time constant (the loop
  // below alternates the two instantiations): every G / record address is a
  // loop-invariant register plus an immediate.  Returns true when done.
  auto step = [&](auto parity) -> bool {
    constexpr int b = decltype(parity)::value, nb = b ^ 1;
    const bool last = st + 1 == R;  // this phase solves step 0 of the next sweep
    if (wave == 0) {
      // solver wave: its duty blocks (lanes < W, j = 0) and nothing else of Q
      update_blocks(b, nb, true, last);
      if (last) {  // every rotation of sweep sw is decided by now
        const int rot = __any(racc) ? 1 : 0;
        if (lane == 0) rot_flag[sw & 1] = rot;
        racc = racc_next;
        racc_next = 0;
      }
    } else {
      // Q waves: this step's Q rotation (records read up front)
      const QT2 rqs = rq[b][slot];
      const QT cq = rqs.x, sq = rqs.y;
      update_blocks(b, nb, false, last);
      // Q <- Q J in registers (c = 1, s = 0 for no rotation)
#pragma unroll
      for (int i = 0; i < RPL; ++i) {
        const QT x = qf[i], y = qs[i];
        qf[i] = cq * x - sq * y;
        qs[i] = sq * x + cq * y;
      }
      // advance the ordering (DPP lane moves of the slot layout)
#pragma unroll
      for (int i = 0; i < RPL; ++i) O::move(qf[i], qs[i], slot);
      O::move(pf, ps, slot);
    }
    __syncthreads();
    ++gs;
    if (++st < R) return false;
    st = 0;
    if (!rot_flag[sw & 1]) return true;
    any = true;
    return ++sw >= max_inner;
  };
  if (run && max_inner > 0)
    while (!step(std::integral_constant<int, 0>{}) && !step(std::integral_constant<int, 1>{})) {
    }

  if (wave == 0 && any) {  // second-order stop test input (metric[4], [5]; svdj_stop.h)
    const float sm = wave_max(smax);
    const uint32_t rc_ = wave_sum(rcount);
    if (lane == 0) {
      atomic_max_pos(&metric[4], sm);
      atomicAdd(&metric[5], rc_);
    }
  }
  if (tid == 0) {
    skip[pair] = any ? 0 : 1;
    if (any) atomicAdd(&metric[1], 1u);
  }
  // Full mode re-measured the diagonal from the data: always refresh D.
  if (!any && !full) return;
  if (any) {
    if (qlane) {
      T* qo = Qout + (size_t)pair * N * N;
#pragma unroll
      for (int i = 0; i < RPL; ++i) {
        const int k = grp * RPL + i;
        if (k < N) {
          qo[k * N + pf] = (T)qf[i];
          qo[k * N + ps] = (T)qs[i];
        }
      }
    }
    // diagonals after the last executed step (records of step gs - 1)
    if (tid < W) {
      const int lb = (gs - 1) & 1;
      int p, q;
      O::players(tid, R - 1, p, q);
      D[p < W ? bi * W + p : bj * W + (p - W)] = rdd[lb][tid].x;
      D[q < W ? bi * W + q : bj * W + (q - W)] = rdd[lb][tid].y;
    }
  } else {
    for (int a = tid; a < N; a += NT) D[a < W ? bi * W + a : bj * W + (a - W)] = dg[a];
  }
}

// ----------------------------------------- evd, cross-only bipartite (mode 3)
// The EVD of a cross step that tracks only what the bipartite ordering
// reads: the W x W cross couplings C and the 2W diagonals.  When a cross
// step starts, each block's own columns are mutually orthogonal (the
// full-Gram step that opens every sweep rotates the within-block pairs), so
// G = [[Dx, C], [C^T, Dy]].  A rotation of (x_i, y) creates within-block
// couplings only at first order in its sine, and those feed back into the
// cross couplings at second order: the update
//   C'[i][j] = c_i c_k C[i][j] - s_i s_k C[k][pi(i)]     (y_j paired with x_k)
// drops them.  Near convergence the sines are tiny and the rotations are the
// exact ones; early on they differ slightly, which the next outer visit of
// the pair re-measures from the data.  CPU emulation (fp32 / fp64, n = 512 /
// 1024, W = 32 / 64): the same sweep counts as the full bipartite EVD +-1,
// the same accuracy.
//
// Position space: at step t, Y position p holds y_{(p + t) mod W}; slot a
// pairs x_a with position a.  E[i][p] = C[i][y at p].  The update pairs
// E[i][p] with E[p][i] (a STATIC transpose pair) and the new values move
// one position left: E_{t+1}[i][p] = E'_t[i][p+1].  Groups {E[i][i+d],
// E[i+d][i]} along diagonals d = 1..W/2:
//   * wave 0, lane a = slot a, holds d = 1 and d = 2 in REGISTERS: its next
//     active coupling E_{t+1}[a][a] = E'_t[a][a+1] needs only values of
//     lanes a+1 and a+2 (their rotations, E_t[a+1][a] = lane a+1's settled
//     coupling, E_t[a+2][a] = lane a+1's previous d = 1 result), fetched
//     with DPP lane rotates -- the solve chain has no LDS read on it;
//   * waves 1.. hold d = 3..W/2 in LDS (row stride W, bank-conflict-free),
//     two diagonals per wave; the d = 2 / d = 3 values cross through LDS.
// ONE barrier per step.  The kernel does not accumulate Q: every step's
// rotations go to global memory as tangent records, and qbuild_kernel forms
// the fp64 (c, s) and Q = J_0 J_1 ... row-parallel on many CUs (rows of Q
// evolve independently).  Measured in isolation (tools/micro/evd_bench.hip, 8
// pairs, W = 64): register Q accumulation and the solve chain made the
// per-step time ~2000 cycles; the G update itself was not the limit.  Round
// 6 ablations (profiles/r6_evd): of 33 us per launch, 14 us are barriers,
// lane rotates, bookkeeping, assembly and launch; the records cost 3.8 us
// (their fp64 (c, s), now formed by the Q builds, and the per-step wait for
// their stores), the rotation solve 6 us.
// DPW: coupling diagonals per wave >= 1 (W = 64; W = 32 keeps 2, one per lane half)
template <int W, int DPW = 2>
__host__ __device__ constexpr int cross_threads() {
  return W == 64 ? SVDJ_WAVE * (1 + (W / 2 - 2 + DPW - 1) / DPW) : 512;
}
constexpr int kCrossMaxInner = 4;  // inner sweeps whose rotation records fit the workspace

// ABL (tools/micro/evd_bench.hip only; production launches ABL = 0): bit 0
// no rotation records; bit 1 waves >= 1 skip their coupling updates
// (barriers kept); bit 2 the solver lane skips the rotation (c = 1, s = 0);
// bit 3 the solver lane skips its LDS coupling read and write; bit 4 no
// steps at all (assembly, launch and the epilogue only).
template <typename T, int W, int ABL = 0, int DPW = 2>
__global__ __launch_bounds__((cross_threads<W, DPW>())) void evd_cross_kernel(
    const int32_t* __restrict__ pairs, const T* __restrict__ slabs, int nchunk,
    T* __restrict__ D, T* __restrict__ rec, int32_t* __restrict__ nsteps,
    int32_t* __restrict__ skip, T tol, int absmode, int max_inner, uint32_t* __restrict__ metric) {
  static_assert(W == 32 || W == 64, "cross EVD: W = 32 or 64");
  static_assert(W == 64 || DPW == 2, "W = 32: two diagonals per wave (one per lane half)");
  constexpr int NT = cross_threads<W, DPW>();
  constexpr int NWAVE = NT / SVDJ_WAVE;
  static_assert(W == 32 ? NWAVE - 1 == (W / 2 - 2) / 2 : NWAVE - 1 == (W / 2 - 2 + DPW - 1) / DPW,
                "DPW diagonals per wave >= 1");
  constexpr int N = 2 * W;
  using T2 = Pair2<T>;
  using Q2 = Pair2<double>;

  __shared__ T Eb[2][W * W];  // cross couplings by (x slot, y position), double-buffered
  __shared__ T dg[N];
  __shared__ T2 rcs[2][W];
  __shared__ int rot_flag[2];
  __shared__ float wmax[NWAVE];
  __shared__ int wneed[NWAVE];
  __shared__ int need_any;

  const int pair = blockIdx.x;
  const int bi = pairs[2 * pair], bj = pairs[2 * pair + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T nfloor = norm_floor<T>(metric);

  // ---- assemble: diagonals from D, E_0[i][p] = C[i][p] (split-K slabs
  // summed in fp64), convergence value and the "anything to rotate" test
  for (int a = tid; a < N; a += NT) dg[a] = D[a < W ? bi * W + a : bj * W + (a - W)];
  __syncthreads();
  {
    float mx = 0.0f;
    int need = 0;
    constexpr int EV = 16 / (int)sizeof(T);
    const T* s0 = slabs + (size_t)pair * nchunk * (W * W);
    for (int gi = tid; gi < W * W / EV; gi += NT) {
      double acc[EV];
#pragma unroll
      for (int u = 0; u < EV; ++u) acc[u] = 0.0;
#pragma unroll SVDJ_EVD_SLAB_UNROLL
      for (int k = 0; k < nchunk; ++k) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(s0 + (size_t)k * W * W + gi * EV);
        const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
        for (int u = 0; u < EV; ++u) acc[u] += (double)e[u];
      }
#pragma unroll
      for (int u = 0; u < EV; ++u) {
        const int i = gi * EV + u;
        const T g = (T)acc[u];
        Eb[0][i] = g;
        const T grr = dg[i / W], gcc = dg[W + i % W];
        const T d = sqrt(grr) * sqrt(gcc);
        if (d > T(0) && (absmode || (grr > nfloor && gcc > nfloor))) {
          const float v = (float)(fabs(g) / d);
          mx = v > mx ? v : mx;
        }
        need |= needs_rotation(grr, gcc, g, tol, absmode, nfloor) ? 1 : 0;
      }
    }
    mx = wave_max(mx);
    need = __any(need) ? 1 : 0;
    if (lane == 0) {
      wmax[wave] = mx;
      wneed[wave] = need;
    }
    __syncthreads();
    if (tid == 0) {
      float m2 = 0.0f;
      int n2 = 0;
      for (int w = 0; w < NWAVE; ++w) {
        m2 = wmax[w] > m2 ? wmax[w] : m2;
        n2 |= wneed[w];
      }
      atomic_max_pos(&metric[0], m2);
      need_any = n2;
    }
    __syncthreads();
  }
  const bool run = need_any != 0 && (ABL & 16) == 0;
  const int inner = max_inner < kCrossMaxInner ? max_inner : kCrossMaxInner;

  // ---- LDS groups of waves >= 1: (i, d), d = DPW (w - 1) + 3 + j (W = 64:
  // all on every lane; W = 32: d = 2w+1 on lanes 0..31, 2w+2 on 32..63);
  // gv bit j: group j exists on this lane (the half diagonal has W/2 groups)
  constexpr int G = W == 64 ? DPW : 1;
  int gi[G], gp[G], rd0[G], rd1[G], wr0[G], wr1[G];
  uint32_t gv = 0;
#pragma unroll
  for (int jg = 0; jg < G; ++jg) {
    const int i = W == 64 ? lane : (lane & 31);
    const int d = W == 64 ? DPW * (wave - 1) + 3 + jg : 2 * wave + 1 + (lane >> 5);
    const bool ok = wave >= 1 && d <= W / 2 && !(d == W / 2 && i >= W / 2);
    const int p = (i + d) % W;
    gi[jg] = i;
    gp[jg] = p;
    rd0[jg] = i * W + p;
    rd1[jg] = p * W + i;
    wr0[jg] = i * W + (p + W - 1) % W;
    wr1[jg] = p * W + (i + W - 1) % W;
    gv |= ok ? 1u << jg : 0u;
  }

  // ---- solver lanes (wave 0, lane a < W): slot a's state in registers
  const bool solver = wave == 0 && lane < W;
  const int a = lane % W;
  T rc = T(1), rs = T(0);   // rotation of slot a at the current step
  T rdx = T(0), rdy = T(0); // x_a / y at position a after the current step's rotation
  T pend = T(0);            // slot a's coupling after the current step's rotation
  T pend_prev = T(0);       // ... after the previous step: E_t[a][a-1]
  T g1 = T(0);              // E_t[a][a+1]
  T h2src = T(0);           // E_t[a+1][a-1] (lane a-1's E_t[(a-1)+2][a-1])
  T dx_out = T(0), dy_out = T(0);
  T* rq = rec + (size_t)pair * (kCrossMaxInner * W) * W;
  T rt = T(0);  // tangent of the latest solved rotation; its fp64 record is
                // written at the start of the next phase (steps 0 .. gs-1 are
                // recorded; the look-ahead rotation solved in the final phase
                // is never used)
  // second-order stop test (svdj_stop.h): largest effective sine and count
  // of the rotations applied (recorded); the effective sine of the latest
  // solved rotation is formed when it is recorded, off the solve chain
  float smax = 0.0f;
  uint32_t rcount = 0;
  auto solve = [&](T dx, T dy, T g, bool& rot) {
    T c, sn, t;
    if constexpr ((ABL & 4) != 0) {
      rot = false;
      c = T(1);
      sn = t = T(0);
    } else {
      rot = rotation_fast(dx, dy, g, tol, absmode, nfloor, c, sn, t);
    }
    rc = c;
    rs = sn;
    rt = t;
    rdx = dx - t * g;
    rdy = dy + t * g;
    pend = rot ? T(0) : g;
  };
  auto record = [&](int step) {  // before the next solve: rs, rdx, rdy still its inputs'
    smax = fmaxf(smax, eff_sine(rs, rdx, rdy));
    rcount += rs != T(0) ? 1u : 0u;
    if constexpr ((ABL & 1) != 0) return;
    // the tangent only: the Q builds form the fp64 (c, s) from it
    // (rotation_cs), off this lane's step
    if (step < kCrossMaxInner * W) rq[(size_t)step * W + a] = rt;
  };
  int racc = 0, racc_next = 0;
  if (run && solver) {  // step 0 of slot a
    pend_prev = Eb[0][a * W + (a + W - 1) % W];
    h2src = Eb[0][((a + 1) % W) * W + (a + W - 1) % W];
    g1 = Eb[0][a * W + (a + 1) % W];
    bool rot;
    solve(dg[a], dg[W + a], Eb[0][a * W + a], rot);
    racc = rot;
    rcs[0][a] = T2{rc, rs};
  }
  __syncthreads();

  bool any = false;
  int gs = 0, sw = 0, st = 0;
  auto step = [&](auto parity) -> bool {
    constexpr int b = decltype(parity)::value, nb = b ^ 1;
    const bool last = st + 1 == W;  // this phase solves step 0 of the next inner sweep
    if (wave == 0) {
      // neighbours' values (slot a+1, a+2) by lane rotates; E_t[a][a+2] from LDS
      const T g2 = solver && (ABL & 8) == 0 ? Eb[b][a * W + (a + 2) % W] : T(0);
      // fp64 record of step gs (solved in the previous phase) while the LDS
      // read is in flight: off the barrier-to-barrier critical path
      if (solver) record(gs);
      const T c1 = bip_shift<W>(rc, a), s1 = bip_shift<W>(rs, a);
      const T c2 = bip_shift<W>(c1, a), s2 = bip_shift<W>(s1, a);
      const T h1 = bip_shift<W>(pend_prev, a);  // E_t[a+1][a]
      const T h2 = bip_shift<W>(h2src, a);      // E_t[a+2][a]
      const T dyn = bip_shift<W>(rdy, a);       // y at position a+1 after this step
      if (solver) {
        const T cc1 = rc * c1, ss1 = rs * s1, cc2 = rc * c2, ss2 = rs * s2;
        const T n0_1 = cc1 * g1 - ss1 * h1;  // E_{t+1}[a][a]: slot a's next coupling
        const T n1_1 = cc1 * h1 - ss1 * g1;  // E_{t+1}[a+1][a-1]
        const T n0_2 = cc2 * g2 - ss2 * h2;  // E_{t+1}[a][a+1]
        const T n1_2 = cc2 * h2 - ss2 * g2;  // E_{t+1}[a+2][a-1] (a d = 3 group's input)
        if constexpr ((ABL & 8) == 0) Eb[nb][((a + 2) % W) * W + (a + W - 1) % W] = n1_2;
        dx_out = rdx;
        dy_out = rdy;
        pend_prev = pend;
        g1 = n0_2;
        h2src = n1_1;
        bool rot;
        solve(rdx, dyn, n0_1, rot);
        if (last) racc_next |= rot; else racc |= rot;
        rcs[nb][a] = T2{rc, rs};
      }
      if (last) {  // every rotation of inner sweep sw is decided by now
        const int r = __any(racc) ? 1 : 0;
        if (lane == 0) rot_flag[sw & 1] = r;
        racc = racc_next;
        racc_next = 0;
      }
    } else if constexpr ((ABL & 2) == 0) {
      T e0[G], e1[G];
      T2 ri[G], rp[G];
#pragma unroll
      for (int j = 0; j < G; ++j)
        if (gv >> j & 1u) {
          e0[j] = Eb[b][rd0[j]];
          e1[j] = Eb[b][rd1[j]];
          ri[j] = rcs[b][gi[j]];
          rp[j] = rcs[b][gp[j]];
        }
#pragma unroll
      for (int j = 0; j < G; ++j)
        if (gv >> j & 1u) {
          const T cc = ri[j].x * rp[j].x, ss = ri[j].y * rp[j].y;
          Eb[nb][wr0[j]] = cc * e0[j] - ss * e1[j];
          Eb[nb][wr1[j]] = cc * e1[j] - ss * e0[j];
        }
    }
    // LDS-only barrier: __syncthreads would also wait for the record stores
    // (vmcnt(0)) every step; nothing in the loop reads global memory
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    ++gs;
    if (++st < W) return false;
    st = 0;
    if (!rot_flag[sw & 1]) return true;
    any = true;
    return ++sw >= inner;
  };
  if (run && inner > 0)
    while (!step(std::integral_constant<int, 0>{}) && !step(std::integral_constant<int, 1>{})) {
    }

  if (wave == 0 && any) {  // second-order stop test input (metric[4], [5]; svdj_stop.h)
    const float sm = wave_max(smax);
    const uint32_t rc_ = wave_sum(rcount);
    if (lane == 0) {
      atomic_max_pos(&metric[4], sm);
      atomicAdd(&metric[5], rc_);
    }
  }
  if (tid == 0) {
    skip[pair] = any ? 0 : 1;
    nsteps[pair] = gs;
    if (any) atomicAdd(&metric[1], 1u);
  }
  if (any && solver) {  // diagonals after the last executed step (gs - 1)
    D[bi * W + a] = dx_out;
    D[bj * W + ((a + gs - 1) & (W - 1))] = dy_out;
  }
}

// Q = J_0 J_1 ... J_{steps-1} of a cross-step EVD from its fp64 rotation
// records (evd_cross_kernel), row-parallel: row k of Q evolves on its own
// (q_k <- q_k J_t), so a pair's 2W rows spread over several workgroups and
// CUs instead of sitting in the EVD workgroup's registers.  Lane = slot a
// (W = 32: two slot groups per wave); per row and step one 2x2 fp64 rotation
// of (Q[k][x_a], Q[k][y at position a]) and a lane rotate of the y column
// (position a takes what position a+1 held).  The records of up to 64 steps
// are staged in LDS first with wide loads (one global latency instead of
// one per step: read step by step from L2 the kernel was latency bound),
// then read two steps ahead.  Rounded to the data type once, at the end.
// R rows per lane: 4 when a step has few pairs (latency: more workgroups per
// pair), 16 with many pairs (throughput: each workgroup stages the pair's
// records once for 4x the rows).
constexpr int kQbThreads = 256;
constexpr int kQbChunk = 64;  // steps staged in LDS at a time
// fp64 (c, s) of a recorded tangent (evd_cross_kernel records t only):
// fp32 data -- the fp32 t normalised in fp64 (Q stays orthogonal to fp64
// rounding); fp64 data -- rotation_fast's own c = 1 / sqrt(1 + t^2), s = t c.
__device__ __forceinline__ Pair2<double> rotation_cs(float t) {
  const double td = (double)t, c = rsqrt64(fma(td, td, 1.0));
  return Pair2<double>{c, td * c};
}
__device__ __forceinline__ Pair2<double> rotation_cs(double t) {
  const double c = 1.0 / sqrt(fma(t, t, 1.0));
  return Pair2<double>{c, t * c};
}
template <int W, int R>
__host__ __device__ constexpr int qbuild_blocks() {  // workgroups per pair
  return (2 * W) / (R * (SVDJ_WAVE / W) * (kQbThreads / SVDJ_WAVE));
}
template <typename T, int W, int R>
__global__ __launch_bounds__(kQbThreads) void qbuild_kernel(
    const T* __restrict__ rec, const int32_t* __restrict__ nsteps,
    const int32_t* __restrict__ skip, T* __restrict__ Qall) {
  constexpr int N = 2 * W;
  constexpr int GPW = SVDJ_WAVE / W;
  static_assert(qbuild_blocks<W, R>() * R * GPW * (kQbThreads / SVDJ_WAVE) == N, "row cover");
  using Q2 = Pair2<double>;
  __shared__ Q2 rs[kQbChunk * W];
  const int pair = blockIdx.x;
  if (skip[pair]) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int a = lane % W;
  const int k0 = ((blockIdx.y * (kQbThreads / SVDJ_WAVE) + wave) * GPW + lane / W) * R;
  const int ns = nsteps[pair];
  const T* rp = rec + (size_t)pair * (kCrossMaxInner * W) * W;
  double qx[R], qy[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    qx[i] = (k0 + i == a) ? 1.0 : 0.0;
    qy[i] = (k0 + i == W + a) ? 1.0 : 0.0;
  }
  for (int t0 = 0; t0 < ns; t0 += kQbChunk) {
    const int nc = ns - t0 < kQbChunk ? ns - t0 : kQbChunk;
    for (int i = threadIdx.x; i < nc * W; i += kQbThreads) rs[i] = rotation_cs(rp[(size_t)t0 * W + i]);
    __syncthreads();
    Q2 n0 = rs[a], n1 = nc > 1 ? rs[W + a] : Q2{1.0, 0.0};
    for (int t = 0; t < nc; ++t) {
      const Q2 cs = n0;
      n0 = n1;
      if (t + 2 < nc) n1 = rs[(t + 2) * W + a];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const double x = qx[i], y = qy[i];
        qx[i] = cs.x * x - cs.y * y;
        qy[i] = bip_shift<W>(cs.y * x + cs.x * y, a);
      }
    }
    __syncthreads();  // the next chunk overwrites rs
  }
  T* qo = Qall + (size_t)pair * N * N;
  const int yc = W + (a + ns) % W;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    qo[(k0 + i) * N + a] = (T)qx[i];
    qo[(k0 + i) * N + yc] = (T)qy[i];
  }
}

// ------------------------------------------------------------------ apply
// Q fragments are read kQPD k-steps ahead of their MFMA (row-layout Q).
constexpr int kQPD = 8;
template <typename T, int W>
__host__ __device__ constexpr int apply_threads() { return kApplyThreads; }
template <typename T, int W>
__global__ __launch_bounds__((apply_threads<T, W>())) void apply_kernel(
    T* __restrict__ A, int lda, int a_chunks, int rows_a, int m_pad, T* __restrict__ V,
    int ldv, int rows_v, int n_v, const int32_t* __restrict__ pairs, const T* __restrict__ Qall,
    const int32_t* __restrict__ skip) {
  using M = Mfma<T>;
  constexpr int TL = M::TILE;
  constexpr int KG = M::KG;
  constexpr int N = 2 * W;
  constexpr int NK = N / KG;   // k values per lane
  constexpr int NCT = N / TL;  // output column tiles
  constexpr int LDQ = N + (sizeof(T) == 8 ? 16 : 0);
  constexpr int NTH = apply_threads<T, W>();
  constexpr int WAVES = NTH / SVDJ_WAVE;
  __shared__ alignas(16) T Qs[N * LDQ];

  const int pair = blockIdx.x;
  if (skip[pair]) return;
  const int bi = pairs[2 * pair], bj = pairs[2 * pair + 1];
  int chunk = blockIdx.y;
  T* base;
  int ld, r_begin, r_end;
  if (chunk < a_chunks) {
    base = A;
    ld = lda;
    r_begin = chunk * rows_a;
    r_end = min(m_pad, r_begin + rows_a);
  } else {
    chunk -= a_chunks;
    base = V;
    ld = ldv;
    r_begin = chunk * rows_v;
    r_end = min(n_v, r_begin + rows_v);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lc = M::lane_col(lane), kg = M::lane_kg(lane);
  // Column k of X = [A_bi A_bj] is base + col(k)*ld.  The lane-dependent
  // part of every address (k group, row lane, acc row group) is folded into
  // one 64-bit lane offset; the per-k / per-tile part is wave-uniform, so the
  // address arithmetic stays in SGPRs.
  T* const xi = base + (size_t)bi * W * ld;
  T* const xj = base + (size_t)bj * W * ld;
  const uint32_t ld_off = (uint32_t)(kg * ld + lc);
  const uint32_t st_off = (uint32_t)(M::acc_row_lane(lane) * ld + lc);
  // Q fragments are loop-invariant: small Q (<= 64 VGPRs of fragments) is
  // left to the compiler to hoist into registers; larger Q is re-read from
  // LDS per row tile (the empty asm with a memory clobber blocks the hoist).
  constexpr bool kHoistQ = (NK * NCT * (int)sizeof(T)) / 4 <= 64;
  auto load_tile = [&](T (&x)[NK], int r) {
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      const int k0 = kk * KG;
      const T* src = (k0 < W ? xi + (size_t)k0 * ld : xj + (size_t)(k0 - W) * ld);
      x[kk] = src[ld_off + (uint32_t)r];
    }
  };
  int r0 = r_begin + wave * TL;
  T xv[NK];
  const T* Qg = Qall + (size_t)pair * N * N;
  // fp64: Q in A-operand fragment order -- for (column tile, group of VEC
  // k-steps, lane) the VEC operands are contiguous, one 16-byte LDS read per
  // VEC MFMAs (fp64 W=64 apply 912 -> 845 us; fp32 W=64 319 -> 338 us, so
  // fp32 keeps the row layout with an element-wise fill -- 16-byte and
  // LDS-DMA fills measured slower or equal, round 2)
  constexpr bool kQFrag = sizeof(T) == 8;
  constexpr int VEC = 16 / (int)sizeof(T);
  using QV = __attribute__((ext_vector_type(VEC))) T;
  const QV* Qgv = reinterpret_cast<const QV*>(Qg);
  if constexpr (kQFrag) {
    for (int iv = threadIdx.x; iv < N * N / VEC; iv += NTH) {
      const QV q = Qgv[iv];
#pragma unroll
      for (int u = 0; u < VEC; ++u) {
        const int i = iv * VEC + u;
        const int k = i / N, c = i % N;
        const int kk = k / KG, kgi = k % KG, ct = c / TL, lci = c % TL;
        Qs[((ct * (NK / VEC) + kk / VEC) * 64 + kgi * TL + lci) * VEC + kk % VEC] = q[u];
      }
    }
  } else {
    for (int i = threadIdx.x; i < N * N; i += NTH) Qs[(i / N) * LDQ + (i % N)] = Qg[i];
  }
  __syncthreads();
  if (r0 >= r_end) return;
  load_tile(xv, r0);
  while (true) {
    const int rn = r0 + WAVES * TL;
    const bool more = rn < r_end;
    T xn[NK];
    if (more) load_tile(xn, rn);  // next tile in flight during this tile's MFMAs
    if constexpr (!kHoistQ) asm volatile("" ::: "memory");
    constexpr int kCtUnroll = kHoistQ ? NCT : 1;
#pragma unroll kCtUnroll
    for (int ct = 0; ct < NCT; ++ct) {
      typename M::acc_t acc = M::zero();
      if constexpr (kQFrag) {
        using V4 = __attribute__((ext_vector_type(VEC))) T;
        const V4* qv = reinterpret_cast<const V4*>(Qs) + (size_t)ct * (NK / VEC) * 64 + lane;
        V4 cur = qv[0];
#pragma unroll
        for (int g = 0; g < NK / VEC; ++g) {
          V4 nxt = cur;
          if (g + 1 < NK / VEC) nxt = qv[(g + 1) * 64];
#pragma unroll
          for (int e = 0; e < VEC; ++e) acc = M::mfma(cur[e], xv[g * VEC + e], acc);
          cur = nxt;
        }
      } else {
        // Q fragments are read kQPD k-steps ahead of their MFMA (sched_barrier
        // keeps the order; just in time, each ds_read's latency sat between
        // two dependent MFMAs).  Two interleaved accumulation chains per wave
        // were measured slower (1269 vs 1145 us, W=64).
        constexpr int PD = kQPD < NK ? kQPD : NK;
        T qa[PD];
#pragma unroll
        for (int i = 0; i < PD; ++i) qa[i] = Qs[(i * KG + kg) * LDQ + ct * TL + lc];
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const T a = qa[kk % PD];
          if (kk + PD < NK) qa[kk % PD] = Qs[((kk + PD) * KG + kg) * LDQ + ct * TL + lc];
          acc = M::mfma(a, xv[kk], acc);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      const int c0 = ct * TL;
      T* dst = (c0 < W ? xi + (size_t)c0 * ld : xj + (size_t)(c0 - W) * ld);
#pragma unroll
      for (int e = 0; e < M::NACC; ++e)
        dst[(size_t)M::acc_row_uni(e) * ld + (st_off + (uint32_t)r0)] = acc[e];
    }
    if (!more) break;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) xv[kk] = xn[kk];
    r0 = rn;
  }
}

// A wave-uniform pointer moved to SGPRs (v_readfirstlane), so an access
// p[lane offset] can use the scalar-base + 32-bit VGPR offset address form.
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}

// Element i of a base pointer with a 32-bit byte offset (the caller
// guarantees i * sizeof(T) < 2^32): for a wave-uniform base the address is
// SGPR base + 32-bit VGPR offset instead of a 64-bit VGPR address.
template <typename T>
__device__ __forceinline__ T& at_u32(T* base, uint32_t i) {
  using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
  return *reinterpret_cast<T*>(reinterpret_cast<B*>(base) + i * (uint32_t)sizeof(T));
}

// -------------------------------------------------- apply on bf16 matrix cores
// fp32 data, bf16 MFMA (v_mfma_f32_32x32x16_bf16, 16x the f32 MFMA rate):
// every operand is split into NP round-to-nearest bf16 parts,
//   x = x0 + x1 + x2,  |x - x0| <= 2^-9|x|, |x - x0 - x1| <= 2^-18|x|, ...
// and the products of total order < NP are accumulated in fp32 (bf16 x bf16
// products are exact):  NP = 3 -> 6 MFMAs (00 01 10 02 11 20), dropped terms
// are O(2^-26)|x||q|, i.e. fp32 rounding level;  NP = 2 -> 3 MFMAs, O(2^-18)
// (the "bf16x3" fast mode).  The 2W x 2W Q is split once per workgroup into
// LDS, already in A-operand fragment order (one ds_read_b128 per part);
// the X tile is split in registers right after its loads land.
// Same transposed formulation as apply_kernel: Out^T = Q^T X^T, lane = row.
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;

template <int NP>
__device__ __forceinline__ void split_bf16(float x, __bf16 (&p)[NP]) {
  float r = x;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    p[i] = (__bf16)r;  // round to nearest even
    r -= (float)p[i];
  }
}

// Eight values at once, two per instruction: v_cvt_pk_bf16_f32 rounds a pair,
// the pair goes back to fp32 with a shift and a mask, and one v_pk_add_f32
// takes both remainders -- 4.5 VALU instructions per value and 3 parts
// instead of 7.5 for split_bf16 one value at a time (the compiler converts
// each scalar alone), bitwise the same parts.
using bf16x2 = __attribute__((ext_vector_type(2))) __bf16;
using f32x2 = __attribute__((ext_vector_type(2))) float;
template <int NP>
__device__ __forceinline__ void split_bf16x8(const float (&v)[8], bf16x8 (&parts)[NP]) {
  f32x2 r[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = f32x2{v[2 * j], v[2 * j + 1]};
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    bf16x2 p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] = __builtin_convertvector(r[j], bf16x2);
      if (i + 1 < NP) r[j] -= __builtin_convertvector(p[j], f32x2);
    }
    parts[i] = __builtin_shufflevector(__builtin_shufflevector(p[0], p[1], 0, 1, 2, 3),
                                       __builtin_shufflevector(p[2], p[3], 0, 1, 2, 3), 0, 1, 2, 3,
                                       4, 5, 6, 7);
  }
}

// Products of total order >= LO (small terms first).
template <int NP, int LO>
__device__ __forceinline__ f32x16 mfma_split(const bf16x8 (&q)[NP], const bf16x8 (&x)[NP],
                                             f32x16 acc) {
#pragma unroll
  for (int ord = NP - 1; ord >= LO; --ord)
#pragma unroll
    for (int a = 0; a <= ord; ++a)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(q[a], x[ord - a], acc, 0, 0, 0);
  return acc;
}

// Waves own OUTPUT COLUMN tiles, not rows: wave w computes the 32 output
// columns ct = w % NCT of the row tile (row group w / NCT; W = 64: all four
// waves on one 32-row tile, W = 32: two 32-row tiles), so its split Q - I
// fragments (NKB x NP bf16x8, 96 VGPRs for W = 64) stay in registers for
// the whole workgroup.  The X tile is loaded once: wave w loads and splits
// the k columns of its own output tile (k blocks 2ct, 2ct+1) into an LDS
// image in B-fragment order (double-buffered, one barrier per tile), and
// keeps those raw fp32 values for the epilogue Y = X + X (Q - I), where a
// v_permlane32_swap moves them from the B-operand lanes to the accumulator
// lanes.  No operand is re-read from global memory.
//
// Delta form (Q - I): the identity part is never rounded inside the
// MFMA.  The bf16 MFMA's internal accumulation is not IEEE round-to-nearest,
// and with X Q directly a dominant diagonal term biased every sum (column
// norms drifted 780 eps in 400 near-identity applies, round 1); with the
// identity added back in fp32 the drift is 0.14-0.17 eps against 3 eps for
// the f32 MFMA (tools/probe_apply.py, profiles/r3_s3/bf16x6).
template <int W, int NP>
__global__ __launch_bounds__(kApplyThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void apply_split_kernel(
    float* __restrict__ A, int lda, int a_chunks, int rows_a, int m_pad, float* __restrict__ V,
    int ldv, int rows_v, int n_v, const int32_t* __restrict__ pairs,
    const float* __restrict__ Qall, const int32_t* __restrict__ skip, int vfirst) {
  constexpr int N = 2 * W;
  constexpr int NCT = N / 32;                   // output column tiles
  constexpr int NKB = N / 16;                   // 16-deep k blocks
  constexpr int WAVES = kApplyThreads / SVDJ_WAVE;
  constexpr int RG = WAVES / NCT;               // 32-row groups per tile
  constexpr int TR = 32 * RG;                   // rows per tile
  static_assert(NCT * RG == WAVES && NKB == 2 * NCT, "wave <-> (column tile, row group)");
  static_assert(W % 16 == 0, "k blocks must not straddle the two column blocks");
  __shared__ bf16x8 Xf[2][RG][NKB][NP][SVDJ_WAVE];

  const int pair = blockIdx.x;
  if (skip[pair]) return;
  const int bi = pairs[2 * pair], bj = pairs[2 * pair + 1];
  // vfirst: V's row chunks dispatched before A's, so A's rows are the most
  // recently written when the next step's Gram reads them
  const int vch = gridDim.y - a_chunks;
  int chunk = vfirst ? (blockIdx.y < (unsigned)vch ? a_chunks + (int)blockIdx.y : (int)blockIdx.y - vch)
                     : (int)blockIdx.y;
  float* base;
  int ld, r_begin, r_end;
  if (chunk < a_chunks) {
    base = A;
    ld = lda;
    r_begin = chunk * rows_a;
    r_end = min(m_pad, r_begin + rows_a);
  } else {
    chunk -= a_chunks;
    base = V;
    ld = ldv;
    r_begin = chunk * rows_v;
    r_end = min(n_v, r_begin + rows_v);
  }
  if (r_begin >= r_end) return;
  // wave index through readfirstlane: everything derived from it (own) is
  // known uniform and stays in SGPRs
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 31, h = lane >> 5;
  const int ct = wave % NCT, rg = wave / NCT;
  float* const xi = base + (size_t)bi * W * ld;
  float* const xj = base + (size_t)bj * W * ld;
  // the wave's own 32 columns (k blocks 2ct, 2ct+1 = output tile ct)
  float* const own = ct * 32 < W ? xi + (size_t)(ct * 32) * ld : xj + (size_t)(ct * 32 - W) * ld;

  // Q - I fragments of column tile ct: (kb, lane) = Q[kb*16 + 8h + e][ct*32 + c] - delta
  bf16x8 qf[NKB][NP];
  {
    const float* Qg = Qall + (size_t)pair * N * N + ct * 32 + c;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = kb * 16 + 8 * h + e;
        __bf16 p[NP];
        split_bf16<NP>(Qg[(size_t)k * N] - (k == ct * 32 + c ? 1.0f : 0.0f), p);
#pragma unroll
        for (int i = 0; i < NP; ++i) qf[kb][i][e] = p[i];
      }
  }
  // raw X of this wave's k blocks for rows r .. r+31: x[kbl][e] = X[r + c][ct*32 + 16 kbl + 8h + e].
  // Column bases are wave-uniform (SGPRs, readfirstlane) with a 32-bit lane
  // offset, so the loads use the scalar-base address form instead of one
  // 64-bit VGPR address per column (32 VGPRs the operand prefetch needs).
  const uint32_t lane_off = (uint32_t)(8 * h * ld + c);
  auto load = [&](float (&x)[2][8], int r) {
#pragma unroll
    for (int kbl = 0; kbl < 2; ++kbl)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        x[kbl][e] = at_u32(own + (size_t)(16 * kbl + e) * ld, lane_off + (uint32_t)r);
  };
  const uint32_t st_off = (uint32_t)(4 * h * ld + c);
  // Loads run two tiles ahead: tile t's raw values are in one register set
  // while tile t+1's are in flight in the other (the loop is unrolled by two
  // so both sets are static); tile t+2 is issued into the first set as soon
  // as tile t's values are in LDS and in the epilogue registers.  One tile of
  // look-ahead left ~16 KB in flight per workgroup, short of what the HBM
  // latency under load needs.
  auto tile = [&](float (&xr)[2][8], int t) -> bool {
    const int rt = r_begin + t * TR;
    if (rt >= r_end) return false;  // uniform over the workgroup
    const int buf = t & 1;
    const int r0 = rt + rg * 32;      // this wave's rows
    const bool mine = r0 < r_end;
    // split this tile's own k blocks into the shared B-fragment image
    if (mine) {
#pragma unroll
      for (int kbl = 0; kbl < 2; ++kbl) {
        bf16x8 parts[NP];
        split_bf16x8<NP>(xr[kbl], parts);
#pragma unroll
        for (int i = 0; i < NP; ++i) Xf[buf][rg][2 * ct + kbl][i][lane] = parts[i];
      }
    }
    // epilogue operand: own raw values moved to accumulator lanes.  Output
    // register g*4+i of lane (c, h) is column 8g + 4h + i of the tile; lane
    // half h holds columns 16 kbl + 8h + e.
    float xo[16];
#pragma unroll
    for (int kbl = 0; kbl < 2; ++kbl)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float keep = h ? xr[kbl][4 + i] : xr[kbl][i];
        const float give = h ? xr[kbl][i] : xr[kbl][4 + i];
        const float got = __int_as_float(half_swap(__float_as_int(give)));
        xo[(2 * kbl) * 4 + i] = h ? got : keep;
        xo[(2 * kbl + 1) * 4 + i] = h ? keep : got;
      }
    if (r0 + 2 * TR < r_end) load(xr, r0 + 2 * TR);
    __syncthreads();
    if (mine) {
      f32x16 acc = Mfma<float>::zero(), lo = Mfma<float>::zero();
      // B operands of k block kb + 1 are read while kb's MFMAs run
      bf16x8 xs[NP], xn[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) xs[i] = Xf[buf][rg][0][i][lane];
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        if (kb + 1 < NKB) {
#pragma unroll
          for (int i = 0; i < NP; ++i) xn[i] = Xf[buf][rg][kb + 1][i][lane];
        }
        // the high-order product in its own accumulator, the small terms in
        // a second one
        lo = mfma_split<NP, 1>(qf[kb], xs, lo);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qf[kb][0], xs[0], acc, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < NP; ++i) xs[i] = xn[i];
      }
      acc += lo;
#pragma unroll
      for (int e = 0; e < 16; ++e)
        at_u32(own + (size_t)Mfma<float>::acc_row_uni(e) * ld, st_off + (uint32_t)r0) = xo[e] + acc[e];
    }
    return true;
  };
  float xa[2][8], xb[2][8];
  const int r0 = r_begin + rg * 32;
  if (r0 < r_end) load(xa, r0);
  if (r0 + TR < r_end) load(xb, r0 + TR);
  for (int t = 0;; t += 2) {
    if (!tile(xa, t)) break;
    if (!tile(xb, t + 1)) break;
  }
}

// ------------------------------------------------------------- quad step
// Two consecutive cross steps fused (fp32, W = 64, split-bf16 apply).  Four
// W-blocks (a, b, c, d) = the block pairs (a,c),(b,d) of step s and
// (a,d),(b,c) of step s+1 (a super-block pair {a,b} x {c,d}, the schedule
// of parallel/schedule.py quad_round_robin / quad_bipartite).  Step s+1's
// couplings are formed in Gram space instead of from the data:
//   gram   : the six cross Grams C_ac, C_bd, C_ad, C_bc, C_ab, C_cd in ONE
//            launch (gram_quad_kernel: each block of the quad read once,
//            products instead of once per step);
//   evd 1  : evd_cross_kernel on (a,c), (b,d)  -> rotation records;
//   T1     : qbuild_quad_kernel<1> -> Q_ac, Q_bd in fp64;
//   update : C(a',d') = [Q_aa;Q_ca]^T [[C_ab,C_ad],[C_cb,C_cd]] [Q_bd;Q_dd] and
//            C(b',c') likewise (quad_update_kernel): exact in Gram space, the
//            within-pair blocks C_ab, C_cd included;
//   evd 2  : evd_cross_kernel on (a,d), (b,c) from those couplings;
//   T      : qbuild_quad_kernel<2> applies the step-(s+1) rotations to the
//            rows of T1 in fp64: T = T1 T2, the whole 256 x 256 transform;
//   apply  : [a b c d] <- [a b c d] T once, for A and V (apply_quad_ts_kernel).
// The data moves through HBM once per two steps instead of twice, and the
// apply contracts over K = 256 instead of 128: its split-bf16 MFMAs, no
// longer waiting on HBM, set the pace.  Numerically it is the two W-block
// steps with the same pairs (same EVDs, the couplings of step s+1 computed
// from the exact rotations of step s), and T is accumulated in fp64 and
// rounded once instead of twice.

// Q of an EVD pair (phase 1, rows of the pair, output fp64 T1) or the quad's
// T (phase 2: rows of all 4 blocks, starting from the phase-1 transforms,
// output T - I split into NP bf16 parts).  Same row-parallel rotation loop as
// qbuild_kernel; a skipped pair contributes the identity (phase 1 writes it:
// T1 is read by update and phase 2 even when its pair did not rotate).
// First element of the split T - I fragment (quad q, 32-row k block kb, 32-column
// tile ct, 16-column sub-tile cs) in the apply's A-operand layout
// (apply_quad_ts_kernel): NP parts of SVDJ_WAVE bf16x8 each; element e of lane
// 16g + i = (T - I)[32 kb + 8g + e][32 ct + 16 cs + i].
__host__ __device__ constexpr size_t ts_frag(int q, int kb, int ct, int cs, int np) {
  return ((((size_t)q * 8 + kb) * 8 + ct) * 2 + cs) * np * SVDJ_WAVE;
}

// Phase 2 writes T - I straight in the apply's split-bf16 fragment layout
// (round 6; a separate split pass over an fp32 T before): a thread's R rows
// k0 .. k0 + R - 1 of one column are elements k0 % 8 .. of one A-operand
// fragment (k block k0 / 32, lane group (k0 / 8) & 3).
template <int PHASE, int R, int NT, int NP = 0>
__global__ __launch_bounds__(NT) void qbuild_quad_kernel(
    const float* __restrict__ rec, const int32_t* __restrict__ nsteps,
    const int32_t* __restrict__ skip, double* __restrict__ T1, bf16x8* __restrict__ Ts = nullptr) {
  static_assert(PHASE == 1 ? NP == 0 : ((NP == 2 || NP == 3) && (R == 2 || R == 4 || R == 8)),
                "phase 2: split T - I, 2 / 4 / 8 rows per thread");
  constexpr int W = 64, N = 2 * W, QN = 4 * W;
  constexpr int WAVES = NT / SVDJ_WAVE;
  static_assert((PHASE == 1 ? N : QN) % (R * WAVES) == 0, "row cover");
  using Q2 = Pair2<double>;
  __shared__ Q2 rs[kQbChunk * W];
  const int pair = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int a = lane;
  const int k0 = (blockIdx.y * WAVES + wave) * R;
  const int ns = skip[pair] ? 0 : nsteps[pair];
  const float* rp = rec + (size_t)pair * (kCrossMaxInner * W) * W;
  const int q = pair >> 1, j = pair & 1;
  double qx[R], qy[R];
  if constexpr (PHASE == 1) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      qx[i] = (k0 + i == a) ? 1.0 : 0.0;
      qy[i] = (k0 + i == W + a) ? 1.0 : 0.0;
    }
  } else {
    // sub-pair j = 0: (a', d'), x = a' (column a of Q_ac), y = d' (column
    // W + a of Q_bd); j = 1: (b', c'), x = b' (Q_bd), y = c' (Q_ac).  Quad
    // row k is block k >> 6 in [a b c d] order: Q_ac holds rows of a, c (even
    // blocks), Q_bd rows of b, d (odd blocks).
    const double* tx = T1 + (size_t)(2 * q + j) * N * N;
    const double* ty = T1 + (size_t)(2 * q + 1 - j) * N * N;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int k = k0 + i, rb = k >> 6, kl = ((rb >> 1) << 6) + (k & 63);
      qx[i] = (rb & 1) == j ? tx[(size_t)kl * N + a] : 0.0;
      qy[i] = (rb & 1) != j ? ty[(size_t)kl * N + W + a] : 0.0;
    }
  }
  for (int t0 = 0; t0 < ns; t0 += kQbChunk) {
    const int nc = ns - t0 < kQbChunk ? ns - t0 : kQbChunk;
    for (int i = threadIdx.x; i < nc * W; i += NT) rs[i] = rotation_cs(rp[(size_t)t0 * W + i]);
    __syncthreads();
    Q2 n0 = rs[a], n1 = nc > 1 ? rs[W + a] : Q2{1.0, 0.0};
    for (int t = 0; t < nc; ++t) {
      const Q2 cs = n0;
      n0 = n1;
      if (t + 2 < nc) n1 = rs[(t + 2) * W + a];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const double x = qx[i], y = qy[i];
        qx[i] = cs.x * x - cs.y * y;
        qy[i] = bip_shift<W>(cs.y * x + cs.x * y, a);
      }
    }
    __syncthreads();
  }
  const int yr = (a + ns) & (W - 1);
  if constexpr (PHASE == 1) {
    double* qo = T1 + (size_t)pair * N * N;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      qo[(size_t)(k0 + i) * N + a] = qx[i];
      qo[(size_t)(k0 + i) * N + W + yr] = qy[i];
    }
  } else {  // element e of lane 16g + i of fragment (kb, ct, cs) = (T - I)[32 kb +
            // 8g + e][32 ct + 16 cs + i]; R < 8 rows per thread fill elements
            // k0 % 8 .. + R - 1 of the fragment
    using bfR = __attribute__((ext_vector_type(R))) __bf16;
    const int xc = (j == 0 ? 0 : W) + a, yc = (j == 0 ? 3 * W : 2 * W) + yr;
    const int kb = k0 >> 5, gg = (k0 >> 3) & 3, e0 = k0 & 7;
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int col = side ? yc : xc;
      bfR parts[NP];
#pragma unroll
      for (int e = 0; e < R; ++e) {
        __bf16 pp[NP];
        // T rounded to fp32 first, then T - I (exact: |T| <= 1)
        const float t = (float)(side ? qy[e] : qx[e]) - (k0 + e == col ? 1.0f : 0.0f);
        split_bf16<NP>(t, pp);
#pragma unroll
        for (int pi = 0; pi < NP; ++pi) parts[pi][e] = pp[pi];
      }
      __bf16* dst = reinterpret_cast<__bf16*>(Ts + ts_frag(q, kb, col >> 5, (col >> 4) & 1, NP) +
                                              (col & 15) + 16 * gg) + e0;
#pragma unroll
      for (int pi = 0; pi < NP; ++pi) *reinterpret_cast<bfR*>(dst + pi * SVDJ_WAVE * 8) = parts[pi];
    }
  }
}

// Step-(s+1) couplings of quad q in Gram space, one workgroup per output
// pair and column half (blockIdx.x = 2q + j, blockIdx.y = oj): j = 0
// C(a',d') = L^T M R with L = Q_ac[:, :W] (rows a;c), M = [[C_ab, C_ad],
// [C_cb, C_cd]] (rows a;c, columns b;d), R = Q_bd[:, W:]; j = 1 C(b',c') =
// Q_bd[:, :W]^T M^T Q_ac[:, W:].  M is summed over the Gram's row chunks in
// fp64, R's and L's columns are staged in LDS (fp32), both products on f32
// MFMA (the data Gram is f32 MFMA as well).  Output: one W x W slab per pair
// of step s+1 (nchunk = 1), the layout evd_cross_kernel reads.
// NT = 512: the same MFMA waves (4, then 2), twice the loads in flight in the
// fill phases (the kernel is load-latency bound: 1 workgroup per CU).
template <int NT>
__global__ __launch_bounds__(NT) void quad_update_kernel(
    const float* __restrict__ slabs, int gch, const double* __restrict__ T1,
    float* __restrict__ upd) {
  constexpr int kUpdThreads = NT;
  // M's row stride is odd (129 = 1 mod 64 banks): its transposed fill and
  // both read orders are conflict-free (MP = N + 4 had 52 % bank-conflict
  // cycles, profiles/r5_prof_final)
  constexpr int W = 64, N = 2 * W, MP = N + 1, HP = 32 + 4;
  using M = Mfma<float>;
  __shared__ float Ms[N * MP];
  __shared__ float Rs[N * HP];  // R[:, 32 oj .. + 32]
  __shared__ float Ys[N * HP];  // Y = Mx R_oj
  __shared__ float Ls[N * (W + 4)];
  const int q = blockIdx.x >> 1, j = blockIdx.x & 1, oj = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double* Rg = T1 + (size_t)(j == 0 ? 2 * q + 1 : 2 * q) * N * N + W + 32 * oj;
  const double* Lg = T1 + (size_t)(j == 0 ? 2 * q : 2 * q + 1) * N * N;
  // 16-byte loads, all issued before the first use (latency-bound otherwise)
#pragma unroll
  for (int u = 0; u < N * 32 / 2 / kUpdThreads; ++u) {
    const int idx = u * kUpdThreads + tid, r = idx >> 4, cc = (idx & 15) * 2;
    const double2 v = *reinterpret_cast<const double2*>(Rg + (size_t)r * N + cc);
    Rs[r * HP + cc] = (float)v.x;
    Rs[r * HP + cc + 1] = (float)v.y;
  }
#pragma unroll
  for (int u = 0; u < N * W / 2 / kUpdThreads; ++u) {
    const int idx = u * kUpdThreads + tid, r = idx >> 5, cc = (idx & 31) * 2;
    const double2 v = *reinterpret_cast<const double2*>(Lg + (size_t)r * N + cc);
    Ls[r * (W + 4) + cc] = (float)v.x;
    Ls[r * (W + 4) + cc + 1] = (float)v.y;
  }
  // slabs of quad q: r = 0 (a,d), 1 (b,c), 2 (a,b), 3 (c,d), gch chunks each
  // (16-byte loads, four independent sums per thread and four slabs' worth in
  // flight: the one-float loop was load-latency bound, 94 us per 128-pair quad
  // step at 83 % wait-any, profiles/r5_prof)
  const float4* base = reinterpret_cast<const float4*>(slabs + (size_t)q * 4 * gch * W * W);
  constexpr int E4 = W * W / 4;
#pragma unroll 4
  for (int idx = tid; idx < 4 * E4; idx += kUpdThreads) {
    const int r = idx / E4, e4 = idx % E4, i = (4 * e4) / W, jj = (4 * e4) % W;
    const float4* p = base + (size_t)r * gch * E4 + e4;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    for (int k = 0; k < gch; ++k) {
      const float4 v = p[(size_t)k * E4];
      s0 += (double)v.x;
      s1 += (double)v.y;
      s2 += (double)v.z;
      s3 += (double)v.w;
    }
    const double sv[4] = {s0, s1, s2, s3};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ju = jj + u;
      const int row = r == 0 ? i : r == 1 ? W + ju : r == 2 ? i : W + i;
      const int col = r == 0 ? W + ju : r == 1 ? i : r == 2 ? ju : W + ju;
      Ms[row * MP + col] = (float)sv[u];
    }
  }
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;
  if (wave < 4) {  // Y = Mx R_oj (N x 32): wave w owns row tile w
    M::acc_t acc = M::zero();
    const int i = wave * 32 + li;
#pragma unroll 8
    for (int l0 = 0; l0 < N; l0 += 2) {
      const int l = l0 + lk;
      const float av = j == 0 ? Ms[i * MP + l] : Ms[l * MP + i];
      acc = M::mfma(av, Rs[l * HP + li], acc);
    }
#pragma unroll
    for (int e = 0; e < M::NACC; ++e) Ys[(wave * 32 + M::acc_row(e, lane)) * HP + li] = acc[e];
  }
  __syncthreads();
  if (wave < 2) {  // out[:, 32 oj ..] = Lx^T Y (W x 32): wave w owns row tile w
    M::acc_t acc = M::zero();
#pragma unroll 8
    for (int k0 = 0; k0 < N; k0 += 2) {
      const int k = k0 + lk;
      acc = M::mfma(Ls[k * (W + 4) + wave * 32 + li], Ys[k * HP + li], acc);
    }
    float* out = upd + (size_t)blockIdx.x * W * W;
#pragma unroll
    for (int e = 0; e < M::NACC; ++e)
      out[(wave * 32 + M::acc_row(e, lane)) * W + 32 * oj + li] = acc[e];
  }
}

// [a b c d] <- [a b c d] T, T-STATIONARY (round 5; 16x16x32 MFMAs round 6).
// The round-4 apply streamed the 384 KB split T through LDS for every 128-row
// tile (3.2 GB of T per 64-pair quad step against 2.1 GB of data; 1.71 ms per
// 128-pair quad step, profiles/r4_quad).  Here a workgroup keeps T in
// REGISTERS for thousands of rows:
//   * 8 waves (two per SIMD), wave w owns output column tile w (32 of the
//     quad's 256 columns, two 16-column sub-tiles) and holds its split T - I
//     slice, 8 k blocks of 32 x 2 sub-tiles x NP bf16x8 = 192 VGPRs for
//     NP = 3, for the whole launch;
//   * the workgroup walks a contiguous range of 32-row tiles of A then V
//     (every tile all 256 columns: it owns its rows, so in place is safe);
//   * each wave LDS-DMAs (global_load_lds_dwordx4) its own 32 columns of the
//     tile two tiles ahead into a wave-private raw image (no VGPRs in
//     flight), splits them -- exactly k block w -- into the shared B-fragment
//     image of the tile (double-buffered, one barrier per tile), runs 8 k
//     blocks x 2 x 2 sub-tiles x (1 + 5) v_mfma_f32_16x16x32_bf16 (leading
//     product and the small ones in two accumulators, as apply_split_kernel),
//     and reads its own raw values for the delta-form epilogue
//     Y = X + X (T - I) back from its raw image.
// MFMA shape (round 6): the kernel is power-limited -- the dense form runs at
// 1.77 GHz with its matrix pipe 61 % busy at that clock, without global
// memory at 2.10 GHz, memory alone at 2.45 GHz (profiles/r6_clock) -- and the
// 16x16x32 bf16 MFMA holds a higher clock than 32x32x16 for the same flops
// (MI355X_MICROARCH "DVFS give-back" (7)); same cycles, registers and LDS
// reads per flop.
// (The raw image is plain [col][row]: the split's and epilogue's dword reads
// meet 2-way bank conflicts, which cost less than the registers a swizzle's
// extra lane offsets took from the T slice.)
// Work: the active quads (some step-s or step-(s+1) pair rotated) are listed
// by every wave with ballots over the skip flags (no extra launch, no host
// sync); their tiles, flattened, are dealt to the persistent grid in equal
// contiguous ranges (one workgroup per CU: the LDS is 160 KB).
constexpr int kQuadTsThreads = 512;
constexpr int kQuadTsGrid = 256;
// While the other chain's latency-bound kernels (Gram, EVDs, Q builds, update)
// run concurrently on another stream (two-chain issue, every multi-GPU plan),
// a smaller grid leaves them CUs to start on at once instead of behind the
// persistent apply's 160 KB-LDS workgroups.  16384^2 rank plans, ms per sweep
// (profiles/r6_grid): P = 4 (8 quads per apply) 256 WGs 65.5-69.8, 224
// 64.6-65.3, 208 63.8-65.6, 192 63.4-64.1; P = 2 (16 quads) 256 118.0-125.5,
// 224 116.4-118.3, 192 118.4-120.7.  The merged one-GPU issue keeps the
// whole chip.
__host__ __device__ constexpr int quad_ts_grid_shared(int nq) { return nq <= 8 ? 192 : 224; }
template <int NP>
struct QuadTsLds {
  static constexpr int S_BYTES = 16 * NP * SVDJ_WAVE * 16;  // split image of a 32-row tile
  static constexpr int R_BYTES = 8 * 32 * 32 * 4;           // raw tile, wave w at 4 KB * w: [col][row]
  static constexpr int TOTAL = 2 * S_BYTES + 2 * R_BYTES;
};
static_assert(QuadTsLds<3>::TOTAL <= 163840, "T-stationary quad apply LDS");

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ABL (tools/micro/quad_apply_ab.hip only; production launches ABL = 0):
// bit 0 one MFMA per k block and sub-tile instead of 1 + (products of order
// < NP), B fragments still read; bit 1 no global memory (no DMA, no waits, no
// stores); bit 2 no MFMA loop at all (split, barrier, epilogue, DMA only);
// bit 3 never the cheap (first-order) k-block form.
template <int NP, int ABL = 0>
__global__ __launch_bounds__(kQuadTsThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void
apply_quad_ts_kernel(float* __restrict__ A, int lda, int a_tiles, float* __restrict__ V, int ldv,
                     int v_tiles, const int32_t* __restrict__ pairs, int nq,
                     const bf16x8* __restrict__ Ts, const int32_t* __restrict__ skip1,
                     const int32_t* __restrict__ skip2, uint32_t* __restrict__ work = nullptr,
                     float cheap_tol = 0.0078125f) {
  using L = QuadTsLds<NP>;
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i16 = lane & 15, g = lane >> 4;
  auto active = [&](int q) -> bool {  // all four flags loaded (no short-circuit branches)
    if (q >= nq) return false;
    return (skip1[2 * q] & skip1[2 * q + 1] & skip2[2 * q] & skip2[2 * q + 1]) == 0;
  };
  int nact = 0;
  for (int b0 = 0; b0 < nq; b0 += SVDJ_WAVE) nact += __popcll(__ballot(active(b0 + lane)));
  if (nact == 0) return;
  const int G = (int)gridDim.x, nt = a_tiles + v_tiles;
  // The active quads' tiles, flattened quad-major, are dealt to the grid in
  // equal contiguous ranges (a range may span two quads: one more T-slice
  // load).  Round 5 split each quad into G / nact equal slices, which left
  // G mod nact workgroups idle -- up to a quarter of the grid (52 active
  // quads: 208 of 256 busy) once quads start to skip.
  const long long total = (long long)nact * nt;
  const long long g_end = (long long)(blockIdx.x + 1) * total / G;
  for (long long pos = (long long)blockIdx.x * total / G; pos < g_end;) {
    const int qi = (int)(pos / nt);
    const int t0 = (int)(pos % nt);
    const int t1 = (int)((long long)t0 + (g_end - pos) < nt ? (long long)t0 + (g_end - pos) : nt);
    pos += t1 - t0;
    int q = 0;
    for (int b0 = 0, seen = 0; b0 < nq; b0 += SVDJ_WAVE) {  // the qi-th active quad
      const bool a = active(b0 + lane);
      const unsigned long long m = __ballot(a);
      const int cnt = __popcll(m);
      if (seen <= qi && qi < seen + cnt) {
        const int pre = __popcll(m & ((1ull << lane) - 1ull));
        q = b0 + __ffsll((long long)__ballot(a && pre == qi - seen)) - 1;
      }
      seen += cnt;
    }
    q = __builtin_amdgcn_readfirstlane(q);
    // this wave's split T - I slice: Ts[q][kb][ct = wave][cs][part][lane]
    bf16x8 qf[8][2][NP];
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
#pragma unroll
      for (int cs = 0; cs < 2; ++cs) {
        const bf16x8* tp = Ts + ts_frag(q, kb, wave, cs, NP) + lane;
#pragma unroll
        for (int p = 0; p < NP; ++p) qf[kb][cs][p] = tp[p * SVDJ_WAVE];
      }
    // Halves of the k range (k blocks 0-3 = blocks a, b of the quad, 4-7 =
    // c, d) whose slice of T - I is below cheap_tol = 2^-7 in magnitude: there
    // the order-2 products (q0 x2, q1 x1, q2 x0 <= 3 2^-18 |t||x| <= 3 2^-25
    // |x| per term, at the fp32 rounding of the output) are dropped, 3 MFMAs
    // per k block and sub-tile instead of 6.  Round 5 used 2^-9; 2^-7 and
    // 2^-6 measured 16384^2 -27 / -45 ms with residual 1.141 -> 1.151 / 1.173
    // e-5 and the same orthogonality (profiles/r6_issue); 2^-7 kept.  With T = T1 T2 (pairs (a,c), (b,d) then
    // (a,d), (b,c)), for an output column in a or b the rows of a and b are
    // second order in the rotation angles (T_aa - I, T_ba = T1_bd T2_da),
    // those of c and d first order; for c or d the other way round -- so once
    // the angles are below ~0.04 one half of every column tile takes the
    // cheap form.
    uint32_t cheap = 0;
    if constexpr (NP == 3 && (ABL & 8) == 0) {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        float mx = 0.0f;
#pragma unroll
        for (int kb = 4 * hf; kb < 4 * hf + 4; ++kb)
#pragma unroll
          for (int cs = 0; cs < 2; ++cs)
#pragma unroll
            for (int e = 0; e < 8; ++e) mx = fmaxf(mx, fabsf((float)qf[kb][cs][0][e]));
        if (wave_max(mx) <= cheap_tol) cheap |= 1u << hf;
      }
      cheap = __builtin_amdgcn_readfirstlane(cheap);
    }
    // this wave's 32 columns: block wave >> 1 of [a b c d], half wave & 1
    const int32_t* qp = pairs + 4 * q;
    const int qb = wave >> 1;
    const int col0 = __builtin_amdgcn_readfirstlane(qp[(qb & 1) * 2 + (qb >> 1)] * 64 + (wave & 1) * 32);
    float* const ownA = A + (size_t)col0 * lda;
    float* const ownV = V ? V + (size_t)col0 * ldv : nullptr;

    // raw tile t, own 32 columns -> R[buf] (4 x 1 KB): lane -> column
    // 8i + lane / 8, row chunk lane % 8 (one 32-bit lane offset from a
    // wave-uniform column base)
    auto dma = [&](int t, int buf) {
      if constexpr ((ABL & 2) != 0) return;
      const bool isA = t < a_tiles;
      const float* base = isA ? ownA : ownV;
      const int ld = isA ? lda : ldv, r0 = (isA ? t : t - a_tiles) * 32;
      char* dst = lds + 2 * L::S_BYTES + buf * L::R_BYTES + wave * 4096;
      const uint32_t o = (uint32_t)((lane >> 3) * ld + (lane & 7) * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds(&at_u32(base + (size_t)(8 * i) * ld + r0, o), dst + i * 1024,
                                         16, 0, 0);
    };
    // lane bases into the raw image [col][row]: split reads (column 8g + e,
    // row 16 rs + i) and epilogue reads (column 16 cs + 4g + e, row 16 rs + i)
    const int sb = 256 * g + i16, eb = 128 * g + i16;
    auto tile = [&](int t, auto bufc, auto chc) {
      constexpr int buf = decltype(bufc)::value;
      constexpr int CH = decltype(chc)::value;  // cheap halves (bit 0: k blocks 0-3, bit 1: 4-7)
      // 1. own DMA of tile t landed (younger: stores of t-1, DMA of t+1)
      const int younger = (t > t0 ? 16 : 0) + (t + 1 < t1 ? 4 : 0);
      if constexpr ((ABL & 2) != 0) (void)younger;
      else if (younger == 20) wait_vmcnt<20>();
      else if (younger == 16) wait_vmcnt<16>();
      else if (younger == 4) wait_vmcnt<4>();
      else wait_vmcnt<0>();
      const float* R = reinterpret_cast<const float*>(lds + 2 * L::S_BYTES + buf * L::R_BYTES + wave * 4096);
      // 2. split own columns (k block `wave`) into the shared B-fragment image
      //    S[buf]: [kb][rs][part][lane (i, g)] element e = X[16 rs + i][32 kb + 8g + e]
      {
        bf16x8* Sw = reinterpret_cast<bf16x8*>(lds + buf * L::S_BYTES) + lane;
#pragma unroll
        for (int rs = 0; rs < 2; ++rs) {
          bf16x8 parts[NP];
          float xv[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) xv[e] = R[sb + 32 * e + 16 * rs];
          split_bf16x8<NP>(xv, parts);
#pragma unroll
          for (int i = 0; i < NP; ++i) Sw[((2 * wave + rs) * NP + i) * SVDJ_WAVE] = parts[i];
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      // 3. per 16-row half rs of the tile: 8 k blocks x 2 column sub-tiles x
      //    (1 + 5) MFMAs (1 + 2 in a cheap half) against the register-resident
      //    slice, then that half's epilogue (one half's accumulators live at a
      //    time: 16 VGPRs, what lets the T slice stay in registers)
      const bf16x8* Sr = reinterpret_cast<const bf16x8*>(lds + buf * L::S_BYTES) + lane;
      const bool isA = t < a_tiles;
      float* const own = isA ? ownA : ownV;
      const int ld = isA ? lda : ldv, r0 = (isA ? t : t - a_tiles) * 32;
      const uint32_t st_off = (uint32_t)(4 * g * ld + i16) + (uint32_t)r0;
#pragma unroll
      for (int rs = 0; rs < 2; ++rs) {
        f32x4 acc[2], lo[2];
#pragma unroll
        for (int cs = 0; cs < 2; ++cs)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[cs][e] = lo[cs][e] = 0.0f;
        auto khalf = [&](auto k0c) {
          constexpr int k0 = decltype(k0c)::value;
#pragma unroll
          for (int kb = k0; kb < k0 + 4; ++kb) {
            bf16x8 xs[NP];
            if constexpr ((ABL & 1) != 0) {
              using i32x4 = __attribute__((ext_vector_type(4))) int;
              i32x4 x = __builtin_bit_cast(i32x4, Sr[((kb * 2 + rs) * NP) * SVDJ_WAVE]);
#pragma unroll
              for (int i = 1; i < NP; ++i)
                x ^= __builtin_bit_cast(i32x4, Sr[((kb * 2 + rs) * NP + i) * SVDJ_WAVE]);
#pragma unroll
              for (int cs = 0; cs < 2; ++cs) acc[cs] = mfma16(qf[kb][cs][0], __builtin_bit_cast(bf16x8, x), acc[cs]);
            } else if constexpr (NP == 3 && ((CH >> (k0 / 4)) & 1) != 0) {
              xs[0] = Sr[((kb * 2 + rs) * NP + 0) * SVDJ_WAVE];
              xs[1] = Sr[((kb * 2 + rs) * NP + 1) * SVDJ_WAVE];
#pragma unroll
              for (int cs = 0; cs < 2; ++cs) {
                lo[cs] = mfma16(qf[kb][cs][0], xs[1], lo[cs]);
                lo[cs] = mfma16(qf[kb][cs][1], xs[0], lo[cs]);
                acc[cs] = mfma16(qf[kb][cs][0], xs[0], acc[cs]);
              }
            } else {
#pragma unroll
              for (int i = 0; i < NP; ++i) xs[i] = Sr[((kb * 2 + rs) * NP + i) * SVDJ_WAVE];
#pragma unroll
              for (int cs = 0; cs < 2; ++cs) {
#pragma unroll
                for (int ord = NP - 1; ord >= 1; --ord)  // products of order ord, small first
#pragma unroll
                  for (int a = 0; a <= ord; ++a) lo[cs] = mfma16(qf[kb][cs][a], xs[ord - a], lo[cs]);
                acc[cs] = mfma16(qf[kb][cs][0], xs[0], acc[cs]);
              }
            }
            // no scheduling across k blocks: hoisted fragment loads of later
            // blocks pushed the T slice out of registers
            __builtin_amdgcn_sched_barrier(0);
          }
        };
        if constexpr ((ABL & 4) == 0) {
          khalf(std::integral_constant<int, 0>{});
          khalf(std::integral_constant<int, 4>{});
        }
        // 4. own raw values of this half, still in this wave's raw image R[buf]
        //    (its refill, tile t + 2, is issued below), and the delta-form
        //    store, in place (acc[cs] register e is own column 16 cs + 4g + e,
        //    row 16 rs + i).  (Staging the finished tile
        //    through R[buf] for 16-byte stores cut the compute-only time of the
        //    32x32x16 form 1229 -> 1037 us but not the solve's:
        //    profiles/r6_apply/ablation_vector_epilogue_rejected.jsonl.)
#pragma unroll
        for (int cs = 0; cs < 2; ++cs) {
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = R[eb + 512 * cs + 32 * e + 16 * rs];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float y = v[e] + (acc[cs][e] + lo[cs][e]);
            if ((ABL & 2) == 0 || y == -1.2345e-30f)
              at_u32(own + (size_t)(16 * cs + e) * ld + 16 * rs, st_off) = y;
          }
        }
      }
      // 5. tile t + 2 into the raw image this wave just consumed
      if (t + 2 < t1) dma(t + 2, buf);
    };
    if (t0 < t1) dma(t0, 0);
    if (t0 + 1 < t1) dma(t0 + 1, 1);
    // the tile loop specialised per cheap-half mask (a branch per k half
    // inside one loop made the compiler spill the T slice)
    auto run = [&](auto chc) {
      for (int t = t0; t < t1; t += 2) {
        tile(t, std::integral_constant<int, 0>{}, chc);
        if (t + 1 < t1) tile(t + 1, std::integral_constant<int, 1>{}, chc);
      }
    };
    if (cheap == 0) run(std::integral_constant<int, 0>{});
    else if constexpr (NP == 3) {
      if (cheap == 1) run(std::integral_constant<int, 1>{});
      else if (cheap == 2) run(std::integral_constant<int, 2>{});
      else run(std::integral_constant<int, 3>{});
    }
    // work counters of the sweep (metric words 6, 7; svdj_stop.h): MFMAs this
    // wave issued in 32x32x16 units of 24 (96, 72 or 48 per tile = twice as
    // many 16x16x32 ones), and tiles moved
    if (work && lane == 0) {
      const uint32_t per = NP == 3 ? 4u - (cheap & 1u) - ((cheap >> 1) & 1u) : 2u;
      atomicAdd(&work[0], (uint32_t)(t1 - t0) * per);
      if (wave == 0) atomicAdd(&work[1], (uint32_t)(t1 - t0));
    }
    // the next item re-stages both images
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}

// The quad step's Grams summed over their row chunks, spread over 4 x 3P
// workgroups: fp64 sums in chunk order rounded once -- bitwise what
// evd_cross_kernel and quad_update_kernel compute from the chunks -- so that
// with many chunks (few quads: 64 at 4 quads) the latency-bound consumers,
// one workgroup per pair, read one slab instead of all chunks (8-GPU plan:
// quad_update 334 us per launch reading 64 chunks, profiles/r5_quad2).
constexpr int kRedThreads = 256;
__global__ __launch_bounds__(kRedThreads) void slab_reduce_kernel(const float* __restrict__ in,
                                                                  int gch, float* __restrict__ out) {
  constexpr int W = 64, E4 = W * W / 4;
  const int slab = blockIdx.x, e4 = blockIdx.y * kRedThreads + threadIdx.x;
  const float4* p = reinterpret_cast<const float4*>(in) + (size_t)slab * gch * E4 + e4;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll 8
  for (int k = 0; k < gch; ++k) {
    const float4 v = p[(size_t)k * E4];
    s0 += (double)v.x;
    s1 += (double)v.y;
    s2 += (double)v.z;
    s3 += (double)v.w;
  }
  reinterpret_cast<float4*>(out)[(size_t)slab * E4 + e4] =
      make_float4((float)s0, (float)s1, (float)s2, (float)s3);
}

// The six cross Grams of a quad step, every block read ONCE (round 5).  The
// round-4 form computed them as 3P independent f32-MFMA slabs, each reading
// its two blocks: every block of a quad was read three times and the f32
// MFMAs (1/16 of the bf16 rate) set the pace (722 us per 128-pair quad step
// vs 2 x 215 us for the two single-step Grams it replaces).  Here
// one workgroup (8 waves) per (quad, row chunk):
//   * wave w LDS-DMAs column tile w (32 of the quad's 256 columns, [a b c d]
//     order) of each 32-row slab two slabs ahead into a wave-private raw
//     image, and splits it into 3 RNE bf16 parts -- lane (i, g) of 16-column
//     sub-tile s: column 16 s + i, rows 8g .. 8g+7, exactly the A and the B
//     operand of v_mfma_f32_16x16x32_bf16 -- kept in registers and written to
//     the shared fragment image for the other waves;
//   * OWNER-based tiles (round 6): the 24 needed 32 x 32 output tiles are the
//     pairs of column tiles from different blocks; each is computed by one
//     of its two column tiles' waves (kGramPartner: every wave 3 partners), so
//     a wave's own operand never leaves its registers and it reads only its 3
//     partners' fragments (18 x 1 KB per slab and wave instead of 36: the
//     round-5 form, any 3 tiles per wave with both operands from LDS, was
//     LDS-bandwidth bound -- 142 us of 278 with one MFMA per product,
//     profiles/r6_apply/ablation_gram.jsonl);
//   * each 16 x 16 sub-tile takes the 6 products of order < 3 (leading product
//     and the small ones in two accumulators), the error of a product below
//     2^-26 relative, like the split apply;
//   * the tiles go straight to the slab layout the consumers read: slab
//     (pair 2q) = C_ac, (2q+1) = C_bd, then per quad C_ad, C_bc, C_ab, C_cd
//     (the order quad_update_kernel reads), one W x W slab per row chunk; a
//     tile whose owner is its slab's column block is stored transposed.
constexpr int kGramQThreads = 512;
template <int NP>
struct GramQLds {
  static constexpr int S_BYTES = 8 * 2 * NP * SVDJ_WAVE * 16;  // 8 col tiles x 2 sub-tiles x NP parts
  static constexpr int R_BYTES = 8 * 32 * 32 * 4;              // raw 32-row slab, wave w at 4 KB * w
  static constexpr int TOTAL = 2 * S_BYTES + 2 * R_BYTES;
};
static_assert(GramQLds<3>::TOTAL <= 163840, "quad Gram LDS");
// Partners of column tile w (tile t is block t >> 1 of [a b c d], half t & 1):
// the 24 pairs of tiles from different blocks, each listed once, 3 per tile
// (3 bits each, partner j at bits 3j).
constexpr int kGramPartners[8] = {2 | 3 << 3 | 4 << 6, 2 | 3 << 3 | 5 << 6, 4 | 5 << 3 | 6 << 6,
                                  4 | 5 << 3 | 7 << 6, 1 | 6 << 3 | 7 << 6, 0 | 6 << 3 | 7 << 6,
                                  0 | 1 << 3 | 3 << 6, 0 | 1 << 3 | 2 << 6};
// every unordered pair of tiles from different blocks exactly once, none within a block
constexpr bool gram_partners_cover() {
  int seen[8][8] = {};
  for (int w = 0; w < 8; ++w)
    for (int j = 0; j < 3; ++j) {
      const int y = kGramPartners[w] >> (3 * j) & 7;
      if ((y >> 1) == (w >> 1)) return false;
      ++seen[w < y ? w : y][w < y ? y : w];
    }
  for (int x = 0; x < 8; ++x)
    for (int y = x + 1; y < 8; ++y)
      if (seen[x][y] != ((x >> 1) != (y >> 1) ? 1 : 0)) return false;
  return true;
}
static_assert(gram_partners_cover(), "quad Gram partner table");
__device__ __forceinline__ int gram_partners(int w) {
  int r = kGramPartners[0];
#pragma unroll
  for (int t = 1; t < 8; ++t) r = w == t ? kGramPartners[t] : r;
  return r;
}
// Product (slab) of blocks (x, y) of [a b c d]: ac bd ad bc ab cd = 0 .. 5;
// bit 3 set when (x, y) is the transposed order.
__host__ __device__ constexpr int gram_product_fwd(int x, int y) {
  return x == 0 && y == 2 ? 0 : x == 1 && y == 3 ? 1 : x == 0 && y == 3 ? 2 : x == 1 && y == 2 ? 3
       : x == 0 && y == 1 ? 4 : x == 2 && y == 3 ? 5 : -1;
}
__host__ __device__ constexpr int gram_product(int x, int y) {
  return gram_product_fwd(x, y) >= 0 ? gram_product_fwd(x, y) : 8 | gram_product_fwd(y, x);
}
static_assert(gram_product(2, 0) == 8 && gram_product(3, 2) == 13, "gram_product");
// ABL (tools/micro/quad_apply_ab.hip only; production launches ABL = 0):
// bit 0 one MFMA per output sub-tile and slab instead of 6; bit 1 no global
// reads (no DMA, no waits).
// NP = 2 (sweeps far from convergence, see launch_quad_gram_evd): 2 bf16
// parts and the 3 products of order < 2 -- couplings to ~2^-17 |x||y|,
// which only steers the rotation angles (T stays orthogonal to fp64).
template <int ABL = 0, int NP = 3>
__global__ __launch_bounds__(kGramQThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void
gram_quad_kernel(const float* __restrict__ A, int lda, int m_pad, const int32_t* __restrict__ pairs,
                 int P, int rows_per_chunk, float* __restrict__ slabs) {
  constexpr int W = 64;
  using L = GramQLds<NP>;
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  const int q = blockIdx.x, chunk = blockIdx.y, nchunk = gridDim.y;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i16 = lane & 15, g = lane >> 4;
  const int32_t* qp = pairs + 4 * q;  // (a, c), (b, d)
  auto blk = [&](int qb) { return qp[(qb & 1) * 2 + (qb >> 1)]; };  // [a b c d] -> block id
  const int r_begin = chunk * rows_per_chunk;
  const int r_end = min(m_pad, r_begin + rows_per_chunk);
  const int ns = (r_end - r_begin) / 32;  // rows_per_chunk and m_pad are multiples of 128
  const float* own = A + (size_t)__builtin_amdgcn_readfirstlane(blk(wave >> 1) * W + (wave & 1) * 32) * lda;
  const int pk = __builtin_amdgcn_readfirstlane(gram_partners(wave));
  // raw image [col][16-byte row chunk], chunk slot j of column col holding
  // rows 4 (j ^ (col & 7)) .. + 3: the split's reads (8 rows of one column per
  // lane, lanes at a 128-byte column stride) then spread over the banks
  // instead of piling onto a few (35 % bank-conflict cycles unswizzled)
  auto dma = [&](int sl, int buf) {
    if constexpr ((ABL & 2) != 0) return;
    const int r0 = r_begin + 32 * sl;
    char* dst = lds + 2 * L::S_BYTES + buf * L::R_BYTES + wave * 4096;
    const int jr = ((lane & 7) ^ (lane >> 3)) * 4;  // col & 7 == lane >> 3 for every i
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds(own + (size_t)(8 * i + (lane >> 3)) * lda + r0 + jr,
                                       dst + i * 1024, 16, 0, 0);
  };
  // [partner j][own sub-tile s][partner sub-tile s2]
  f32x4 acc[3][2][2], lo[3][2][2];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[j][s][s2][e] = lo[j][s][s2][e] = 0.0f;
  auto slab = [&](int sl, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    if constexpr ((ABL & 2) != 0) {
    } else if (sl + 1 < ns) wait_vmcnt<4>();
    else wait_vmcnt<0>();
    bf16x8 xf[2][NP];
    {  // split own column tile: sub-tile s, column 16 s + i, rows 8g .. 8g+7
      const float* R = reinterpret_cast<const float*>(lds + 2 * L::S_BYTES + buf * L::R_BYTES + wave * 4096);
      bf16x8* Sw = reinterpret_cast<bf16x8*>(lds + buf * L::S_BYTES) + lane;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int c = 16 * s + i16;
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(R + c * 32 + 4 * ((2 * g) ^ (c & 7)));
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(R + c * 32 + 4 * ((2 * g + 1) ^ (c & 7)));
        const float xv[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        split_bf16x8<NP>(xv, xf[s]);
#pragma unroll
        for (int i = 0; i < NP; ++i) Sw[((wave * 2 + s) * NP + i) * SVDJ_WAVE] = xf[s][i];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const bf16x8* Sr = reinterpret_cast<const bf16x8*>(lds + buf * L::S_BYTES) + lane;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int yt = (pk >> (3 * j)) & 7;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 yf[NP];
#pragma unroll
        for (int i = 0; i < NP; ++i) yf[i] = Sr[((yt * 2 + s2) * NP + i) * SVDJ_WAVE];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if constexpr ((ABL & 1) != 0) {
            using i32x4 = __attribute__((ext_vector_type(4))) int;
            i32x4 yy = __builtin_bit_cast(i32x4, yf[0]);
#pragma unroll
            for (int i = 1; i < NP; ++i) yy ^= __builtin_bit_cast(i32x4, yf[i]);
            acc[j][s][s2] = mfma16(xf[s][0], __builtin_bit_cast(bf16x8, yy), acc[j][s][s2]);
          } else {
#pragma unroll
            for (int ord = NP - 1; ord >= 1; --ord)  // products of order ord, small first
#pragma unroll
              for (int a = 0; a <= ord; ++a) lo[j][s][s2] = mfma16(xf[s][a], yf[ord - a], lo[j][s][s2]);
            acc[j][s][s2] = mfma16(xf[s][0], yf[0], acc[j][s][s2]);
          }
        }
      }
    }
    if (sl + 2 < ns) dma(sl + 2, buf);
  };
  if (ns > 0) dma(0, 0);
  if (ns > 1) dma(1, 1);
  for (int sl = 0; sl < ns; sl += 2) {
    slab(sl, std::integral_constant<int, 0>{});
    if (sl + 1 < ns) slab(sl + 1, std::integral_constant<int, 1>{});
  }
  // register e of lane (i, g) of sub-tile (s, s2) = C[own column 16 s + 4g + e]
  // [partner column 16 s2 + i]; straight to the slabs
  const int bx = wave >> 1;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int yt = (pk >> (3 * j)) & 7, by = yt >> 1;
    const int code = gram_product(bx, by), pr = code & 7;
    const size_t sidx = pr < 2 ? (size_t)(2 * q + pr) * nchunk + chunk
                               : (size_t)P * nchunk + ((size_t)q * 4 + (pr - 2)) * nchunk + chunk;
    float* out = slabs + sidx * (W * W);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const f32x4 v = acc[j][s][s2] + lo[j][s][s2];
        const int xr = 32 * (wave & 1) + 16 * s + 4 * g, yc = 32 * (yt & 1) + 16 * s2 + i16;
        if (code & 8) {  // slab rows are the partner's block
          *reinterpret_cast<f32x4*>(out + yc * W + xr) = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) out[(xr + e) * W + yc] = v[e];
        }
      }
  }
}

// ------------------------------------------------------------- host side
struct Geometry {
  int gchunks, grows;  // gram
  int a_chunks, rows_a, v_chunks, rows_v;
  // quad steps (fp32 W = 64): gram row chunks, apply row chunks
  int qgch, qgrows;
};

// Quad-step geometry: row chunks of gram_quad_kernel (its slabs are summed
// by evd_cross_kernel / quad_update_kernel); the apply is a persistent grid.
static void quad_geometry(Geometry& g, int P, int m_pad, int n_v) {
  // gram_quad_kernel: one workgroup (160 KB LDS, one per CU) per quad and row
  // chunk, ~256 of them; from 32 quads per launch every quad keeps 4 chunks,
  // so a merged one-GPU launch (two chains' quads in one) sums every Gram
  // exactly as the two chains do (bitwise the same solve, as make_geometry).
  // 64 quads (16384^2 merged), us per quad step: 2 chunks 963-979, 4 chunks
  // 874-884, 8 chunks 933 (profiles/r5_gram)
  const int nq = P / 2 > 0 ? P / 2 : 1;
  int want = nq >= 32 ? 4 : (256 + nq - 1) / nq;
  static const int forced = svdj_debug_knob("quad_gram_chunks", 0);  // A/B only (svdj_debug.h)
  if (forced > 0) want = forced;
  const int maxc = m_pad / 128;
  g.qgch = want < 1 ? 1 : (want > maxc ? maxc : want);
  g.qgrows = round_up((m_pad + g.qgch - 1) / g.qgch, 128);
  g.qgch = (m_pad + g.qgrows - 1) / g.qgrows;
}

static Geometry make_geometry(int W, int P, int m_pad, int n_v, int mma = 0) {
  Geometry g;
  // Gram: split-K over row chunks (>= 128 rows each), ~512 workgroups.
  // Many pairs per step want few chunks (every chunk is a slab the EVD sums:
  // 1-GPU 16384^2, W=64, 5.92 s at 512 vs 6.23 s at 2048).  With few pairs
  // (many GPUs) 64-256 measured slower (8-GPU rank plan 65.5 -> 74-78 ms).
  // With the split-bf16 apply, steps of >= 32 pairs want ~256 (1 GPU 16384^2
  // 4.94 -> 4.84 s, 8192^2 674 -> 659 ms, P=2 plan 165.8 -> 163.5 ms per sweep);
  // the P=4 plan (16 pairs) is 6 % slower at 256 (profiles/r3_s3/gram).
  // Steps of >= 64 pairs keep the 64-pair chunking (4 row chunks): a merged
  // one-GPU step (two chains' 64-pair steps in one launch, pipeline.py
  // run_merged) then sums every pair's Gram exactly as the two chains do, so
  // the solve is bitwise the two-chain one (same sweeps).  Measured at 128
  // pairs (16384^2 merged, quad off): 4 chunks 4.70 s vs 2 chunks (the
  // target rule) 4.73 s, residual 1.37e-5 vs 1.52e-5 (profiles/r5_gram).
  // Round 5 (profiles/r5_ab): below 32 pairs, at most ~512 workgroups AND
  // chunks of at least 512 rows -- rank plans, ms per sweep: 16384^2 P = 8
  // (8 pairs) 53.5 at 256 rows (512 workgroups, the old rule), 52.9 at 384,
  // 43.5 at 512, 55.2 at 1024; P = 4 (16 pairs) 100.9 / 82.8 / 83.9 / 86.7 at
  // 256 / 384 / 512 / 1024 rows; 32768 x 32768 P = 8 (16 pairs) 307 at 1024
  // rows (512 workgroups) vs 325 at 512 (1024 workgroups).  The EVD sums one
  // slab per chunk, so short chunks put more slab data on its critical path.
  int want = P >= 32 ? (256 + P - 1) / P : min((m_pad + 511) / 512, (512 + P - 1) / P);
  // (the bump applies to the split-bf16 launches it was measured on: merged
  // fp32 one-GPU steps of 128 pairs; fp64 steps keep the target rule)
  if (mma != 0 && P >= 64 && want < 4) want = 4;
  static const int forced = svdj_debug_knob("gram_chunks", 0);  // A/B only (svdj_debug.h)
  if (forced > 0) want = forced;
  int maxc = m_pad / 128;
  g.gchunks = want < 1 ? 1 : (want > maxc ? maxc : want);
  g.grows = round_up((m_pad + g.gchunks - 1) / g.gchunks, 128);
  g.gchunks = (m_pad + g.grows - 1) / g.grows;
  // Apply: workgroups over A and V rows (128..2048 rows each, every one
  // fills the pair's 2W x 2W Q into LDS first).  ~2048 workgroups for W = 32
  // and for steps with >= 64 pairs (one GPU: 16384^2 5.79 s vs 5.87 s at
  // 512); ~512 for W = 64 with fewer pairs, where the 64 KB Q fill of short
  // workgroups costs more than the occupancy gains: 16384^2 rank plans
  // P=2/4/8 206.5/126.2/63.0 -> 203.5/114.5/59.8 ms per sweep, 8192^2 one GPU
  // 866 -> 799 ms, 32768x8192 (QR) 943 -> 888 ms; W = 32 (4096^2, fp64
  // 5000^2) 2-3.5 % slower at 512 (profiles/r2_awg).  The split-bf16 applies
  // (mma != 0) keep 2048: their larger Q images (32768x8192 bf16 with QR:
  // 811 -> 847 ms at 512).
  int total_rows = m_pad + n_v;
  // The split-bf16 apply (mma != 0, Q held in registers per output column
  // tile) wants 2048 unless a step has few pairs: 1 GPU 8192^2 664 ms at
  // 2048 vs 756 at 512, 16384^2 P=8 rank plan 52.3 vs 50.3 ms per sweep at
  // 2048 vs 512 (profiles/r3_s3/bf16x6).
  const int wg_target = mma == 0 ? (W == 64 && P < 64 ? 512 : 2048) : (P <= 16 ? 512 : 2048);
  int rows = round_up((int)(((long)total_rows * P + wg_target - 1) / wg_target), 128);
  if (rows < 128) rows = 128;
  if (rows > 2048) rows = 2048;
  g.rows_a = rows;
  g.rows_v = rows;
  g.a_chunks = (m_pad + rows - 1) / rows;
  g.v_chunks = n_v > 0 ? (n_v + rows - 1) / rows : 0;
  quad_geometry(g, P, m_pad, n_v);
  return g;
}

static size_t rup256(size_t b) { return (b + 255) / 256 * 256; }
// Quad-step scratch (fp32 W = 64, only when the step list has quad steps):
// the 3P Gram slabs, T1 (fp64 Q of the P step-s pairs), the step-(s+1)
// couplings, the double-buffered split T - I (P/2 quads x 256 x 256 in 3
// bf16 parts = 1.5 x an fp32 T each) and the skip flags of both EVDs
// (chain_init's layout).
static bool has_quad(int esize, int W) { return esize == 4 && W == 64; }
static size_t quad_bytes(int P, int m_pad) {
  Geometry g;
  quad_geometry(g, P, m_pad, 0);
  constexpr int W = 64;
  const size_t kstride = rup256((size_t)P * sizeof(int32_t));
  const size_t tstride = rup256((size_t)(P / 2 > 0 ? P / 2 : 1) * 16 * W * W * sizeof(float));
  return rup256((size_t)3 * P * g.qgch * W * W * sizeof(float)) +
         rup256((size_t)3 * P * W * W * sizeof(float)) +
         rup256((size_t)P * 4 * W * W * sizeof(double)) + rup256((size_t)P * W * W * sizeof(float)) +
         3 * tstride + 4 * kstride;
}
static bool has_quad_steps(const int32_t* modes, int steps) {
  for (int s = 0; modes && s < steps; ++s)
    if (modes[s] == 4) return true;
  return false;
}
static size_t ws_bytes_for(int esize, int W, int P, int m_pad, bool quad) {
  // the Gram chunking depends on the apply mode (split-bf16 launches may take
  // more chunks): size the slabs for the larger of the two
  Geometry g = make_geometry(W, P, m_pad, 0, 0);
  const Geometry gs = make_geometry(W, P, m_pad, 0, 1);
  if (gs.gchunks > g.gchunks) g = gs;
  size_t slabs = (size_t)P * g.gchunks * 4 * W * W * esize;
  size_t q = (size_t)P * 4 * W * W * esize;
  size_t sk = (size_t)P * sizeof(int32_t);
  size_t rec = (size_t)P * kCrossMaxInner * W * W * esize;
  // slabs + double-buffered Q and skip flags (evd(s+1) may run while apply(s)
  // reads) + the cross EVD's rotation records and step counts (consumed by
  // qbuild(s) before evd(s+1) on the same stream: single-buffered)
  return rup256(slabs) + 2 * rup256(q) + 2 * rup256(sk) + rup256(rec) + rup256(sk) +
         (quad && has_quad(esize, W) ? quad_bytes(P, m_pad) : 0);
}

// One chain of steps: resident buffers, its pair list and its workspace.
template <typename T>
struct Chain {
  int m_pad, lda, n_v, ldv, P, steps;
  T *A, *V, *D;
  const int32_t* pairs;
  const int32_t* modes;
  Geometry g;
  T* slabs;
  T* Qb[2];
  int32_t* skipb[2];
  T* rec;  // cross EVD rotation records (tangents)
  int32_t* nsteps;
  // quad steps (has_quad)
  float* qslabs;
  float* qred;  // the 3P Grams summed over their row chunks (when qgch > 4)
  double* T1;
  float* upd;
  bf16x8* Ts[2];
  int32_t* skip1[2];
  int32_t* skip2[2];
  hipStream_t st;
  int gram_np;  // bf16 parts of the quad Gram (3; 2 far from convergence)
  int shared;  // another chain runs concurrently on this GPU (svdj_block_steps mma bit 9)
};

template <typename T, int W>
static int chain_init(Chain<T>& c, int m_pad, T* A, int lda, T* V, int n_v, int ldv, T* D,
                      const int32_t* pairs, int P, int steps, const int32_t* modes, void* ws,
                      size_t ws_bytes, int mma, hipStream_t st) {
  const bool quad = has_quad_steps(modes, steps);
  if (quad && !has_quad(sizeof(T), W)) {
    set_error("quad steps need fp32 data and W = 64");
    return -3;
  }
  const size_t need = ws_bytes_for(sizeof(T), W, P, m_pad, quad);
  if (ws_bytes < need) {
    set_error("workspace too small: %zu < %zu", ws_bytes, need);
    return -4;
  }
  if (mma != 0 && sizeof(T) != 4) {
    set_error("split-bf16 matrix-core modes need fp32 data");
    return -3;
  }
  if (sizeof(T) == 4 && W == 64 && lda % 4) {  // gram_cross_f32_kernel's 16-byte loads
    set_error("fp32 W = 64 needs lda %% 4 == 0, got %d", lda);
    return -2;
  }
  c.m_pad = m_pad; c.lda = lda; c.n_v = n_v; c.ldv = ldv; c.P = P; c.steps = steps;
  c.gram_np = 3;
  c.shared = 0;
  c.A = A; c.V = V; c.D = D; c.pairs = pairs; c.modes = modes; c.st = st;
  c.g = make_geometry(W, P, m_pad, V ? n_v : 0, mma);
  char* w = (char*)ws;
  c.slabs = (T*)w;
  w += ((size_t)P * c.g.gchunks * 4 * W * W * sizeof(T) + 255) / 256 * 256;
  const size_t qstride = ((size_t)P * 4 * W * W * sizeof(T) + 255) / 256 * 256;
  c.Qb[0] = (T*)w;
  c.Qb[1] = (T*)(w + qstride);
  w += 2 * qstride;
  const size_t kstride = ((size_t)P * sizeof(int32_t) + 255) / 256 * 256;
  c.skipb[0] = (int32_t*)w;
  c.skipb[1] = (int32_t*)(w + kstride);
  w += 2 * kstride;
  c.rec = (T*)w;
  w += rup256((size_t)P * kCrossMaxInner * W * W * sizeof(T));
  c.nsteps = (int32_t*)w;
  w += kstride;
  c.qslabs = nullptr;
  c.qred = nullptr;
  c.T1 = nullptr;
  c.upd = nullptr;
  c.Ts[0] = c.Ts[1] = nullptr;
  c.skip1[0] = c.skip1[1] = c.skip2[0] = c.skip2[1] = nullptr;
  if (quad) {
    c.qslabs = (float*)w;
    w += rup256((size_t)3 * P * c.g.qgch * W * W * sizeof(float));
    c.qred = (float*)w;
    w += rup256((size_t)3 * P * W * W * sizeof(float));
    c.T1 = (double*)w;
    w += rup256((size_t)P * 4 * W * W * sizeof(double));
    c.upd = (float*)w;
    w += rup256((size_t)P * W * W * sizeof(float));
    const size_t tstride = rup256((size_t)(P / 2 > 0 ? P / 2 : 1) * 16 * W * W * sizeof(float));
    c.Ts[0] = (bf16x8*)w;  // 3 bf16 parts = 1.5 x the fp32 size of T
    c.Ts[1] = (bf16x8*)(w + 3 * tstride / 2);
    w += 3 * tstride;
    c.skip1[0] = (int32_t*)w;
    c.skip1[1] = (int32_t*)(w + kstride);
    c.skip2[0] = (int32_t*)(w + 2 * kstride);
    c.skip2[1] = (int32_t*)(w + 3 * kstride);
  }
  return 0;
}

// Quad step s (steps s, s+1 fused; see "quad step"): gram, evd 1, T1,
// update, evd 2, T on the chain's stream.
template <typename T, int W>
static int launch_quad_gram_evd(const Chain<T>& c, int s, double tol, int absmode, int max_inner,
                                uint32_t* metric, int mma) {
  if constexpr (sizeof(T) == 4 && W == 64) {
    if (c.P % 2 || s + 1 >= c.steps || c.modes[s + 1] != 5) {
      set_error("quad step %d: needs an even pair count (%d) and a following mode-5 step", s, c.P);
      return -2;
    }
    const int b = s & 1;
    const int32_t* pr = c.pairs + (size_t)s * c.P * 2;
    const int32_t* pr1 = pr + 2 * c.P;
    if (c.gram_np == 2)
      hipLaunchKernelGGL((gram_quad_kernel<0, 2>), dim3(c.P / 2, c.g.qgch), dim3(kGramQThreads), 0,
                         c.st, c.A, c.lda, c.m_pad, pr, c.P, c.g.qgrows, c.qslabs);
    else
      hipLaunchKernelGGL((gram_quad_kernel<0, 3>), dim3(c.P / 2, c.g.qgch), dim3(kGramQThreads), 0,
                         c.st, c.A, c.lda, c.m_pad, pr, c.P, c.g.qgrows, c.qslabs);
    SVDJ_LAUNCH_CHECK();
    // many row chunks (few quads): sum them once, wide, for both consumers
    const bool red = c.g.qgch > 4;
    const float* gs = red ? c.qred : c.qslabs;
    const int gn = red ? 1 : c.g.qgch;
    if (red) {
      hipLaunchKernelGGL(slab_reduce_kernel, dim3(3 * c.P, 64 * 64 / 4 / kRedThreads),
                         dim3(kRedThreads), 0, c.st, c.qslabs, c.g.qgch, c.qred);
      SVDJ_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL((evd_cross_kernel<float, 64>), dim3(c.P), dim3(cross_threads<64>()), 0, c.st,
                       pr, gs, gn, c.D, c.rec, c.nsteps, c.skip1[b], (float)tol,
                       absmode, max_inner, metric);
    SVDJ_LAUNCH_CHECK();
    constexpr int R = 8;
    // 1024 threads: one workgroup per pair (phase 1) / two (phase 2), so each
    // pair's rotation records are staged 1-2 times instead of 4-8 (128-pair
    // quad step 832 -> 824 us, profiles/r5_ab)
    constexpr int QBT = 1024, QBW = QBT / SVDJ_WAVE;
    // below 64 pairs the Q builds are on the latency path: 2 rows per lane
    // (16384^2 rank plans, ms per sweep: P = 4 76.9 -> 72.5, P = 2 131.9 ->
    // 130.0, profiles/r5_quad2/reduce)
    const bool lat = c.P < 64;
    static const int qb1 = svdj_debug_knob("qb1_threads", 512);  // A/B only (svdj_debug.h)
    if (lat)
      hipLaunchKernelGGL((qbuild_quad_kernel<1, 2, QBT>), dim3(c.P, 128 / (2 * QBW)), dim3(QBT), 0,
                         c.st, c.rec, c.nsteps, c.skip1[b], c.T1);
    else if (qb1 == 512)  // two workgroups per pair: all CUs busy at 128 pairs
      hipLaunchKernelGGL((qbuild_quad_kernel<1, R, 512>), dim3(c.P, 128 / (R * 8)), dim3(512), 0,
                         c.st, c.rec, c.nsteps, c.skip1[b], c.T1);
    else
      hipLaunchKernelGGL((qbuild_quad_kernel<1, R, QBT>), dim3(c.P, 128 / (R * QBW)), dim3(QBT), 0,
                         c.st, c.rec, c.nsteps, c.skip1[b], c.T1);
    SVDJ_LAUNCH_CHECK();
    // 512 threads: 16384^2 -27 ms, 4096^2 -1 ms against 256 (profiles/r6_chain)
    static const int updt = svdj_debug_knob("upd_threads", 512);  // A/B only (svdj_debug.h)
    if (updt == 512)
      hipLaunchKernelGGL(quad_update_kernel<512>, dim3(c.P, 2), dim3(512), 0, c.st,
                         gs + (size_t)c.P * gn * 64 * 64, gn, c.T1, c.upd);
    else
      hipLaunchKernelGGL(quad_update_kernel<256>, dim3(c.P, 2), dim3(256), 0, c.st,
                         gs + (size_t)c.P * gn * 64 * 64, gn, c.T1, c.upd);
    SVDJ_LAUNCH_CHECK();
    hipLaunchKernelGGL((evd_cross_kernel<float, 64>), dim3(c.P), dim3(cross_threads<64>()), 0, c.st,
                       pr1, c.upd, 1, c.D, c.rec, c.nsteps, c.skip2[b], (float)tol, absmode,
                       max_inner, metric);
    SVDJ_LAUNCH_CHECK();
    // the split T is written directly (no tsplit pass)
    if (lat && mma == 2)
      hipLaunchKernelGGL((qbuild_quad_kernel<2, 2, QBT, 2>), dim3(c.P, 256 / (2 * QBW)), dim3(QBT), 0,
                         c.st, c.rec, c.nsteps, c.skip2[b], c.T1, c.Ts[b]);
    else if (lat)
      hipLaunchKernelGGL((qbuild_quad_kernel<2, 2, QBT, 3>), dim3(c.P, 256 / (2 * QBW)), dim3(QBT), 0,
                         c.st, c.rec, c.nsteps, c.skip2[b], c.T1, c.Ts[b]);
    else if (mma == 2)
      hipLaunchKernelGGL((qbuild_quad_kernel<2, R, QBT, 2>), dim3(c.P, 256 / (R * QBW)), dim3(QBT),
                         0, c.st, c.rec, c.nsteps, c.skip2[b], c.T1, c.Ts[b]);
    else
      hipLaunchKernelGGL((qbuild_quad_kernel<2, R, QBT, 3>), dim3(c.P, 256 / (R * QBW)), dim3(QBT),
                         0, c.st, c.rec, c.nsteps, c.skip2[b], c.T1, c.Ts[b]);
    SVDJ_LAUNCH_CHECK();
    return 0;
  } else {
    (void)c; (void)s; (void)tol; (void)absmode; (void)max_inner; (void)metric; (void)mma;
    set_error("quad steps need fp32 data and W = 64");
    return -3;
  }
}

// Gram + EVD of step s (Q and the skip flags are double-buffered so evd(s+1)
// never overwrites what apply(s) may still read).
// Dispatch order of the row chunks (SVDJ_DEBUG stream_order, bit 0: cross
// Gram chunks last-first, bit 1: the apply's V chunks before A's).
// Default 2: V first, so A -- which the next step's Gram reads -- holds the
// most recently written lines (single-stream 16384^2 step 642 -> 614 us,
// bitwise the same result; neutral with two concurrent chains).
static int stream_order() {
  static const int v = svdj_debug_knob("stream_order", 2);
  return v;
}

template <typename T, int W>
static int launch_gram_evd(const Chain<T>& c, int s, double tol, int absmode, int max_inner,
                           uint32_t* metric, int mma) {
  const int b = s & 1;
  const int32_t* pr = c.pairs + (size_t)s * c.P * 2;
  // 0 cross (cyclic EVD), 1 full Gram, 2 cross + bipartite EVD, 3 cross +
  // cross-only bipartite EVD (evd_cross_kernel)
  const int mode = c.modes ? c.modes[s] : 0;
  if (mode == 5) return 0;  // second step of a quad: done by its first (mode 4)
  if (mode == 4) return launch_quad_gram_evd<T, W>(c, s, tol, absmode, max_inner, metric, mma);
  const int full = mode == 1;
  constexpr int XS = gram_xsplit<T, W>();
  if (full) {
    if constexpr (XS > 1)  // see GRAM_SPLIT
      hipLaunchKernelGGL((gram_kernel<T, W, GRAM_SPLIT>), dim3(c.P, c.g.gchunks, 3 * XS),
                         dim3(kGramThreads), 0, c.st, c.A, c.lda, c.m_pad, pr, c.g.grows, c.slabs);
    else
      hipLaunchKernelGGL((gram_kernel<T, W, GRAM_FULL>), dim3(c.P, c.g.gchunks),
                         dim3(kGramThreads), 0, c.st, c.A, c.lda, c.m_pad, pr, c.g.grows, c.slabs);
  } else if constexpr (sizeof(T) == 4 && W == 64) {  // coalesced loads, LDS transpose
    hipLaunchKernelGGL((gram_cross_f32_kernel<GRAM_CROSS>), dim3(c.P, c.g.gchunks),
                       dim3(kGramThreads), 0, c.st, c.A, c.lda, c.m_pad, pr, c.g.grows, c.slabs,
                       stream_order() & 1);
  } else {
    hipLaunchKernelGGL((gram_kernel<T, W, GRAM_CROSS>), dim3(c.P, c.g.gchunks, XS),
                       dim3(kGramThreads), 0, c.st, c.A, c.lda, c.m_pad, pr, c.g.grows, c.slabs);
  }
  SVDJ_LAUNCH_CHECK();
  if (mode == 3) {
    // many row chunks (few pairs per step: the 8-GPU plans read 32): sum them
    // once, wide, instead of on the EVD's critical path (one workgroup per
    // pair reading every chunk); bitwise the same sums (slab_reduce_kernel)
    const T* gs = c.slabs;
    int gn = c.g.gchunks;
    if constexpr (sizeof(T) == 4 && W == 64) {
      static const int red_from = svdj_debug_knob("cross_reduce_chunks", 9);  // A/B only
      if (gn >= red_from) {
        float* red = c.slabs + (size_t)c.P * gn * W * W;  // inside the full-Gram slab area
        hipLaunchKernelGGL(slab_reduce_kernel, dim3(c.P, W * W / 4 / kRedThreads), dim3(kRedThreads),
                           0, c.st, c.slabs, gn, red);
        SVDJ_LAUNCH_CHECK();
        gs = red;
        gn = 1;
      }
    }
    hipLaunchKernelGGL((evd_cross_kernel<T, W>), dim3(c.P), dim3(cross_threads<W>()), 0, c.st, pr,
                       gs, gn, c.D, c.rec, c.nsteps, c.skipb[b], (T)tol, absmode, max_inner, metric);
    SVDJ_LAUNCH_CHECK();
    constexpr int RL = W == 64 ? 16 : 8;  // one workgroup per pair
    // 16 rows per lane from 64 pairs per step; at 32 pairs 4 rows per lane is
    // faster (1 GPU 8192^2 709 -> 672 ms, 16384^2 P=2 plan 171.4 -> 169.1 ms per
    // sweep; 1 GPU 16384^2 (64 pairs) equal at 4/8/16, profiles/r3_s3/qbuild)
    // below 16 pairs (8-GPU plans) 2 rows per lane: a shorter rotation chain
    // per lane on the latency path (16384^2 P = 8: 44.1-44.5 -> 43.6-43.7 ms
    // per sweep, profiles/r5_ab/qb2)
    if (c.P >= 64)
      hipLaunchKernelGGL((qbuild_kernel<T, W, RL>), dim3(c.P, qbuild_blocks<W, RL>()),
                         dim3(kQbThreads), 0, c.st, c.rec, c.nsteps, c.skipb[b], c.Qb[b]);
    else if (W == 64 && c.P < 16)
      hipLaunchKernelGGL((qbuild_kernel<T, W, 2>), dim3(c.P, qbuild_blocks<W, 2>()),
                         dim3(kQbThreads), 0, c.st, c.rec, c.nsteps, c.skipb[b], c.Qb[b]);
    else
      hipLaunchKernelGGL((qbuild_kernel<T, W, 4>), dim3(c.P, qbuild_blocks<W, 4>()),
                         dim3(kQbThreads), 0, c.st, c.rec, c.nsteps, c.skipb[b], c.Qb[b]);
  } else if (mode == 2)
    hipLaunchKernelGGL((evd_kernel<T, W, EVD_BIP>), dim3(c.P), dim3(evd_threads(W)), 0, c.st, pr,
                       0, c.slabs, c.g.gchunks, c.D, c.Qb[b], c.skipb[b], (T)tol, absmode,
                       max_inner, metric);
  else
    hipLaunchKernelGGL((evd_kernel<T, W, EVD_CYCLIC>), dim3(c.P), dim3(evd_threads(W)), 0, c.st,
                       pr, full, c.slabs, c.g.gchunks, c.D, c.Qb[b], c.skipb[b], (T)tol, absmode,
                       max_inner, metric);
  SVDJ_LAUNCH_CHECK();
  return 0;
}

template <typename T, int W>
static int launch_apply(const Chain<T>& c, int s, int mma, uint32_t* metric) {
  const int b = s & 1;
  const int32_t* pr = c.pairs + (size_t)s * c.P * 2;
  const int nv = c.V ? c.n_v : 0, ych = c.V ? c.g.v_chunks : 0;
  const int mode = c.modes ? c.modes[s] : 0;
  if (mode == 5) return 0;
  if (mode == 4) {
    if constexpr (sizeof(T) == 4 && W == 64) {
      if (mma != 1 && mma != 2) {
        set_error("quad steps run the split-bf16 apply (mma 1 or 2), got %d", mma);
        return -3;
      }
      // T-stationary persistent apply (apply_quad_ts_kernel)
      const int nq = c.P / 2, at = c.m_pad / 32, vt = c.V ? c.n_v / 32 : 0;
      uint32_t* work = metric ? metric + 6 : nullptr;
      // cheap k halves: |T - I| <= 2^-7 (A/B only: SVDJ_DEBUG cheap_log2, svdj_debug.h)
      static const float cheap_tol = ldexpf(1.0f, -svdj_debug_knob("cheap_log2", 7));
      // persistent grid (A/B override: SVDJ_DEBUG apply_grid)
      static const int grid_knob = svdj_debug_knob("apply_grid", 0);
      const int grid = grid_knob > 0 ? grid_knob : c.shared ? quad_ts_grid_shared(nq) : kQuadTsGrid;
      if (mma == 1)
        hipLaunchKernelGGL((apply_quad_ts_kernel<3>), dim3(grid), dim3(kQuadTsThreads), 0,
                           c.st, c.A, c.lda, at, c.V, c.ldv, vt, pr, nq, c.Ts[b], c.skip1[b],
                           c.skip2[b], work, cheap_tol);
      else
        hipLaunchKernelGGL((apply_quad_ts_kernel<2>), dim3(grid), dim3(kQuadTsThreads), 0,
                           c.st, c.A, c.lda, at, c.V, c.ldv, vt, pr, nq, c.Ts[b], c.skip1[b],
                           c.skip2[b], work);
      SVDJ_LAUNCH_CHECK();
      return 0;
    } else {
      set_error("quad steps need fp32 data and W = 64");
      return -3;
    }
  }
  const dim3 grid(c.P, c.g.a_chunks + ych);
  if constexpr (sizeof(T) == 4) {
    if (mma == 1 || mma == 2) {
      if (mma == 1)
        hipLaunchKernelGGL((apply_split_kernel<W, 3>), grid, dim3(kApplyThreads), 0, c.st, c.A,
                           c.lda, c.g.a_chunks, c.g.rows_a, c.m_pad, c.V, c.ldv, c.g.rows_v, nv,
                           pr, c.Qb[b], c.skipb[b], (stream_order() >> 1) & 1);
      else
        hipLaunchKernelGGL((apply_split_kernel<W, 2>), grid, dim3(kApplyThreads), 0, c.st, c.A,
                           c.lda, c.g.a_chunks, c.g.rows_a, c.m_pad, c.V, c.ldv, c.g.rows_v, nv,
                           pr, c.Qb[b], c.skipb[b], (stream_order() >> 1) & 1);
      SVDJ_LAUNCH_CHECK();
      return 0;
    }
  }
  hipLaunchKernelGGL((apply_kernel<T, W>), grid, dim3(apply_threads<T, W>()), 0, c.st, c.A, c.lda,
                     c.g.a_chunks, c.g.rows_a, c.m_pad, c.V, c.ldv, c.g.rows_v, nv, pr, c.Qb[b],
                     c.skipb[b]);
  SVDJ_LAUNCH_CHECK();
  return 0;
}

// Step pipeline on the chain's stream: gram(s) -> evd(s) -> apply(s).
//
// mma: 0 = native matrix cores for the data type (f32 / f64 MFMA),
//      1 = fp32 data on bf16 MFMA, 3-way split (fp32-level accuracy),
//      2 = fp32 data on bf16 MFMA, 2-way split (~2^-17 accuracy, fast mode).
// Both split modes run in delta form, Y = X + X (Q - I) (apply_split_kernel).
// Measured on MI355X (bench.py accuracy block, profiles/r3_s3/bf16x6,
// profiles/r4_accuracy): mode 1 matches the f32 MFMA path in U/V orthogonality
// and sigma error (16384^2: 2.43e-7 both), its residual is 1.37-1.55e-5 vs
// 1.03-1.05e-5, and it is 12-23 % faster per sweep for W = 64, so it is the
// fp32 default there (svdj_choose_mma).  Deferring V's rotation to a side
// stream (it is not needed by the next Gram) was measured neutral on one
// stream and 22 % slower with two chains (8192^2, round 4): not kept.
template <typename T, int W>
static int block_steps_t(const Chain<T>& c, double tol, int absmode, int max_inner,
                         uint32_t* metric, int mma) {
  for (int s = 0; s < c.steps; ++s) {
    int rc = launch_gram_evd<T, W>(c, s, tol, absmode, max_inner, metric, mma);
    if (!rc) rc = launch_apply<T, W>(c, s, mma, metric);
    if (rc) return rc;
  }
  return 0;
}

}  // namespace svdj

using namespace svdj;

// Cross-step EVD ordering for a step of `pairs` pairs of W-wide blocks
// (models/block.py choose_inner_order, measurements there): 2 = cross-only
// (low-latency EVD + row-parallel Q build) for fp32 W = 64 and for fp64
// W = 64 with more than 16 pairs, else 1 = bipartite.  The inner_order codes
// of svdj_block_solve / svdj_dist_problem.
extern "C" int svdj_choose_inner_order(int dtype, int W, int pairs) {
  if (W != 64) return 1;
  return (dtype == 0 || pairs > 16) ? 2 : 1;
}

// Default matrix-core mode ("auto") for data type `dtype` (0 fp32, 1 fp64)
// and block width W (models/block.py choose_mma): the split-bf16 apply for
// fp32 W = 64; W = 32 steps stay on f32 MFMA (4096^2 P=8
// rank plan, W = 32: 8.55 vs 9.61 ms per sweep with the split).
extern "C" int svdj_choose_mma(int dtype, int W) { return (dtype == 0 && W == 64) ? 1 : 0; }

extern "C" size_t svdj_block_workspace_bytes(int dtype, int W, int P, int m_pad, int quad) {
  return ws_bytes_for(dtype == 1 ? 8 : 4, W, P, m_pad, quad != 0);
}

static int check_dims(int m_pad, int lda, const void* V, int n_v, int ldv, int mma) {
  if (m_pad <= 0 || m_pad % SVDJ_ROW_ALIGN || lda < m_pad) {
    set_error("bad m_pad/lda %d/%d", m_pad, lda);
    return -2;
  }
  if (V && (n_v <= 0 || n_v % SVDJ_ROW_ALIGN || ldv < n_v)) {
    set_error("bad n_v/ldv %d/%d", n_v, ldv);
    return -2;
  }
  if (mma < 0 || mma > 2) {
    set_error("bad matrix-core mode %d", mma);
    return -2;
  }
  return 0;
}

template <typename T, int W>
static int steps_dispatch(int m_pad, void* A, int lda, void* V, int n_v, int ldv, void* D,
                          const int32_t* pairs, int P, int steps, const int32_t* modes,
                          double tol, int absmode, int max_inner, void* ws, size_t ws_bytes,
                          uint32_t* metric, int mma, void* stream) {
  Chain<T> c;
  const int gram2 = (mma >> 8) & 1;  // svdj_block_steps' mma bit 8
  const int shared = (mma >> 9) & 1;  // bit 9
  mma &= 0xff;
  int rc = chain_init<T, W>(c, m_pad, (T*)A, lda, (T*)V, n_v, ldv, (T*)D, pairs, P, steps, modes,
                            ws, ws_bytes, mma, (hipStream_t)stream);
  if (rc) return rc;
  if (gram2) c.gram_np = 2;
  c.shared = shared;
  return block_steps_t<T, W>(c, tol, absmode, max_inner, metric, mma);
}

extern "C" int svdj_block_steps(int dtype, int W, int m_pad, void* A, int lda, void* V, int n_v,
                                int ldv, void* D, const int32_t* pairs, int P, int steps,
                                const int32_t* modes, double tol, int tol_mode, int max_inner,
                                void* ws, size_t ws_bytes, uint32_t* metric, int mma,
                                void* stream) {
  // mma bits 0-7: the apply's matrix-core mode; bit 8: quad Gram with 2 bf16
  // parts (gram_quad_kernel<0, 2>) for sweeps far from convergence; bit 9:
  // another chain runs concurrently on this GPU (quad apply on
  // quad_ts_grid_shared workgroups)
  int rc = check_dims(m_pad, lda, V, n_v, ldv, mma & 0xff);
  if (rc) return rc;
  if (tol_mode != 0 && tol_mode != 1) {
    set_error("bad tol_mode %d (0 relative, 1 absolute)", tol_mode);
    return -2;
  }
  if (P <= 0 || steps < 0) return 0;
#define SVDJ_STEPS_ARGS                                                                       \
  m_pad, A, lda, V, n_v, ldv, D, pairs, P, steps, modes, tol, tol_mode, max_inner, ws, ws_bytes, \
      metric, mma, stream
  if (dtype == 0 && W == 32) return steps_dispatch<float, 32>(SVDJ_STEPS_ARGS);
  if (dtype == 0 && W == 64) return steps_dispatch<float, 64>(SVDJ_STEPS_ARGS);
  if (dtype == 1 && W == 32) return steps_dispatch<double, 32>(SVDJ_STEPS_ARGS);
  if (dtype == 1 && W == 64) return steps_dispatch<double, 64>(SVDJ_STEPS_ARGS);
#undef SVDJ_STEPS_ARGS
  set_error("unsupported (dtype=%d, W=%d); supported: W in {32, 64}", dtype, W);
  return -3;
}

extern "C" int svdj_block_solve(int dtype, int W, int m_pad, void* A, int lda, void* V, int n_v,
                                int ldv, void* D, int ncols, double tol, int tol_mode,
                                int max_inner, int max_sweeps, int inner_order, void* ws,
                                size_t ws_bytes, uint32_t* metric, double* hist, int mma,
                                int stop_rule, void* stream) {
  if (W <= 0 || ncols % W) {
    set_error("ncols %d not a multiple of W %d", ncols, W);
    return -2;
  }
  const int nb = ncols / W;
  if (nb < 2 || (nb & 1)) {
    set_error("block count %d must be even and >= 2", nb);
    return -2;
  }
  const int P = nb / 2, steps = nb - 1;
  std::vector<int32_t> h((size_t)steps * P * 2);
  for (int r = 0; r < steps; ++r) {
    int32_t* o = h.data() + (size_t)r * P * 2;
    o[0] = r;
    o[1] = nb - 1;
    for (int k = 1; k < P; ++k) {
      int a = (r + k) % (nb - 1), b = (r - k + nb - 1) % (nb - 1);
      o[2 * k] = a < b ? a : b;
      o[2 * k + 1] = a < b ? b : a;
    }
  }
  if (inner_order == 3) inner_order = svdj_choose_inner_order(dtype, W, P);  // auto
  if (inner_order < 0 || inner_order > 2) {
    set_error("inner_order %d (0 cyclic, 1 bipartite, 2 cross, 3 auto)", inner_order);
    return -2;
  }
  std::vector<int32_t> modes(steps, inner_order == 2 ? 3 : (inner_order ? 2 : 0));
  modes[0] = 1;
  hipStream_t st = (hipStream_t)stream;
  int32_t* dpairs = nullptr;
  SVDJ_HIP_CHECK(hipMallocAsync((void**)&dpairs, h.size() * sizeof(int32_t), st));
  SVDJ_HIP_CHECK(hipMemcpyAsync(dpairs, h.data(), h.size() * sizeof(int32_t),
                                hipMemcpyHostToDevice, st));
  int sweeps = 0, rc = 0;
  uint32_t hm[6];
  // underflow floor of this solve (metric[2..3])
  rc = svdj_set_norm_floor_scaled(dtype, m_pad, D, ncols, metric, stream);
  for (int sw = 0; sw < max_sweeps && rc >= 0; ++sw) {
    if (svdj_reset_metric(metric, stream) != 0) { rc = -100; break; }
    rc = svdj_block_steps(dtype, W, m_pad, A, lda, V, n_v, ldv, D, dpairs, P, steps,
                          modes.data(), tol, tol_mode, max_inner, ws, ws_bytes, metric, mma,
                          stream);
    if (rc) break;
    if (hipMemcpyAsync(hm, metric, sizeof(hm), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      set_error("metric readback failed");
      rc = -100;
      break;
    }
    float mx, ms;
    memcpy(&mx, &hm[0], sizeof(float));
    memcpy(&ms, &hm[4], sizeof(float));
    if (hist) hist[sw] = mx;
    sweeps = sw + 1;
    if (svdj_sweep_converged_inline(mx, ms, hm[1], hm[5], tol, tol_mode, stop_rule)) break;
  }
  (void)hipFreeAsync(dpairs, st);
  return rc ? rc : sweeps;
}

// Cross Gram alone (tests / kernel A/B): slabs (P x nchunk x W x W) of
// A_bi^T A_bj for the device pair list, with the given row chunking.
extern "C" int svdj_gram_cross(int dtype, int W, const void* A, int lda, int m_pad,
                               const int32_t* pairs, int P, int rows_per_chunk, void* slabs,
                               void* stream) {
  if (m_pad <= 0 || m_pad % SVDJ_ROW_ALIGN || lda < m_pad || P <= 0 || rows_per_chunk <= 0 ||
      rows_per_chunk % SVDJ_ROW_ALIGN) {
    set_error("svdj_gram_cross: bad m_pad/lda/P/rows %d/%d/%d/%d", m_pad, lda, P, rows_per_chunk);
    return -2;
  }
  hipStream_t st = (hipStream_t)stream;
  const int nchunk = (m_pad + rows_per_chunk - 1) / rows_per_chunk;
  if (dtype == 0 && W == 64) {
    if (lda % 4) {
      set_error("svdj_gram_cross: lda %d must be a multiple of 4", lda);
      return -2;
    }
    hipLaunchKernelGGL((gram_cross_f32_kernel<GRAM_CROSS>), dim3(P, nchunk, 1), dim3(kGramThreads),
                       0, st, (const float*)A, lda, m_pad, pairs, rows_per_chunk, (float*)slabs, 0);
  } else if (dtype == 0 && W == 32) {
    hipLaunchKernelGGL((gram_kernel<float, 32, GRAM_CROSS>), dim3(P, nchunk, 1), dim3(kGramThreads),
                       0, st, (const float*)A, lda, m_pad, pairs, rows_per_chunk, (float*)slabs);
  } else {
    set_error("svdj_gram_cross: unsupported dtype=%d W=%d", dtype, W);
    return -3;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("svdj_gram_cross launch: %s", hipGetErrorString(e));
    return -101;
  }
  return 0;
}

// The six cross Grams of a quad step (fp32, W = 64) alone (tests / kernel
// A/B): pairs = the step's P pairs in quad order ((a,c),(b,d) per quad);
// slabs (3P x nchunk x W x W): [0, P) the pairs' Grams, then C_ad, C_bc, C_ab,
// C_cd of every quad (gram_quad_kernel).
extern "C" int svdj_gram_quad(const void* A, int lda, int m_pad, const int32_t* pairs, int P,
                              int rows_per_chunk, void* slabs, int parts, void* stream) {
  if (m_pad <= 0 || m_pad % SVDJ_ROW_ALIGN || lda < m_pad || lda % 4 || P <= 0 || P % 2 ||
      rows_per_chunk <= 0 || rows_per_chunk % SVDJ_ROW_ALIGN || (parts != 2 && parts != 3)) {
    set_error("svdj_gram_quad: bad m_pad/lda/P/rows/parts %d/%d/%d/%d/%d", m_pad, lda, P,
              rows_per_chunk, parts);
    return -2;
  }
  const int nchunk = (m_pad + rows_per_chunk - 1) / rows_per_chunk;
  if (parts == 2)
    hipLaunchKernelGGL((gram_quad_kernel<0, 2>), dim3(P / 2, nchunk), dim3(kGramQThreads), 0,
                       (hipStream_t)stream, (const float*)A, lda, m_pad, pairs, P, rows_per_chunk,
                       (float*)slabs);
  else
    hipLaunchKernelGGL((gram_quad_kernel<0, 3>), dim3(P / 2, nchunk), dim3(kGramQThreads), 0,
                       (hipStream_t)stream, (const float*)A, lda, m_pad, pairs, P, rows_per_chunk,
                       (float*)slabs);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("svdj_gram_quad launch: %s", hipGetErrorString(e));
    return -101;
  }
  return 0;
}

// Test/diagnostic hook: X <- X Q for ONE column-block pair (blocks 0 and 1 of
// X, 2W columns with leading dimension ld, rows padded to SVDJ_ROW_ALIGN),
// Q row-major 2W x 2W on the device, with the given matrix-core mode.
extern "C" int svdj_apply_q(int dtype, int W, int mma, void* X, int rows, int ld, const void* Q,
                            void* stream) {
  if (rows <= 0 || rows % SVDJ_ROW_ALIGN || ld < rows) {
    set_error("bad rows/ld %d/%d", rows, ld);
    return -2;
  }
  static const int32_t hpair[2] = {0, 1};
  static const int32_t hskip[1] = {0};
  hipStream_t st = (hipStream_t)stream;
  int32_t* dbuf = nullptr;
  SVDJ_HIP_CHECK(hipMallocAsync((void**)&dbuf, 3 * sizeof(int32_t), st));
  SVDJ_HIP_CHECK(hipMemcpyAsync(dbuf, hpair, 2 * sizeof(int32_t), hipMemcpyHostToDevice, st));
  SVDJ_HIP_CHECK(hipMemcpyAsync(dbuf + 2, hskip, sizeof(int32_t), hipMemcpyHostToDevice, st));
  const int rows_chunk = 512, chunks = (rows + rows_chunk - 1) / rows_chunk;
  const dim3 grid(1, chunks), blk(kApplyThreads);
  int rc = 0;
  if (dtype == 0 && mma == 1 && W == 64)
    hipLaunchKernelGGL((apply_split_kernel<64, 3>), grid, blk, 0, st, (float*)X, ld, chunks,
                       rows_chunk, rows, (float*)nullptr, 0, 0, 0, dbuf, (const float*)Q, dbuf + 2, 0);
  else if (dtype == 0 && mma == 1 && W == 32)
    hipLaunchKernelGGL((apply_split_kernel<32, 3>), grid, blk, 0, st, (float*)X, ld, chunks,
                       rows_chunk, rows, (float*)nullptr, 0, 0, 0, dbuf, (const float*)Q, dbuf + 2, 0);
  else if (dtype == 0 && mma == 2 && W == 64)
    hipLaunchKernelGGL((apply_split_kernel<64, 2>), grid, blk, 0, st, (float*)X, ld, chunks,
                       rows_chunk, rows, (float*)nullptr, 0, 0, 0, dbuf, (const float*)Q, dbuf + 2, 0);
  else if (dtype == 0 && mma == 2 && W == 32)
    hipLaunchKernelGGL((apply_split_kernel<32, 2>), grid, blk, 0, st, (float*)X, ld, chunks,
                       rows_chunk, rows, (float*)nullptr, 0, 0, 0, dbuf, (const float*)Q, dbuf + 2, 0);
  else if (dtype == 0 && mma == 0 && W == 64)
    hipLaunchKernelGGL((apply_kernel<float, 64>), grid, dim3(apply_threads<float, 64>()), 0, st, (float*)X, ld, chunks,
                       rows_chunk, rows, (float*)nullptr, 0, 0, 0, dbuf, (const float*)Q, dbuf + 2);
  else if (dtype == 0 && mma == 0 && W == 32)
    hipLaunchKernelGGL((apply_kernel<float, 32>), grid, blk, 0, st, (float*)X, ld, chunks,
                       rows_chunk, rows, (float*)nullptr, 0, 0, 0, dbuf, (const float*)Q, dbuf + 2);
  else if (dtype == 1 && mma == 0 && W == 32)
    hipLaunchKernelGGL((apply_kernel<double, 32>), grid, blk, 0, st, (double*)X, ld, chunks,
                       rows_chunk, rows, (double*)nullptr, 0, 0, 0, dbuf, (const double*)Q,
                       dbuf + 2);
  else if (dtype == 1 && mma == 0 && W == 64)
    hipLaunchKernelGGL((apply_kernel<double, 64>), grid, blk, 0, st, (double*)X, ld, chunks,
                       rows_chunk, rows, (double*)nullptr, 0, 0, 0, dbuf, (const double*)Q,
                       dbuf + 2);
  else {
    set_error("svdj_apply_q: unsupported dtype=%d W=%d mma=%d", dtype, W, mma);
    rc = -3;
  }
  if (rc == 0) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      set_error("svdj_apply_q launch: %s", hipGetErrorString(e));
      rc = -101;
    }
  }
  (void)hipFreeAsync(dbuf, st);
  return rc;
}
