// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// Wave64 everywhere: reductions use 64-lane butterflies (__shfl_xor over
// 32,16,8,4,2,1), never 32-lane warp idioms.  MFMA traits describe the two
// matrix-core shapes the framework uses:
//   fp32: v_mfma_f32_32x32x2_f32  (exact f32 fma chain, 16 acc regs/lane)
//   fp64: v_mfma_f64_16x16x4_f64  (4 f64 acc regs/lane, own C/D map)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define SVDJ_WAVE 64

namespace svdj {

// --------------------------------------------------------------- error text
void set_error(const char* fmt, ...);

#define SVDJ_HIP_CHECK(expr)                                                   \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      ::svdj::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,           \
                        hipGetErrorString(_e));                                \
      return -100;                                                             \
    }                                                                          \
  } while (0)

#define SVDJ_LAUNCH_CHECK()                                                    \
  do {                                                                         \
    hipError_t _e = hipGetLastError();                                         \
    if (_e != hipSuccess) {                                                    \
      ::svdj::set_error("%s:%d launch -> %s", __FILE__, __LINE__,              \
                        hipGetErrorString(_e));                                \
      return -101;                                                             \
    }                                                                          \
  } while (0)

// ------------------------------------------------------------ wave helpers
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, SVDJ_WAVE);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    T w = __shfl_xor(v, o, SVDJ_WAVE);
    v = v > w ? v : w;
  }
  return v;
}

// Positive float max via integer atomics (bit order == value order for x>=0).
__device__ __forceinline__ void atomic_max_pos(uint32_t* addr, float v) {
  if (!(v > 0.0f)) return;  // also drops NaN
  atomicMax(addr, __float_as_uint(v));
}

// Overflow-safe symmetric Schur rotation, reference formula
// (reference main.cu:715-725): tau=(gamma-beta)/(2 alpha),
// t = sign(tau)/(|tau|+sqrt(1+tau^2)), c = 1/sqrt(1+t^2), s = t c.
// Column update convention: x' = c x - s y ; y' = s x + c y.
template <typename T>
__device__ __forceinline__ void schur_rotation(T alpha, T beta, T gamma, T& c, T& s, T& t) {
  const T tau = (gamma - beta) / (T(2) * alpha);
  const T big = sizeof(T) == 8 ? T(1e150) : T(1e18);
  const T at = fabs(tau);
  if (at > big) {
    t = T(1) / (T(2) * tau);
  } else {
    t = T(1) / (at + sqrt(T(1) + tau * tau));
    if (tau < T(0)) t = -t;
  }
  c = T(1) / sqrt(T(1) + t * t);
  s = t * c;
}

// ------------------------------------------------------------- MFMA traits
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using f64x2 = __attribute__((ext_vector_type(2))) double;
using f64x4 = __attribute__((ext_vector_type(4))) double;

template <typename T>
struct Mfma;

// v_mfma_f32_32x32x2_f32: lane l holds A[i=l&31][k=l>>5], B[k=l>>5][j=l&31];
// acc reg e -> D[row=(e&3)+8(e>>2)+4(l>>5)][col=l&31].
template <>
struct Mfma<float> {
  static constexpr int TILE = 32;   // output tile edge
  static constexpr int KG = 2;      // k groups across the wave (lane >> 5)
  static constexpr int NACC = 16;   // accumulator values per lane
  static constexpr int LPL = 16;    // rows per lane per 32-row slab (gram)
  using acc_t = f32x16;
  __device__ static __forceinline__ int lane_col(int l) { return l & 31; }
  __device__ static __forceinline__ int lane_kg(int l) { return l >> 5; }
  __device__ static __forceinline__ int acc_row(int e, int l) {
    return (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
  }
  __host__ __device__ static constexpr int acc_row_uni(int e) { return (e & 3) + 8 * (e >> 2); }
  __device__ static __forceinline__ int acc_row_lane(int l) { return 4 * (l >> 5); }
  __device__ static __forceinline__ acc_t mfma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ acc_t zero() {
    acc_t z;
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = 0.0f;
    return z;
  }
};

// v_mfma_f64_16x16x4_f64: lane l holds A[i=l&15][k=l>>4], B[k=l>>4][j=l&15];
// acc reg e -> D[row=(l>>4)+4e][col=l&15]  (f64 has its own C/D map).
template <>
struct Mfma<double> {
  static constexpr int TILE = 16;
  static constexpr int KG = 4;
  static constexpr int NACC = 4;
  static constexpr int LPL = 8;
  using acc_t = f64x4;
  __device__ static __forceinline__ int lane_col(int l) { return l & 15; }
  __device__ static __forceinline__ int lane_kg(int l) { return l >> 4; }
  __device__ static __forceinline__ int acc_row(int e, int l) { return (l >> 4) + 4 * e; }
  __host__ __device__ static constexpr int acc_row_uni(int e) { return 4 * e; }
  __device__ static __forceinline__ int acc_row_lane(int l) { return l >> 4; }
  __device__ static __forceinline__ acc_t mfma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ acc_t zero() {
    acc_t z;
    z[0] = z[1] = z[2] = z[3] = 0.0;
    return z;
  }
};

// 64 bytes of one column, rows [r, r+LPL): 4 x 16-byte vector loads.
template <typename T>
__device__ __forceinline__ void load_col64B(const T* __restrict__ p, T (&v)[64 / sizeof(T)]) {
  const f32x4* q = reinterpret_cast<const f32x4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x4 x = q[i];
    const T* xs = reinterpret_cast<const T*>(&x);
#pragma unroll
    for (int j = 0; j < 16 / (int)sizeof(T); ++j) v[i * (16 / sizeof(T)) + j] = xs[j];
  }
}

}  // namespace svdj
