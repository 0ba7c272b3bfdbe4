// Initialisation / post-processing kernels and library utilities.
//
// Replaces the reference's OpenMP host loops for V := I
// (reference main.cu:461-474) and for sigma / U (main.cu:1394-1421):
//   * sigma_k = ||a_k|| with fp64 accumulation (one wave per column),
//   * U = A / sigma with a sigma == 0 guard (the reference divides blindly),
//   * squared column norms D used to seed the block path.
#include "common.hpp"
#include "svdj_hip.h"

#include <stdarg.h>
#include <string.h>

namespace svdj {

static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

template <typename T>
__global__ __launch_bounds__(256) void identity_kernel(T* V, int n_v, int ldv, int ncols,
                                                        int col_offset) {
  const int c = blockIdx.x;
  T* col = V + (size_t)c * ldv;
  const int diag = c + col_offset;
  for (int i = threadIdx.x; i < n_v; i += blockDim.x) col[i] = (i == diag) ? T(1) : T(0);
}

// One wave per column: sum of squares in fp64.
template <typename T>
__global__ __launch_bounds__(256) void colnorm2_kernel(const T* __restrict__ A, int m_pad,
                                                        int lda, int ncols, T* __restrict__ D) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + wave;
  if (c >= ncols) return;
  const T* a = A + (size_t)c * lda;
  double acc = 0.0;
  for (int i = lane; i < m_pad; i += 64) {
    const double x = (double)a[i];
    acc += x * x;
  }
  acc = wave_sum(acc);
  if (lane == 0) D[c] = (T)acc;
}

template <typename T>
__global__ __launch_bounds__(256) void finalize_kernel(T* __restrict__ A, int m_pad, int lda,
                                                        int ncols, T* __restrict__ sigma,
                                                        int scale_u) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + wave;
  if (c >= ncols) return;
  T* a = A + (size_t)c * lda;
  double acc = 0.0;
  for (int i = lane; i < m_pad; i += 64) {
    const double x = (double)a[i];
    acc += x * x;
  }
  acc = wave_sum(acc);
  const double nrm = sqrt(acc);
  if (lane == 0) sigma[c] = (T)nrm;
  if (scale_u && nrm > 0.0) {
    const T inv = (T)(1.0 / nrm);
    for (int i = lane; i < m_pad; i += 64) a[i] *= inv;
  }
}

// One-lane timed wait on a stream (the simulated-exchange link model of
// parallel/comm.py SimCommunicator): returns once the constant-rate wall
// clock has advanced by `ticks` (always terminates; sleeps between polls).
__global__ __launch_bounds__(64) void spin_kernel(unsigned long long ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

}  // namespace svdj

using namespace svdj;

extern "C" int svdj_spin_ns(double ns, void* stream) {
  if (!(ns > 0.0)) return 0;
  const double cap = 10e9;  // 10 s: a modelled transfer never needs more
  int dev = 0, khz = 0;
  SVDJ_HIP_CHECK(hipStreamGetDevice((hipStream_t)stream, &dev));
  SVDJ_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  if (khz <= 0) khz = 100000;  // 100 MHz on gfx9
  const unsigned long long ticks = (unsigned long long)((ns < cap ? ns : cap) * 1e-6 * khz);
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ticks);
  SVDJ_LAUNCH_CHECK();
  return 0;
}

extern "C" const char* svdj_hip_last_error(void) { return g_err; }

extern "C" const char* svdj_hip_version(void) {
  return "svdj-hip 0.1 gfx950 (mfma_f32_32x32x2f32, mfma_f32_32x32x16_bf16 split-fp32, mfma_f64_16x16x4f64)";
}

extern "C" int svdj_set_identity(int dtype, void* V, int n_v, int ldv, int ncols, int col_offset,
                                 void* stream) {
  if (ncols <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(identity_kernel<float>, dim3(ncols), dim3(256), 0, st, (float*)V, n_v, ldv,
                       ncols, col_offset);
  else if (dtype == 1)
    hipLaunchKernelGGL(identity_kernel<double>, dim3(ncols), dim3(256), 0, st, (double*)V, n_v,
                       ldv, ncols, col_offset);
  else {
    set_error("unsupported dtype %d", dtype);
    return -3;
  }
  SVDJ_LAUNCH_CHECK();
  return 0;
}

extern "C" int svdj_col_norms2(int dtype, const void* A, int m_pad, int lda, int ncols, void* D,
                               void* stream) {
  if (ncols <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int blocks = (ncols + 3) / 4;
  if (dtype == 0)
    hipLaunchKernelGGL(colnorm2_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)A,
                       m_pad, lda, ncols, (float*)D);
  else if (dtype == 1)
    hipLaunchKernelGGL(colnorm2_kernel<double>, dim3(blocks), dim3(256), 0, st, (const double*)A,
                       m_pad, lda, ncols, (double*)D);
  else {
    set_error("unsupported dtype %d", dtype);
    return -3;
  }
  SVDJ_LAUNCH_CHECK();
  return 0;
}

// metric[2..3] (a double) = the negligible-column floor of the block EVDs
// (block.hip needs_rotation).  svdj_norm_floor_value is its scale-relative
// factor m realmin / eps (times the largest squared column norm, see
// svdj_set_norm_floor_scaled).
__global__ void norm_floor_kernel(double v, uint32_t* __restrict__ metric) {
  if (threadIdx.x == 0) *reinterpret_cast<double*>(metric + 2) = v;
}

extern "C" double svdj_norm_floor_value(int dtype, int m) {
  return dtype == 1 ? (double)m * 2.2250738585072014e-308 / 2.220446049250313e-16
                    : (double)m * 1.1754943508222875e-38 / 1.1920928955078125e-07;
}

extern "C" int svdj_set_norm_floor(double floor, uint32_t* metric, void* stream) {
  hipLaunchKernelGGL(norm_floor_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, floor, metric);
  SVDJ_LAUNCH_CHECK();
  return 0;
}

// Per-sweep words of a block-path metric: [0], [1] and [4..7] (svdj_stop.h).
extern "C" int svdj_reset_metric(uint32_t* metric, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  SVDJ_HIP_CHECK(hipMemsetAsync(metric, 0, 2 * sizeof(uint32_t), st));
  SVDJ_HIP_CHECK(hipMemsetAsync(metric + 4, 0, (SVDJ_METRIC_WORDS - 4) * sizeof(uint32_t), st));
  return 0;
}

// Scale-relative floor (ops/kernels.py norm_floor): metric[2..3] =
// max(m realmin, m realmin / eps * max_j D[j]) over the n squared norms D,
// on the device (one workgroup).
template <typename T>
__global__ __launch_bounds__(256) void norm_floor_scaled_kernel(const T* __restrict__ D, int n,
                                                                double fabs_, double frel,
                                                                uint32_t* __restrict__ metric) {
  __shared__ double wm[4];
  double mx = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) mx = fmax(mx, (double)D[i]);
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    mx = fmax(fmax(wm[0], wm[1]), fmax(wm[2], wm[3]));
    *reinterpret_cast<double*>(metric + 2) = fmax(fabs_, frel * mx);
  }
}

extern "C" int svdj_set_norm_floor_scaled(int dtype, int m, const void* D, int n,
                                          uint32_t* metric, void* stream) {
  const double tiny = dtype == 1 ? 2.2250738585072014e-308 : 1.1754943508222875e-38;
  const double fabs_ = (double)m * tiny, frel = svdj_norm_floor_value(dtype, m);
  if (dtype == 1)
    hipLaunchKernelGGL(norm_floor_scaled_kernel<double>, dim3(1), dim3(256), 0,
                       (hipStream_t)stream, (const double*)D, n, fabs_, frel, metric);
  else
    hipLaunchKernelGGL(norm_floor_scaled_kernel<float>, dim3(1), dim3(256), 0,
                       (hipStream_t)stream, (const float*)D, n, fabs_, frel, metric);
  SVDJ_LAUNCH_CHECK();
  return 0;
}

extern "C" int svdj_finalize(int dtype, void* A, int m_pad, int lda, int ncols, void* sigma,
                             int scale_u, void* stream) {
  if (ncols <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int blocks = (ncols + 3) / 4;
  if (dtype == 0)
    hipLaunchKernelGGL(finalize_kernel<float>, dim3(blocks), dim3(256), 0, st, (float*)A, m_pad,
                       lda, ncols, (float*)sigma, scale_u);
  else if (dtype == 1)
    hipLaunchKernelGGL(finalize_kernel<double>, dim3(blocks), dim3(256), 0, st, (double*)A, m_pad,
                       lda, ncols, (double*)sigma, scale_u);
  else {
    set_error("unsupported dtype %d", dtype);
    return -3;
  }
  SVDJ_LAUNCH_CHECK();
  return 0;
}
