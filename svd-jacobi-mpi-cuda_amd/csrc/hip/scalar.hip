// Scalar (column-pair) one-sided Jacobi step -- the reference-parity path.
//
// Reference behaviour being replaced (reference main.cu:685-766): per pair,
// the CPU computes the dot triple alpha/beta/gamma over m rows
// (main.cu:698-707), solves the 2x2 rotation on the host (main.cu:712-725),
// then does 4 synchronous H2D + 4 D2H cudaMemcpys and two launches of the
// 16-thread `jacobi_rotation` kernel (main.cu:139-147, 727-758).
//
// Here ONE launch covers a whole parallel step: one 256-thread workgroup
// (4 x wave64) per disjoint column pair.  The pair's two columns are read
// once into registers with 16-byte vector loads, the dot triple is reduced
// with 64-lane butterflies + a 4-entry LDS combine, the rotation is solved
// redundantly in every lane, and the rotated columns are written back from
// registers (A) / streamed (V).  A and V never leave HBM.  The convergence
// value |alpha|/sqrt(beta*gamma) -- computed and discarded by the reference
// (main.cu:710) -- is max-reduced into a device word and used as the stop
// test.
#include "common.hpp"
#include "svdj_hip.h"

#include <cstring>
#include <vector>

namespace svdj {

constexpr int kScalarThreads = 256;
constexpr int kScalarCacheVec = 4;  // 16-byte vectors cached per thread

template <typename T>
__global__ __launch_bounds__(kScalarThreads) void scalar_step_kernel(
    T* __restrict__ A, int lda, int m_pad, T* __restrict__ V, int ldv, int n_v,
    const int32_t* __restrict__ pairs, T tol, int tol_mode,
    uint32_t* __restrict__ metric) {
  constexpr int VEC = 16 / sizeof(T);
  using vec_t = f32x4;  // 16 bytes, reinterpreted
  const int k = blockIdx.x;
  const int p = pairs[2 * k], q = pairs[2 * k + 1];
  if (p < 0 || q < 0) return;
  const int tid = threadIdx.x;
  T* ap = A + (size_t)p * lda;
  T* aq = A + (size_t)q * lda;
  const int stride = kScalarThreads * VEC;  // rows per pass
  const bool cached = m_pad <= stride * kScalarCacheVec;

  vec_t xr[kScalarCacheVec], yr[kScalarCacheVec];
  T alpha = 0, beta = 0, gamma = 0;
  if (cached) {
#pragma unroll
    for (int r = 0; r < kScalarCacheVec; ++r) {
      const int i = r * stride + tid * VEC;
      if (i < m_pad) {
        xr[r] = *reinterpret_cast<const vec_t*>(ap + i);
        yr[r] = *reinterpret_cast<const vec_t*>(aq + i);
        const T* xs = reinterpret_cast<const T*>(&xr[r]);
        const T* ys = reinterpret_cast<const T*>(&yr[r]);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          alpha += xs[j] * ys[j];
          beta += xs[j] * xs[j];
          gamma += ys[j] * ys[j];
        }
      }
    }
  } else {
    for (int i = tid * VEC; i < m_pad; i += stride) {
      vec_t xv = *reinterpret_cast<const vec_t*>(ap + i);
      vec_t yv = *reinterpret_cast<const vec_t*>(aq + i);
      const T* xs = reinterpret_cast<const T*>(&xv);
      const T* ys = reinterpret_cast<const T*>(&yv);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        alpha += xs[j] * ys[j];
        beta += xs[j] * xs[j];
        gamma += ys[j] * ys[j];
      }
    }
  }
  alpha = wave_sum(alpha);
  beta = wave_sum(beta);
  gamma = wave_sum(gamma);
  __shared__ T red[3][kScalarThreads / SVDJ_WAVE];
  const int lane = tid & 63, wave = tid >> 6;
  if (lane == 0) {
    red[0][wave] = alpha;
    red[1][wave] = beta;
    red[2][wave] = gamma;
  }
  __syncthreads();
  alpha = beta = gamma = 0;
#pragma unroll
  for (int w = 0; w < kScalarThreads / SVDJ_WAVE; ++w) {
    alpha += red[0][w];
    beta += red[1][w];
    gamma += red[2][w];
  }
  const T nrm = sqrt(beta) * sqrt(gamma);
  if (tid == 0 && nrm > T(0)) atomic_max_pos(&metric[0], (float)(fabs(alpha) / nrm));
  const bool rotate = (tol_mode == 1) ? (fabs(alpha) > tol)
                                      : (nrm > T(0) && fabs(alpha) > tol * nrm);
  if (!rotate || alpha == T(0)) return;
  T c, s, t;
  schur_rotation(alpha, beta, gamma, c, s, t);
  if (tid == 0) atomicAdd(&metric[1], 1u);

  auto rot = [&](vec_t& xv, vec_t& yv) {
    T* xs = reinterpret_cast<T*>(&xv);
    T* ys = reinterpret_cast<T*>(&yv);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const T x = xs[j], y = ys[j];
      xs[j] = c * x - s * y;
      ys[j] = s * x + c * y;
    }
  };
  if (cached) {
#pragma unroll
    for (int r = 0; r < kScalarCacheVec; ++r) {
      const int i = r * stride + tid * VEC;
      if (i < m_pad) {
        rot(xr[r], yr[r]);
        *reinterpret_cast<vec_t*>(ap + i) = xr[r];
        *reinterpret_cast<vec_t*>(aq + i) = yr[r];
      }
    }
  } else {
    for (int i = tid * VEC; i < m_pad; i += stride) {
      vec_t xv = *reinterpret_cast<const vec_t*>(ap + i);
      vec_t yv = *reinterpret_cast<const vec_t*>(aq + i);
      rot(xv, yv);
      *reinterpret_cast<vec_t*>(ap + i) = xv;
      *reinterpret_cast<vec_t*>(aq + i) = yv;
    }
  }
  if (V != nullptr) {
    T* vp = V + (size_t)p * ldv;
    T* vq = V + (size_t)q * ldv;
    for (int i = tid * VEC; i < n_v; i += stride) {
      vec_t xv = *reinterpret_cast<const vec_t*>(vp + i);
      vec_t yv = *reinterpret_cast<const vec_t*>(vq + i);
      rot(xv, yv);
      *reinterpret_cast<vec_t*>(vp + i) = xv;
      *reinterpret_cast<vec_t*>(vq + i) = yv;
    }
  }
}

template <typename T>
static int scalar_step_t(int m_pad, void* A, int lda, void* V, int n_v, int ldv,
                         const int32_t* pairs, int per_step, double tol,
                         int tol_mode, uint32_t* metric, hipStream_t st) {
  if (per_step <= 0) return 0;
  hipLaunchKernelGGL(scalar_step_kernel<T>, dim3(per_step), dim3(kScalarThreads), 0, st,
                     (T*)A, lda, m_pad, (T*)V, ldv, n_v, pairs, (T)tol, tol_mode, metric);
  SVDJ_LAUNCH_CHECK();
  return 0;
}

}  // namespace svdj

using namespace svdj;

static int check_dims(int m_pad, int lda, int n_v, int ldv, const void* V) {
  if (m_pad <= 0 || (m_pad % SVDJ_ROW_ALIGN) != 0 || lda < m_pad) {
    set_error("bad m_pad/lda (%d/%d): m_pad must be a positive multiple of %d", m_pad, lda,
              SVDJ_ROW_ALIGN);
    return -2;
  }
  if (V != nullptr && (n_v <= 0 || (n_v % SVDJ_ROW_ALIGN) != 0 || ldv < n_v)) {
    set_error("bad n_v/ldv (%d/%d)", n_v, ldv);
    return -2;
  }
  return 0;
}

extern "C" int svdj_scalar_step(int dtype, int m_pad, void* A, int lda, void* V, int n_v,
                                int ldv, const int32_t* sched, int per_step, double tol,
                                int tol_mode, uint32_t* metric, void* stream) {
  int rc = check_dims(m_pad, lda, n_v, ldv, V);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    return scalar_step_t<float>(m_pad, A, lda, V, n_v, ldv, sched, per_step, tol, tol_mode, metric, st);
  if (dtype == 1)
    return scalar_step_t<double>(m_pad, A, lda, V, n_v, ldv, sched, per_step, tol, tol_mode, metric, st);
  set_error("unsupported dtype %d", dtype);
  return -3;
}

extern "C" int svdj_scalar_solve(int dtype, int m_pad, void* A, int lda, void* V, int n_v,
                                 int ldv, const int32_t* sched, int steps, int per_step,
                                 double tol, int tol_mode, int max_sweeps, uint32_t* metric,
                                 double* hist, void* stream) {
  int rc = check_dims(m_pad, lda, n_v, ldv, V);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  uint32_t hm[2];
  int sweeps = 0;
  for (int sw = 0; sw < max_sweeps; ++sw) {
    SVDJ_HIP_CHECK(hipMemsetAsync(metric, 0, 2 * sizeof(uint32_t), st));
    for (int s = 0; s < steps; ++s) {
      rc = svdj_scalar_step(dtype, m_pad, A, lda, V, n_v, ldv, sched + (size_t)s * per_step * 2,
                            per_step, tol, tol_mode, metric, st);
      if (rc) return rc;
    }
    SVDJ_HIP_CHECK(hipMemcpyAsync(hm, metric, sizeof(hm), hipMemcpyDeviceToHost, st));
    SVDJ_HIP_CHECK(hipStreamSynchronize(st));
    float mx;
    memcpy(&mx, &hm[0], sizeof(float));
    if (hist) hist[sw] = mx;
    sweeps = sw + 1;
    if (hm[1] == 0) break;
  }
  return sweeps;
}
