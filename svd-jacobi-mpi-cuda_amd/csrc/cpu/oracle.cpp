// CPU oracle: scalar one-sided Hestenes Jacobi SVD (host C++ / OpenMP).
//
// This is BASELINE config 1 ("512x512 fp64 random dense matrix, single-process
// CPU reference sweep") and the numerical ground truth for GPU tests.
//
// Semantics follow the reference solver API
// (reference main.cu:440-448 omp_mpi_cuda_dgesvd_local_matrices,
// lib/JacobiMethods.cuh:44-62):  column-major A is overwritten by U, s gets
// the (unsorted) singular values, V (not V^T) is n x n column-major.
// Per pair the work is the reference's dot triple (main.cu:698-707), the
// symmetric-Schur rotation (main.cu:712-725) and the Givens column update
// (the reference's only CUDA kernel, main.cu:139-147).
//
// Deliberate fixes over the reference:
//  * real stopping test: sweeps repeat until a sweep applies no rotation
//    (reference runs exactly one sweep, main.cu:482);
//  * relative threshold |a_p.a_q| > tol*||a_p||*||a_q|| by default (the
//    absolute 1e-16 of lib/global.cuh:9 is kept as tol_mode=1 for parity);
//  * the convergence value (main.cu:710) is recorded per sweep, not dropped;
//  * sigma = 0 columns are not divided (main.cu:1405-1421 has no guard);
//  * NoVec does not rotate an uninitialised V.
#include "svdj_cpu.h"

#include <cmath>
#include <cstring>
#include <vector>
#include <algorithm>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

template <typename T>
inline void rotation_params(T alpha, T beta, T gamma, T& c, T& s) {
  // Golub & Van Loan symmetric Schur on [[beta, alpha],[alpha, gamma]]
  // written exactly as the reference (main.cu:715-725) but overflow-safe
  // for huge tau.
  const T tau = (gamma - beta) / (T(2) * alpha);
  T t;
  const T big = sizeof(T) == 8 ? T(1e150) : T(1e18);
  if (std::fabs(tau) > big) {
    t = T(1) / (T(2) * tau);
  } else if (tau >= T(0)) {
    t = T(1) / (tau + std::sqrt(T(1) + tau * tau));
  } else {
    t = T(1) / (tau - std::sqrt(T(1) + tau * tau));
  }
  c = T(1) / std::sqrt(T(1) + t * t);
  s = t * c;
}

// "Ordered" one-sided rotation (Erricos, Handbook of Parallel Computing and
// Statistics p.128; reference lib/Utils.cu:57-80, compiled there but never
// called).  xi = 2 a_p.a_q, beta = ||a_p||^2 - ||a_q||^2 (the reference's
// comment says ||a_q||^2; the difference is what makes the formula orthogonalise),
// gamma = sqrt(xi^2 + beta^2).  Applied as a_p' = c a_p + s a_q,
// a_q' = -s a_p + c a_q it also moves the larger norm into column p, so the
// sweep tends to leave sigma sorted.  Returned in this file's convention
// (x' = c x - s y) i.e. with s negated.
template <typename T>
inline void rotation_params_ordered(T alpha, T np2, T nq2, T& c, T& s) {
  const T xi = T(2) * alpha;
  const T beta = np2 - nq2;
  const T gamma = std::sqrt(xi * xi + beta * beta);
  T so;
  if (beta > T(0)) {
    c = std::sqrt((beta + gamma) / (T(2) * gamma));
    so = xi / (T(2) * gamma * c);
  } else {
    so = std::sqrt((gamma - beta) / (T(2) * gamma));
    c = xi / (T(2) * gamma * so);
  }
  s = -so;
}

template <typename T>
int jacobi_impl(int jobu, int jobv, int m, int n, T* A, int lda, T* s, T* V,
                int ldv, int ordering, int max_sweeps, double tol, int tol_mode,
                double* hist, int num_threads) {
  if (m < 1 || n < 1 || lda < m || A == nullptr) return -1;
  if (m < n) return -2;  // wide matrices: caller transposes (see api.py)
  const bool want_v = (jobv == 0 || jobv == 1) && V != nullptr;
  if ((jobv == 0 || jobv == 1) && ldv < n) return -1;
#ifdef _OPENMP
  if (num_threads > 0) omp_set_num_threads(num_threads);
#endif
  // V := I (reference main.cu:461-474).
  if (want_v) {
    for (int j = 0; j < n; ++j) {
      T* col = V + (long)j * ldv;
      std::fill(col, col + n, T(0));
      col[j] = T(1);
    }
  }
  // ordering: bits 0-3 schedule (0 Sameh, 1 round robin),
  //           bits 4-7 rotation formula (0 symmetric Schur, 1 ordered).
  const int rot_kind = (ordering >> 4) & 0xF;
  ordering &= 0xF;
  // Schedule.
  int steps, per_step;
  std::vector<int32_t> sched;
  if (ordering == 0) {
    steps = svdj_sameh_num_steps(n);
    per_step = n / 2;
    sched.resize((size_t)std::max(steps, 1) * std::max(per_step, 1) * 2);
    svdj_sameh_schedule(n, sched.data());
  } else {
    const int nb = n + (n & 1);
    steps = nb - 1;
    per_step = nb / 2;
    sched.resize((size_t)steps * per_step * 2);
    svdj_round_robin(nb, sched.data());
    for (auto& x : sched)
      if (x >= n) x = -1;  // dummy column for odd n
  }
  int sweeps = 0;
  // One parallel region for the whole solve (a fork/join per step costs more
  // than the step itself for small n); each step is an `omp for` whose
  // implicit barrier orders the steps.
  double maxconv = 0.0;
  long rotations = 0;
  bool done = false;
#pragma omp parallel
  for (int sweep = 0; sweep < max_sweeps && !done; ++sweep) {
#pragma omp single
    {
      maxconv = 0.0;
      rotations = 0;
    }
    for (int st = 0; st < steps; ++st) {
      const int32_t* pr = sched.data() + (size_t)st * per_step * 2;
#pragma omp for schedule(static) reduction(max : maxconv) reduction(+ : rotations)
      for (int k = 0; k < per_step; ++k) {
        const int p = pr[2 * k], q = pr[2 * k + 1];
        if (p < 0 || q < 0) continue;
        T* ap = A + (long)p * lda;
        T* aq = A + (long)q * lda;
        T alpha = 0, beta = 0, gamma = 0;
        for (int i = 0; i < m; ++i) {
          const T x = ap[i], y = aq[i];
          alpha += x * y;
          beta += x * x;
          gamma += y * y;
        }
        const T nrm = std::sqrt(beta) * std::sqrt(gamma);
        if (nrm > T(0)) {
          const double conv = std::fabs((double)alpha) / (double)nrm;
          if (conv > maxconv) maxconv = conv;
        }
        bool rotate;
        if (tol_mode == 1)
          rotate = std::fabs(alpha) > T(tol);
        else
          rotate = nrm > T(0) && std::fabs(alpha) > T(tol) * nrm;
        if (!rotate || alpha == T(0)) continue;
        T c, sn;
        if (rot_kind == 1)
          rotation_params_ordered(alpha, beta, gamma, c, sn);
        else
          rotation_params(alpha, beta, gamma, c, sn);
        ++rotations;
        for (int i = 0; i < m; ++i) {
          const T x = ap[i], y = aq[i];
          ap[i] = c * x - sn * y;
          aq[i] = sn * x + c * y;
        }
        if (want_v) {
          T* vp = V + (long)p * ldv;
          T* vq = V + (long)q * ldv;
          for (int i = 0; i < n; ++i) {
            const T x = vp[i], y = vq[i];
            vp[i] = c * x - sn * y;
            vq[i] = sn * x + c * y;
          }
        }
      }
    }
#pragma omp single
    {
      if (hist) hist[sweep] = maxconv;
      sweeps = sweep + 1;
      if (rotations == 0) done = true;
    }
  }
  // Sigma and U (reference main.cu:1394-1421, with sigma=0 guard).
  const int k = std::min(m, n);
#pragma omp parallel for schedule(static)
  for (int j = 0; j < n; ++j) {
    T* a = A + (long)j * lda;
    double nrm2 = 0.0;
    for (int i = 0; i < m; ++i) nrm2 += (double)a[i] * (double)a[i];
    const T sig = (T)std::sqrt(nrm2);
    if (j < k && s) s[j] = sig;
    if ((jobu == 0 || jobu == 1) && sig > T(0)) {
      const T inv = T(1) / sig;
      for (int i = 0; i < m; ++i) a[i] *= inv;
    }
  }
  return sweeps;
}

}  // namespace

extern "C" int svdj_cpu_jacobi_f64(int jobu, int jobv, int m, int n, double* A,
                                   int lda, double* s, double* V, int ldv,
                                   int ordering, int max_sweeps, double tol,
                                   int tol_mode, double* hist, int num_threads) {
  return jacobi_impl<double>(jobu, jobv, m, n, A, lda, s, V, ldv, ordering,
                             max_sweeps, tol, tol_mode, hist, num_threads);
}

extern "C" int svdj_cpu_jacobi_f32(int jobu, int jobv, int m, int n, float* A,
                                   int lda, float* s, float* V, int ldv,
                                   int ordering, int max_sweeps, double tol,
                                   int tol_mode, double* hist, int num_threads) {
  return jacobi_impl<float>(jobu, jobv, m, n, A, lda, s, V, ldv, ordering,
                            max_sweeps, tol, tol_mode, hist, num_threads);
}

extern "C" double svdj_cpu_residual_f64(int m, int n, int k, const double* A,
                                        int lda, const double* U, int ldu,
                                        const double* s, const double* V,
                                        int ldv, int num_threads) {
#ifdef _OPENMP
  if (num_threads > 0) omp_set_num_threads(num_threads);
#endif
  double total = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : total)
  for (int j = 0; j < n; ++j) {
    std::vector<double> col(A + (long)j * lda, A + (long)j * lda + m);
    for (int l = 0; l < k; ++l) {
      const double coef = s[l] * V[(long)l * ldv + j];  // V(j,l)
      if (coef == 0.0) continue;
      const double* u = U + (long)l * ldu;
      for (int i = 0; i < m; ++i) col[i] -= u[i] * coef;
    }
    for (int i = 0; i < m; ++i) total += col[i] * col[i];
  }
  return std::sqrt(total);
}

extern "C" double svdj_cpu_orth_f64(int m, int k, const double* Q, int ldq,
                                    int num_threads) {
#ifdef _OPENMP
  if (num_threads > 0) omp_set_num_threads(num_threads);
#endif
  double total = 0.0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : total)
  for (int a = 0; a < k; ++a) {
    const double* qa = Q + (long)a * ldq;
    for (int b = a; b < k; ++b) {
      const double* qb = Q + (long)b * ldq;
      double d = 0.0;
      for (int i = 0; i < m; ++i) d += qa[i] * qb[i];
      if (a == b) d -= 1.0;
      total += (a == b ? 1.0 : 2.0) * d * d;
    }
  }
  return std::sqrt(total);
}

extern "C" const char* svdj_cpu_version(void) { return "svdj-cpu 0.1 (host C++/OpenMP)"; }
