// Reference input generator, bit-exact.
//
// The reference fills an upper-triangular R with U(0,1) draws from
// std::default_random_engine(1000000) (libstdc++: minstd_rand0) row by row,
// j >= i, into column-major storage (reference main.cu:1445, 1558-1567).
// Using the same libstdc++ engine + distribution here reproduces the stream
// bit for bit.  The dense variant is what the
// reference's broken '#ifdef TESTS' block (main.cu:1569-1579) intended.
#include "svdj_cpu.h"

#include <random>

extern "C" void svdj_ref_triu_input(int m, int n, double* A, int lda, uint32_t seed) {
  std::default_random_engine e(seed);
  std::uniform_real_distribution<double> unif(0.0, 1.0);
  const int k = m < n ? m : n;
  for (int i = 0; i < k; ++i)
    for (int j = i; j < k; ++j) A[(long)j * lda + i] = unif(e);
}

extern "C" void svdj_ref_dense_input(int m, int n, double* A, int lda, uint32_t seed) {
  std::default_random_engine e(seed);
  std::uniform_real_distribution<double> unif(0.0, 1.0);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < n; ++j) A[(long)j * lda + i] = unif(e);
}

extern "C" void svdj_ref_uniform_stream(uint32_t seed, int count, double* out) {
  std::default_random_engine e(seed);
  std::uniform_real_distribution<double> unif(0.0, 1.0);
  for (int i = 0; i < count; ++i) out[i] = unif(e);
}

// Columns [c0, c0 + nc) of the triangular (dense = 0) or dense (dense = 1)
// reference input, out[(j - c0) * ld + i]: the full stream is drawn (the
// engine cannot seek) but only these columns are stored, so a rank of the
// distributed driver keeps O(m nc) host memory instead of the whole matrix.
extern "C" void svdj_ref_input_cols(int m, int n, int dense, uint32_t seed, int c0, int nc,
                                    double* out, int ld) {
  std::default_random_engine e(seed);
  std::uniform_real_distribution<double> unif(0.0, 1.0);
  const int c1 = c0 + nc;
  for (int j = 0; j < nc; ++j)
    for (int i = 0; i < m; ++i) out[(long)j * ld + i] = 0.0;
  if (dense) {
    for (int i = 0; i < m; ++i)
      for (int j = 0; j < n; ++j) {
        const double v = unif(e);
        if (j >= c0 && j < c1) out[(long)(j - c0) * ld + i] = v;
      }
    return;
  }
  const int k = m < n ? m : n;
  for (int i = 0; i < k; ++i)
    for (int j = i; j < k; ++j) {
      const double v = unif(e);
      if (j >= c0 && j < c1) out[(long)(j - c0) * ld + i] = v;
    }
}
