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
