// Host-side (CPU) native API of the MI355X Jacobi-SVD framework.
//
// Everything here is plain C ABI so it can be bound from Python with ctypes and
// linked from the native C++ driver alike.  No HIP / GPU dependency: this
// library builds and runs on the CPU-only container.
//
// Contents
//   * schedules   - Sameh 1971 parallel ordering (reference parity,
//                   reference main.cu:500-538 / 945-983), round-robin
//                   (circle) tournament, bipartite cross schedule and the
//                   multi-GPU super-block tournament with one-block exchange.
//   * oracle      - scalar one-sided Hestenes Jacobi SVD on the CPU
//                   (reference main.cu:440-1423 semantics, fixed: relative
//                   threshold, real stopping test, sigma=0 guard).
//   * rng         - bit-exact reproduction of the reference input generator
//                   (std::default_random_engine(1000000) + uniform(0,1),
//                   reference main.cu:1558-1567) and a dense variant.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---------------------------------------------------------------- schedules
// Number of parallel steps of the Sameh ordering for n columns
// (n-1 for even n, n for odd n).
int svdj_sameh_num_steps(int n);
// Fill out[steps][n/2][2] with 0-based (p,q) pairs.  Unused slots (odd n never
// leaves any; kept for safety) are -1.  Returns number of steps.
int svdj_sameh_schedule(int n, int32_t* out);

// Round-robin (circle method) 1-factorisation of K_nb, nb even.
// out[nb-1][nb/2][2].  Returns nb-1 or -1 if nb is odd/invalid.
int svdj_round_robin(int nb, int32_t* out);

// Bipartite schedule between two groups of k blocks, X = [0,k), Y = [k,2k):
// step t pairs (a, k + (a+t) mod k).  out[k][k][2].  Returns k.
int svdj_bipartite(int k, int32_t* out);

// Quad orders (two steps fused over the four blocks of a super-block pair
// {a, b} x {c, d}: step s pairs (a, c), (b, d), step s+1 (a, d), (b, c) as
// pairs 2q, 2q+1).  svdj_quad_round_robin: out[nb-1][nb/2][2], nb % 4 == 0,
// step 0 the within-super-block pairs (2i, 2i+1), then a round robin over the
// nb/2 super-blocks, two steps each.  svdj_quad_bipartite: out[h][h][2], the
// cross pairs of block lists xs, ys (h even).  Return the step count or -1.
int svdj_quad_round_robin(int nb, int32_t* out);
int svdj_quad_bipartite(int h, const int32_t* xs, const int32_t* ys, int32_t* out);

// Multi-GPU super-block tournament: 2P super-blocks, 2P-1 rounds, one pair per
// GPU per round; between consecutive rounds every GPU replaces exactly one of
// its two super-blocks (one send + one recv per GPU per round).
//   held[r][g][2]   super-block ids held by GPU g in slot 0/1 during round r
//   xslot[r][g]     (r>=1) slot of GPU g that is replaced before round r
//   send_to[r][g]   (r>=1) GPU that receives the outgoing block of g
//   recv_from[r][g] (r>=1) GPU that sends g its incoming block
// Entries for r=0 of xslot/send_to/recv_from are -1.  Returns 2P-1.
int svdj_tournament(int P, int32_t* held, int32_t* xslot, int32_t* send_to, int32_t* recv_from);

// ------------------------------------------------------------------ oracle
// jobu/jobv: 0 = AllVec, 1 = SomeVec, 2 = NoVec (reference SVD_OPTIONS).
// ordering : bits 0-3: 0 = Sameh (reference), 1 = round-robin;
//            bits 4-7: rotation formula 0 = symmetric Schur (reference
//            main.cu:712-725), 1 = ordered (reference lib/Utils.cu:57-80).
// tol_mode : 0 = relative |a_p.a_q| > tol*||a_p||*||a_q|| (default),
//            1 = absolute |a_p.a_q| > tol (reference TOLERANCE=1e-16).
// Column-major A (m x n, lda) is overwritten by U; s[min(m,n)] gets sigma
// (unsorted, reference layout); V (n x n, ldv) gets V (not V^T).
// offnorm_hist[sweep] = max_{p<q} |a_p.a_q|/(||a_p|| ||a_q||) measured during
// the sweep.  Returns number of sweeps executed (>=1), or <0 on error.
int svdj_cpu_jacobi_f64(int jobu, int jobv, int m, int n, double* A, int lda,
                        double* s, double* V, int ldv, int ordering,
                        int max_sweeps, double tol, int tol_mode,
                        double* offnorm_hist, int num_threads);
int svdj_cpu_jacobi_f32(int jobu, int jobv, int m, int n, float* A, int lda,
                        float* s, float* V, int ldv, int ordering,
                        int max_sweeps, double tol, int tol_mode,
                        double* offnorm_hist, int num_threads);

// ---------------------------------------------------------------------- rng
// Reference input: upper-triangular R with U(0,1) entries from
// std::default_random_engine(seed), filled row by row (j >= i) into
// column-major A (m x n, lda).  Other entries are left untouched.
void svdj_ref_triu_input(int m, int n, double* A, int lda, uint32_t seed);
// Dense variant (reference '#ifdef TESTS' intent, fixed): row by row all j.
void svdj_ref_dense_input(int m, int n, double* A, int lda, uint32_t seed);
// First `count` raw draws of uniform_real_distribution<double>(0,1) with
// default_random_engine(seed) -- used by tests to pin bit parity.
void svdj_ref_uniform_stream(uint32_t seed, int count, double* out);
// Columns [c0, c0 + nc) of the triangular (dense = 0) / dense (dense = 1)
// input into out (ld >= m), without storing the rest of the matrix.
void svdj_ref_input_cols(int m, int n, int dense, uint32_t seed, int c0, int nc, double* out, int ld);

// --------------------------------------------------------------- verification
// ||A - U diag(s) V^T||_F for column-major inputs (blocked, OpenMP).
double svdj_cpu_residual_f64(int m, int n, int k, const double* A, int lda,
                             const double* U, int ldu, const double* s,
                             const double* V, int ldv, int num_threads);
// ||Q^T Q - I||_F for column-major Q (m x k).
double svdj_cpu_orth_f64(int m, int k, const double* Q, int ldq, int num_threads);

// ------------------------------------------------------------------ stop test
// Block-path sweep stop test (svdj_stop.h): 0 = continue, 1 = the sweep
// rotated nothing, 2 = the second-order rule (relative mode,
// second_order != 0).  mx, ms, nrot_pairs, nrot_cols: the sweep's global
// largest coupling, largest effective sine of an applied rotation, rotated
// block pairs and applied column rotations.
int svdj_sweep_converged(double mx, double ms, double nrot_pairs, double nrot_cols, double tol,
                         int tol_mode, int second_order);

const char* svdj_cpu_version(void);

#ifdef __cplusplus
}
#endif
