// Device-side (MI355X / gfx950) native API of the Jacobi-SVD framework.
//
// Plain C ABI over raw device pointers + a hipStream_t passed as void*, so the
// library has no PyTorch dependency: Python binds it with ctypes and passes
// tensor.data_ptr() / torch.cuda.current_stream().cuda_stream; the native C++
// driver links it directly.
//
// Storage convention (all entry points): a column-major matrix with leading
// dimension ld is addressed as column c at base + c*ld.  Row counts passed to
// kernels are PADDED row counts (multiple of SVDJ_ROW_ALIGN, pad rows zero),
// so no kernel needs a row bounds check.
//
// dtype codes: 0 = fp32, 1 = fp64.
#pragma once
#include <stddef.h>
#include <stdint.h>

#define SVDJ_ROW_ALIGN 128
#include "svdj_stop.h"

#ifdef __cplusplus
extern "C" {
#endif

// Returns a static version/feature string ("gfx950 ...").
const char* svdj_hip_version(void);
// Last error message recorded by this library (thread-local), "" if none.
const char* svdj_hip_last_error(void);

// ---------------------------------------------------------------------------
// Scalar (column-pair) path: one fused kernel per parallel step, one
// workgroup per pair (wave64 reductions of the reference's dot triple,
// rotation solved in registers, Givens update of A and V in place).
//   sched     device int32 [steps][per_step][2] (pairs < 0 are skipped)
//   tol_mode  0 relative, 1 absolute
//   metric    device uint32[2]: [0] = max convergence value (float bits),
//             [1] = number of rotations applied.  Accumulated (not reset).
int svdj_scalar_step(int dtype, int m_pad, void* A, int lda, void* V, int n_v,
                     int ldv, const int32_t* sched, int per_step, double tol,
                     int tol_mode, uint32_t* metric, void* stream);

// Full solve on one GPU: repeats sweeps over `steps` until a sweep applies
// no rotation or max_sweeps is reached.  hist (host, may be NULL) receives
// the per-sweep max convergence value.  Returns sweeps executed, <0 on error.
int svdj_scalar_solve(int dtype, int m_pad, void* A, int lda, void* V, int n_v,
                      int ldv, const int32_t* sched, int steps, int per_step,
                      double tol, int tol_mode, int max_sweeps, uint32_t* metric,
                      double* hist, void* stream);

// ---------------------------------------------------------------------------
// Block path (one-sided block Jacobi, MFMA).  Columns are grouped in blocks
// of W (32 or 64; fp64 supports 32).  One step processes P disjoint block
// pairs (bi, bj):
//   1. Gram (MFMA, split over rows):  mode 0 (cross) C = A_bi^T A_bj,
//                                     mode 1 (full)  G = [A_bi A_bj]^T[..]
//   2. EVD of the 2W x 2W Gram (cyclic parallel Jacobi in LDS), in cross
//      mode with the diagonal blocks taken from the tracked squared column
//      norms D (blocks are kept internally orthogonal);  Q -> workspace.
//   3. Apply (MFMA):  [A_bi A_bj] <- [A_bi A_bj] Q ,  [V_bi V_bj] <- .. Q
// D (device, dtype, [ncols]) holds squared column norms; updated in place.
//   pairs   device int32 [steps][P][2] block indices
//   modes   host   int32 [steps] (0 cross / 1 full / 2 cross with the bipartite
//           EVD ordering, W steps instead of 2W-1 / 3 cross with the
//           cross-only bipartite EVD), NULL = all cross
//   metric  device uint32[SVDJ_METRIC_WORDS] (svdj_stop.h): [0] max
//           convergence value (float bits), [1] rotated pairs, [2..3] the
//           underflow floor (double, svdj_set_norm_floor; 0 = off), [4] the
//           largest |sin| of an applied rotation (float bits).
//   tol_mode 0: rotate when |g_pq| > tol sqrt(g_pp g_qq) (relative, default);
//            1: when |g_pq| > tol (the reference's absolute TOLERANCE test).
//   mma     matrix-core mode: 0 native (f32 / f64 MFMA), 1 fp32 data on bf16
//           MFMA with a 3-way bf16 split (6 products, fp32-level accuracy),
//           2 fp32 data on bf16 MFMA with a 2-way split (3 products, ~2^-17).
//           Both split modes apply Y = X + X (Q - I), the identity in fp32.
//           Bit 8 (| 256): the quad Gram of quad steps with 2 bf16 parts (3
//           products, couplings to ~2^-17) -- for sweeps far from convergence,
//           where it only steers the rotation angles.
// Workspace size for steps of P pairs: svdj_block_workspace_bytes(); quad != 0
// when the step list holds quad steps (modes 4/5: fp32, W = 64).
size_t svdj_block_workspace_bytes(int dtype, int W, int P, int m_pad, int quad);
// inner_order code (1 bipartite, 2 cross-only) for steps of `pairs` pairs of
// W-wide blocks of data type `dtype` (0 fp32, 1 fp64): models/block.py
// choose_inner_order.
int svdj_choose_inner_order(int dtype, int W, int pairs);
// Default ("auto") matrix-core mode for dtype (0 fp32, 1 fp64) and block width
// W: 1 (split bf16) for fp32 W = 64, else 0 (models/block.py choose_mma).
int svdj_choose_mma(int dtype, int W);
int svdj_block_steps(int dtype, int W, int m_pad, void* A, int lda, void* V,
                     int n_v, int ldv, void* D, const int32_t* pairs, int P,
                     int steps, const int32_t* modes, double tol, int tol_mode,
                     int max_inner_sweeps, void* workspace, size_t ws_bytes,
                     uint32_t* metric, int mma, void* stream);

// Single-GPU block solve: round-robin over nb = ncols/W blocks (nb even),
// first step of every sweep in full mode; inner_order 0 = cyclic EVD in every
// step, 1 = bipartite EVD in the cross steps (mode 2), 2 = cross-only
// bipartite EVD (mode 3).  stop_rule 1: a sweep also ends the iteration by
// the second-order rule of svdj_stop.h (relative mode), 0: only a sweep
// without rotations does.  Returns sweeps, <0 on error.
int svdj_block_solve(int dtype, int W, int m_pad, void* A, int lda, void* V,
                     int n_v, int ldv, void* D, int ncols, double tol, int tol_mode,
                     int max_inner_sweeps, int max_sweeps, int inner_order, void* workspace,
                     size_t ws_bytes, uint32_t* metric, double* hist,
                     int mma, int stop_rule, void* stream);
// Zero the per-sweep words of a block-path metric ([0], [1], [4..7]); the
// floor ([2..3]) stays.
int svdj_reset_metric(uint32_t* metric, void* stream);

// Diagnostic hooks.  Cross Gram slabs (P x nchunk x W x W) of A_bi^T A_bj
// for a device pair list with the given row chunking (fp32).
int svdj_gram_cross(int dtype, int W, const void* A, int lda, int m_pad,
                    const int32_t* pairs, int P, int rows_per_chunk, void* slabs, void* stream);
// The six cross Grams of a quad step (fp32, W = 64; pairs in quad order,
// P even): slabs (3P x nchunk x W x W) = the P pairs' Grams, then C_ad, C_bc,
// C_ab, C_cd of every quad.  parts: 3 (exact to 2^-26) or 2 (2^-16, the
// early-sweep Gram of svdj_block_steps' mma bit 8).
int svdj_gram_quad(const void* A, int lda, int m_pad, const int32_t* pairs, int P,
                   int rows_per_chunk, void* slabs, int parts, void* stream);
// X <- X Q for one pair of column blocks (X = 2W columns, leading dimension
// ld, `rows` a multiple of SVDJ_ROW_ALIGN), Q row-major 2W x 2W on the
// device, with matrix-core mode `mma` (as svdj_block_steps).
int svdj_apply_q(int dtype, int W, int mma, void* X, int rows, int ld, const void* Q, void* stream);

// ---------------------------------------------------------------------------
// Post-processing / utilities.
// V := I on an (n_v x ncols) column-major block (rows >= ncols zeroed).
int svdj_set_identity(int dtype, void* V, int n_v, int ldv, int ncols, int col_offset, void* stream);
// Squared column norms D[c] = sum_i A[i,c]^2 (fp64 accumulation).
int svdj_col_norms2(int dtype, const void* A, int m_pad, int lda, int ncols, void* D, void* stream);
// The block EVDs' underflow floor (relative mode: pairs with a squared norm
// <= it are not rotated): svdj_norm_floor_value = m realmin / eps of the
// data type; svdj_set_norm_floor stores it at metric[2..3] (metric holds 4
// uint32), once per solve.
double svdj_norm_floor_value(int dtype, int m);
int svdj_set_norm_floor(double floor, uint32_t* metric, void* stream);
// Scale-relative floor max(m realmin, m realmin / eps * max D) from the n squared
// column norms D (device, data type) into metric[2..3].
int svdj_set_norm_floor_scaled(int dtype, int m, const void* D, int n, uint32_t* metric,
                               void* stream);
// sigma[c] = ||a_c||; if scale_u, a_c /= sigma[c] (sigma == 0 columns untouched).
int svdj_finalize(int dtype, void* A, int m_pad, int lda, int ncols, void* sigma, int scale_u, void* stream);

// Device-side timed wait of `ns` nanoseconds on `stream` (one lane polling
// the constant 100 MHz clock); used to model link time in simulations.
int svdj_spin_ns(double ns, void* stream);

#ifdef __cplusplus
}
#endif
