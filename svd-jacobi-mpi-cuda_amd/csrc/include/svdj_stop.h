// Sweep stop test of the block path, shared by every engine (the HIP
// library's svdj_block_solve, the native distributed engine and -- through
// libsvdj_cpu's svdj_sweep_converged -- the Python executor).
//
// The reference computes a convergence value per pair and discards it
// (reference main.cu:710); it runs exactly one sweep (main.cu:482).  Here a
// sweep ends the iteration when
//   (a) it rotated nothing (every coupling it met was at most tol), or
//   (b) relative mode only, the "second-order" rule: all the rotations it
//       applied were noise.  Rotating columns (p, r) by an angle with sine s
//       adds s a_r to a_p (and s a_p to a_r), which moves the relative
//       coupling of p with any q by at most |s| sqrt(d_r / d_p) |c_rq|, d the
//       squared norms.  With ms the largest such effective sine
//       |s| max(sqrt(d_r/d_p), sqrt(d_p/d_r)) of an applied rotation, mx the
//       largest coupling met and R the number of column rotations applied in
//       the sweep, every coupling is, to first order, at most
//         tol + R mx ms
//       when the sweep ends (a coupling was at most tol, or rotated to zero,
//       when its pair was last processed; afterwards only the R rotations
//       can move it).  (b) holds when R mx ms <= tol / 2: the sweep that
//       would follow finds nothing above 1.5 tol, i.e. only rounding noise
//       (tol = sqrt(m) eps is the noise level of the couplings).  LAPACK
//       xGESVJ stops on the same kind of product (largest coupling x largest
//       sine, with the factor n instead of the rotation count).
// The metric words a sweep accumulates on the device (uint32 each):
//   [0] mx (float bits), [1] rotated block pairs, [2..3] the negligible-column
//   floor (double, set once per solve), [4] ms (float bits), [5] R, and two
//   work counters of the quad apply (not part of the stop test): [6] MFMAs
//   issued / 24 (one 32x32x16 bf16 MFMA = 32768 flops), [7] 32-row tiles of
//   256 columns moved (read and written once each).
#pragma once

#define SVDJ_METRIC_WORDS 8

#ifdef __cplusplus
extern "C" {
#endif

// 0 = continue, 1 = the sweep rotated nothing, 2 = the second-order rule.
static inline int svdj_sweep_converged_inline(double mx, double ms, double nrot_pairs,
                                              double nrot_cols, double tol, int tol_mode,
                                              int second_order) {
  if (nrot_pairs <= 0) return 1;
  if (!second_order || tol_mode != 0 || !(tol > 0) || !(nrot_cols > 0)) return 0;
  return nrot_cols * mx * ms <= 0.5 * tol ? 2 : 0;
}

#ifdef __cplusplus
}
#endif
