// Exported twin of svdj_stop.h's sweep stop test, so the Python executor
// takes exactly the decision the native engines take.
#include "svdj_cpu.h"
#include "svdj_stop.h"

extern "C" int svdj_sweep_converged(double mx, double ms, double nrot_pairs, double nrot_cols,
                                    double tol, int tol_mode, int second_order) {
  return svdj_sweep_converged_inline(mx, ms, nrot_pairs, nrot_cols, tol, tol_mode, second_order);
}
