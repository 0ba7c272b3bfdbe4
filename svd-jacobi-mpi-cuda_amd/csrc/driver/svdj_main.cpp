// Native single-GPU driver: the reference's `SVD_Jacobi_MPI_CUDA <n>` binary
// (reference main.cu:1426-1676) rebuilt on the framework's C ABI, with no
// Python in the loop.  Multi-GPU runs use the Python/RCCL launcher
// (tools/svd_jacobi.py under torchrun) -- one process per GPU.
//
//   svdj_main N [--m M] [--input triu|dense] [--seed S] [--dtype f32|f64]
//               [--method block|scalar] [--engine pipeline|steps]
//               [--block W (default: by size)] [--max-sweeps K]
//               [--tol T] [--mma auto|native|bf16x6|bf16x3] [--inner cyclic|bipartite]
//               [--verify] [--report-dir DIR]
//
// The block method's default engine ("pipeline") is libsvdj_dist's plan at
// world 1 -- the same engine as bench.py and svdj.svd(): two step chains,
// quad steps and the merged one-GPU issue where they pay -- with no RCCL
// communicator (svdj_dist_solve makes no RCCL call on one GPU).  "steps" is
// the single-stream round robin of svdj_block_solve.
//
// Prints the reference's lines ("Dimensions, height: .., width: ..",
// "SVD MPI+OMP time with U,V calculation: ..", "||A-USVt||_F: ..") and writes
// reporte-dimension-<n>-time-<ts>.txt.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "svdj_cpu.h"
#include "svdj_dist.h"
#include "svdj_hip.h"

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_),      \
                   __FILE__, __LINE__);                                           \
      std::exit(2);                                                               \
    }                                                                             \
  } while (0)

static int rup(int a, int b) { return (a + b - 1) / b * b; }

template <typename T>
static int run(int m, int n, const std::vector<double>& A0, const std::string& method,
               const std::string& engine, int W, int max_sweeps, double tol, int mma,
               int inner_order, bool verify, const std::string& report_dir) {
  const int dtype = sizeof(T) == 8 ? 1 : 0;
  const bool block = method == "block";
  const bool pipe = block && engine == "pipeline";
  int ncols = block ? std::max(rup(n, 2 * W), 2 * W) : n;
  int m_pad = rup(std::max(m, 1), SVDJ_ROW_ALIGN);
  int n_v = rup(ncols, SVDJ_ROW_ALIGN);
  int B = 0;
  int32_t held[2] = {0, 1};
  if (pipe) {  // 2 super-blocks of B columns (even number of W-blocks each), rows padded
    if (svdj_dist_geometry(1, m, n, W, dtype, &B, &ncols, &m_pad, &n_v) < 0 ||
        svdj_dist_initial_held(1, 0, held) < 0) {
      std::fprintf(stderr, "svdj error: %s\n", svdj_dist_last_error());
      return 3;
    }
  }
  // column j in row j of At; the pipeline's slot s holds super-block held[s]
  auto row_of = [&](int j) { return pipe ? (held[0] == j / B ? 0 : 1) * B + j % B : j; };
  std::vector<T> hA((size_t)ncols * m_pad, T(0));
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) hA[(size_t)row_of(j) * m_pad + i] = (T)A0[(size_t)j * m + i];
  T *dA, *dV, *dD, *dS;
  uint32_t* dmetric;
  CHECK(hipMalloc(&dA, hA.size() * sizeof(T)));
  CHECK(hipMalloc(&dV, (size_t)ncols * n_v * sizeof(T)));
  CHECK(hipMalloc(&dD, (size_t)ncols * sizeof(T)));
  CHECK(hipMalloc(&dS, (size_t)ncols * sizeof(T)));
  CHECK(hipMalloc(&dmetric, SVDJ_METRIC_WORDS * sizeof(uint32_t)));
  CHECK(hipMemcpy(dA, hA.data(), hA.size() * sizeof(T), hipMemcpyHostToDevice));
  hipStream_t st, sb;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  std::vector<double> hist(max_sweeps, 0.0);
  // sqrt(m) eps (LAPACK xGESVJ), as utils/metrics.py default_tol
  if (tol <= 0) tol = std::sqrt((double)m) * (sizeof(T) == 8 ? 2.220446049250313e-16 : 1.1920929e-07);

  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, st));
  int sweeps = 0;
  void* ws = nullptr;
  int32_t* dsched = nullptr;
  if (pipe) {
    svdj_dist_problem p{};
    p.rank = 0;
    p.world = 1;
    p.comm = nullptr;
    p.dtype = dtype;
    p.W = W;
    p.m_pad = m_pad;
    p.n_v = n_v;
    p.B = B;
    p.At = dA;
    p.Vt = dV;
    p.D = dD;
    p.held[0] = held[0];
    p.held[1] = held[1];
    p.tol = tol;
    p.tol_mode = 0;  // relative
    p.max_sweeps = max_sweeps;
    p.mma = mma;
    p.inner_order = inner_order;
    p.exchange = 0;
    p.stop_rule = 1;  // second order
    p.quad = 0;       // auto
    p.stream_a = st;
    p.stream_b = sb;
    p.hist = hist.data();
    p.fault_rank = p.fault_sweep = -1;
    for (int s = 0; s < 2; ++s)
      if (svdj_set_identity(dtype, dV + (size_t)s * B * n_v, n_v, n_v, B, held[s] * B, st) < 0) goto fail;
    if (svdj_col_norms2(dtype, dA, m_pad, m_pad, ncols, dD, st) < 0) goto fail;
    if (svdj_dist_solve(&p, dS) < 0) {
      std::fprintf(stderr, "svdj error: %s\n", svdj_dist_last_error());
      return 3;
    }
    sweeps = p.sweeps;
    held[0] = p.held[0];
    held[1] = p.held[1];
    std::printf("engine: pipeline (%s%s)\n", p.merged_used ? "merged chains" : "two chains",
                p.quad_used ? ", quad steps" : "");
  } else if (svdj_set_identity(dtype, dV, n_v, n_v, ncols, 0, st) < 0) {
    goto fail;
  }
  if (pipe) {
  } else if (block) {
    const size_t wsb = svdj_block_workspace_bytes(dtype, W, ncols / W / 2, m_pad, 0);
    CHECK(hipMalloc(&ws, wsb));
    if (svdj_col_norms2(dtype, dA, m_pad, m_pad, ncols, dD, st) < 0) goto fail;
    sweeps = svdj_block_solve(dtype, W, m_pad, dA, m_pad, dV, n_v, n_v, dD, ncols, tol,
                              /*tol_mode relative*/ 0, 1, max_sweeps, inner_order, ws, wsb,
                              dmetric, hist.data(), mma, /*stop_rule second_order*/ 1, st);
  } else {
    const int steps = svdj_sameh_num_steps(n);
    std::vector<int32_t> sched((size_t)steps * (n / 2) * 2);
    svdj_sameh_schedule(n, sched.data());
    CHECK(hipMalloc(&dsched, sched.size() * sizeof(int32_t)));
    CHECK(hipMemcpy(dsched, sched.data(), sched.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    sweeps = svdj_scalar_solve(dtype, m_pad, dA, m_pad, dV, n_v, n_v, dsched, steps, n / 2, tol,
                               0, max_sweeps, dmetric, hist.data(), st);
  }
  if (sweeps < 0) goto fail;
  if (!pipe && svdj_finalize(dtype, dA, m_pad, m_pad, ncols, dS, 1, st) < 0) goto fail;
  CHECK(hipEventRecord(e1, st));
  CHECK(hipEventSynchronize(e1));
  {
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double secs = ms / 1e3;
    std::printf("SVD MPI+OMP time with U,V calculation: %.6f\n", secs);
    std::printf("sweeps: %d  last off value: %.3e  tol: %.3e\n", sweeps,
                sweeps > 0 ? hist[sweeps - 1] : 0.0, tol);
    const double flops = (double)n * (n - 1) / 2.0 * (12.0 * m + 6.0 * n) * sweeps;
    std::printf("GFLOP/s (algorithmic): %.1f\n", flops / secs / 1e9);
    double resid = -1.0;
    if (verify) {
      std::vector<T> hU((size_t)ncols * m_pad), hV((size_t)ncols * n_v), hS(ncols);
      CHECK(hipMemcpy(hU.data(), dA, hU.size() * sizeof(T), hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(hV.data(), dV, hV.size() * sizeof(T), hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(hS.data(), dS, hS.size() * sizeof(T), hipMemcpyDeviceToHost));
      std::vector<double> U((size_t)n * m), V((size_t)n * n), S(n);
      for (int j = 0; j < n; ++j) {
        const size_t r = (size_t)row_of(j);  // final placement (held)
        S[j] = hS[r];
        for (int i = 0; i < m; ++i) U[(size_t)j * m + i] = hU[r * m_pad + i];
        for (int i = 0; i < n; ++i) V[(size_t)j * n + i] = hV[r * n_v + i];
      }
      resid = svdj_cpu_residual_f64(m, n, n, A0.data(), m, U.data(), m, S.data(), V.data(), n, 0);
      const double ou = svdj_cpu_orth_f64(m, n, U.data(), m, 0);
      const double ov = svdj_cpu_orth_f64(n, n, V.data(), n, 0);
      std::printf("||A-USVt||_F: %.6e\n||U^TU-I||_F: %.3e\n||V^TV-I||_F: %.3e\n", resid, ou, ov);
    }
    if (!report_dir.empty()) {
      char ts[64];
      std::time_t t = std::time(nullptr);
      std::strftime(ts, sizeof(ts), "%d-%m-%Y-%H-%M-%S", std::localtime(&t));
      std::string path = report_dir + "/reporte-dimension-" + std::to_string(m) + "-time-" + ts + ".txt";
      if (FILE* f = std::fopen(path.c_str(), "w")) {
        std::fprintf(f, "Number of threads: 1\nDimensions, height: %d, width: %d\n", m, n);
        std::fprintf(f, "SVD MPI+OMP time with U,V calculation: %.6f\n", secs);
        if (resid >= 0) std::fprintf(f, "||A-USVt||_F: %.6e\n", resid);
        std::fclose(f);
        std::printf("report: %s\n", path.c_str());
      }
    }
  }
  (void)hipFree(dA); (void)hipFree(dV); (void)hipFree(dD); (void)hipFree(dS);
  (void)hipFree(dmetric); (void)hipFree(ws); (void)hipFree(dsched);
  return 0;
fail:
  std::fprintf(stderr, "svdj error: %s\n", svdj_hip_last_error());
  return 3;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s N [--m M] [--input triu|dense] [--dtype f32|f64] ...\n", argv[0]);
    return 1;
  }
  int n = std::atoi(argv[1]), m = n, W = 0, max_sweeps = 60, inner_order = 3;  // auto
  unsigned seed = 1000000;
  double tol = -1;
  bool verify = false;
  std::string input = "triu", dtype = "f64", method = "block", engine = "pipeline",
              report_dir = ".", mma = "auto";
  for (int i = 2; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--m") m = std::atoi(next());
    else if (a == "--input") input = next();
    else if (a == "--seed") seed = (unsigned)std::strtoul(next(), nullptr, 10);
    else if (a == "--dtype") dtype = next();
    else if (a == "--method") method = next();
    else if (a == "--engine") engine = next();
    else if (a == "--block") W = std::atoi(next());
    else if (a == "--max-sweeps") max_sweeps = std::atoi(next());
    else if (a == "--tol") tol = std::atof(next());
    else if (a == "--mma") mma = next();
    else if (a == "--inner") {
      const std::string v = next();
      inner_order = v == "auto" ? 3 : (v == "cross" ? 2 : (v == "bipartite" ? 1 : 0));
    }
    else if (a == "--verify") verify = true;
    else if (a == "--report-dir") report_dir = next();
    else if (a == "--no-report") report_dir.clear();
  }
  if (m < n) {
    std::fprintf(stderr, "m >= n required\n");
    return 1;
  }
  std::printf("%s\n", svdj_hip_version());
  std::printf("Dimensions, height: %d, width: %d\n", m, n);
  std::vector<double> A((size_t)m * n, 0.0);
  if (input == "dense")
    svdj_ref_dense_input(m, n, A.data(), m, seed);
  else
    svdj_ref_triu_input(m, n, A.data(), m, seed);
  if (W == 0)  // models/block.py choose_block
    W = dtype == "f32" ? (n >= 1024 ? 64 : 32) : ((m >= 6144 && n >= 2048) ? 64 : 32);
  const int mma_code = mma == "auto" ? svdj_choose_mma(dtype == "f32" ? 0 : 1, W)
                                     : (mma == "bf16x6" ? 1 : (mma == "bf16x3" ? 2 : 0));
  if (engine != "pipeline" && engine != "steps") {
    std::fprintf(stderr, "--engine pipeline|steps\n");
    return 1;
  }
  if (dtype == "f32")
    return run<float>(m, n, A, method, engine, W, max_sweeps, tol, mma_code, inner_order, verify,
                      report_dir);
  return run<double>(m, n, A, method, engine, W, max_sweeps, tol, 0, inner_order, verify, report_dir);
}
