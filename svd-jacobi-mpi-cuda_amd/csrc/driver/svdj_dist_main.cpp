// Native multi-GPU driver: the reference's MPI binary (`mpirun -np P
// SVD_Jacobi_MPI_CUDA <n>`, reference main.cu:1426-1676 and
// build/runSVDMPICUDAWithoutCMake.slurm) rebuilt on RCCL, one process per GPU,
// with no Python and no MPI.
//
//   svdj_dist_main N --np P [--m M] [--input triu|dense] [--seed S]
//                  [--dtype f32|f64] [--block W (default: per-GPU size)] [--max-sweeps K] [--tol T]
//                  [--abs-tol] [--mma auto|native|bf16x6|bf16x3] [--inner auto|cyclic|bipartite|cross]
//                  [--exchange auto|direct|spread] [--stop-rule second_order|no_rotation]
//                  [--quad auto|on|off] [--no-v]
//                  [--shared-gpu] [--verify] [--warmup K] [--timeout SEC]
//                  [--id-file PATH] [--comm-timing] [--progress] [--inject-fault RANK:SWEEP] [--keep-going]
//
// The launcher forks P ranks before anything touches the GPU (the parent never
// does) and waits for them; a rank that fails or a job that exceeds --timeout
// ends every rank.  Launched by an external one-process-per-GPU launcher
// instead (RANK / WORLD_SIZE / LOCAL_RANK in the environment, no --np), the
// process runs its own rank only and the ranks meet through --id-file (or
// SVDJ_DIST_ID), which must name a path all ranks see.
//
// Rank g selects GPU LOCAL_RANK (or g); --shared-gpu puts every rank on GPU 0
// and gives each its own NCCL_HOSTID so RCCL accepts several ranks on one
// device (transport: sockets on loopback, for rehearsal on a one-GPU box).
// Every rank draws the reference input stream (svdj_ref_input_cols) and
// stores only the columns of the two super-blocks the tournament starts it
// with; rank 0 prints the reference's lines and, with --verify, also keeps
// the whole A, gathers U, S, V and checks ||A - U S V^T||_F and
// orthogonality in fp64 on the host.
//
// Failure handling: every solve runs under the library's watchdog (an RCCL
// async error, or no sweep finished within --timeout seconds, aborts the
// communicator and the rank exits 3).  --inject-fault R:S makes rank R exit
// abruptly after sweep S; with --keep-going the launcher does not stop the
// other ranks on a failure, so the survivors' own detection is what ends them.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "svdj_cpu.h"
#include "svdj_dist.h"
#include "svdj_hip.h"

namespace {

struct Opts {
  int n = 0, m = 0, np = 0, W = 0, max_sweeps = 60, mma = 0, warmup = 0, inner = 3;  // auto
  int exchange = 0;  // auto
  int stop_rule = 1;  // second_order (svdj_stop.h)
  int quad = 0;       // auto
  int fault_rank = -1, fault_sweep = -1;
  unsigned seed = 1000000;
  double tol = -1, timeout = 600;
  bool dense = false, f32 = false, abs_tol = false, want_v = true, shared = false, verify = false;
  bool comm_timing = false, keep_going = false, progress = false;
  std::string id_file;
};

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "[rank %d] HIP error %s at %s:%d\n", rank, hipGetErrorString(e_), \
                   __FILE__, __LINE__);                                                    \
      return 2;                                                                            \
    }                                                                                      \
  } while (0)
#define NK(x)                                                                                \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) {                                                                 \
      std::fprintf(stderr, "[rank %d] RCCL error %s at %s:%d\n", rank, ncclGetErrorString(r_), \
                   __FILE__, __LINE__);                                                      \
      return 2;                                                                              \
    }                                                                                        \
  } while (0)

template <typename T>
int run_rank(const Opts& o, int rank, int world, int device) {
  const int dtype = sizeof(T) == 8 ? 1 : 0;
  const ncclDataType_t nt = dtype ? ncclFloat64 : ncclFloat32;
  CK(hipSetDevice(device));
  // The chain and exchange streams are created first: HIP maps streams onto
  // GPU_MAX_HW_QUEUES hardware queues as they are created, and streams made
  // after RCCL's internal ones were seen to share one queue (the chains then
  // serialise: rocprofv3 queue ids, profiles/r2_native_dist).
  hipStream_t sa, sb, sc;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
  void* comm = nullptr;
  if (svdj_dist_comm_init(rank, world, o.id_file.c_str(), o.timeout, &comm) < 0) {
    std::fprintf(stderr, "[rank %d] %s\n", rank, svdj_dist_last_error());
    return 2;
  }
  ncclComm_t nc = (ncclComm_t)comm;
  const int m = o.m, n = o.n;
  const int W = o.W ? o.W : svdj_dist_choose_block(dtype, world, m, n);
  int B, ncols, m_pad, n_v;
  if (svdj_dist_geometry(world, m, n, W, dtype, &B, &ncols, &m_pad, &n_v) < 0) {
    std::fprintf(stderr, "[rank %d] %s\n", rank, svdj_dist_last_error());
    return 1;
  }
  int32_t held[2];
  svdj_dist_initial_held(world, rank, held);
  const int ncs = svdj_dist_storage_cols(world, B);  // 2B (+ B of receive spares)

  // reference input: every rank draws the same stream and stores only its
  // two super-blocks (rank 0 with --verify also the whole A)
  std::vector<double> A;
  if (rank == 0 && o.verify) {
    A.assign((size_t)m * n, 0.0);
    if (o.dense)
      svdj_ref_dense_input(m, n, A.data(), m, o.seed);
    else
      svdj_ref_triu_input(m, n, A.data(), m, o.seed);
  }
  std::vector<T> hA((size_t)2 * B * m_pad, T(0));
  {
    std::vector<double> cols;
    for (int s = 0; s < 2; ++s) {
      const int c0 = held[s] * B, nc = std::min(B, n - c0);
      if (nc <= 0) continue;
      cols.assign((size_t)nc * m, 0.0);
      svdj_ref_input_cols(m, n, o.dense ? 1 : 0, o.seed, c0, nc, cols.data(), m);
      for (int c = 0; c < nc; ++c)
        for (int i = 0; i < m; ++i) hA[(size_t)(s * B + c) * m_pad + i] = (T)cols[(size_t)c * m + i];
    }
  }

  T *dA, *dV = nullptr, *dD, *dS;
  double* dt;
  CK(hipMalloc((void**)&dA, (size_t)ncs * m_pad * sizeof(T)));
  if (o.want_v) CK(hipMalloc((void**)&dV, (size_t)ncs * n_v * sizeof(T)));
  CK(hipMalloc((void**)&dD, (size_t)ncs * sizeof(T)));
  CK(hipMalloc((void**)&dS, (size_t)2 * B * sizeof(T)));
  CK(hipMalloc((void**)&dt, sizeof(double)));
  double tol = o.tol;
  if (tol <= 0)  // sqrt(m) eps (LAPACK xGESVJ), as utils/metrics.py default_tol
    tol = std::sqrt((double)m) * (dtype ? 2.220446049250313e-16 : 1.1920929e-07);
  std::vector<double> hist(o.max_sweeps, 0.0);
  svdj_dist_problem p{};
  p.rank = rank;
  p.world = world;
  p.comm = comm;
  p.dtype = dtype;
  p.W = W;
  p.m_pad = m_pad;
  p.n_v = n_v;
  p.B = B;
  p.At = dA;
  p.Vt = dV;
  p.D = dD;
  p.tol = tol;
  p.tol_mode = o.abs_tol ? 1 : 0;
  p.max_sweeps = o.max_sweeps;
  p.mma = o.mma < 0 ? svdj_choose_mma(dtype, W) : o.mma;
  p.inner_order = o.inner;
  p.exchange = o.exchange;
  p.stop_rule = o.stop_rule;
  p.quad = o.quad;
  p.stream_a = sa;
  p.stream_b = sb;
  p.stream_comm = sc;
  p.hist = hist.data();
  p.timeout_s = o.timeout;
  p.comm_timing = o.comm_timing ? 1 : 0;
  p.progress = o.progress ? 1 : 0;
  p.fault_rank = o.fault_rank;
  p.fault_sweep = o.fault_sweep;
  // persistent handle: workspaces, pair lists and events once, not per solve
  if (svdj_dist_handle_create(&p, &p.handle) < 0) {
    std::fprintf(stderr, "[rank %d] %s\n", rank, svdj_dist_last_error());
    return 2;
  }
  double secs = 0;
  // --warmup solves first (RCCL connects its peers lazily, on the first
  // send/recv), then the timed one; each starts from the original columns
  for (int it = 0; it <= o.warmup; ++it) {
    CK(hipMemcpy(dA, hA.data(), hA.size() * sizeof(T), hipMemcpyHostToDevice));
    p.held[0] = held[0];
    p.held[1] = held[1];
    // ---- timed region: V = I, column norms, sweeps, sigma / U normalisation
    NK(ncclAllReduce(dt, dt, 1, ncclFloat64, ncclSum, nc, sa));  // barrier
    CK(hipStreamSynchronize(sa));
    const auto t0 = std::chrono::steady_clock::now();
    for (int s = 0; s < 2 && o.want_v; ++s)
      if (svdj_set_identity(dtype, dV + (size_t)s * B * n_v, n_v, n_v, B, held[s] * B, sa) < 0) {
        std::fprintf(stderr, "[rank %d] %s\n", rank, svdj_hip_last_error());
        return 2;
      }
    if (svdj_col_norms2(dtype, dA, m_pad, m_pad, 2 * B, dD, sa) < 0) {
      std::fprintf(stderr, "[rank %d] %s\n", rank, svdj_hip_last_error());
      return 2;
    }
    if (const int r = svdj_dist_solve(&p, dS); r < 0) {
      std::fprintf(stderr, "[rank %d] %s\n", rank, svdj_dist_last_error());
      std::fflush(stderr);
      return r == -300 ? 3 : 2;  // -300: watchdog abort (the communicator is gone)
    }
    secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    CK(hipMemcpy(dt, &secs, sizeof(double), hipMemcpyHostToDevice));
    NK(ncclAllReduce(dt, dt, 1, ncclFloat64, ncclMax, nc, sa));
    CK(hipMemcpyAsync(&secs, dt, sizeof(double), hipMemcpyDeviceToHost, sa));
    CK(hipStreamSynchronize(sa));
  }

  if (rank == 0) {
    std::printf("%s\n", svdj_hip_version());
    std::printf("Dimensions, height: %d, width: %d\n", m, n);
    std::printf("ranks: %d  block W: %d  super-block B: %d  %s\n", world, W, B,
                o.shared ? "(shared GPU)" : "");
    std::printf("SVD MPI+OMP time with U,V calculation: %.6f\n", secs);
    std::printf("sweeps: %d  converged: %d  last off value: %.3e  tol: %.3e\n", p.sweeps,
                p.converged, p.sweeps > 0 ? hist[p.sweeps - 1] : 0.0, tol);
    const double flops = (double)n * (n - 1) / 2.0 * (12.0 * m + (o.want_v ? 6.0 * n : 0.0)) * p.sweeps;
    std::printf("GFLOP/s (algorithmic): %.1f\n", flops / secs / 1e9);
    std::printf("issue: %s%s  exchange: %s\n", p.merged_used ? "merged chains" : "two chains",
                p.quad_used ? ", quad steps" : "",
                world == 1 ? "none" : (p.exchange_used == 2 ? "spread" : "direct"));
    if (p.calib_direct_ms > 0)
      std::printf("exchange calibration: direct %.3f ms, spread %.3f ms per half exchange\n",
                  p.calib_direct_ms, p.calib_spread_ms);
    if (o.comm_timing)
      std::printf("comm_ms: %.3f  exposed_comm_ms: %.3f\n", p.comm_ms, p.exposed_comm_ms);
  }

  int rc = 0;
  if (o.verify) {
    // gather (held, sigma, U columns, V columns) on rank 0
    int32_t* dh;
    CK(hipMalloc((void**)&dh, 2 * world * sizeof(int32_t)));
    CK(hipMemcpy(dh + 2 * rank, p.held, 2 * sizeof(int32_t), hipMemcpyHostToDevice));
    T *gA = nullptr, *gV = nullptr, *gS = nullptr;
    if (rank == 0) {
      CK(hipMalloc((void**)&gA, (size_t)world * 2 * B * m_pad * sizeof(T)));
      CK(hipMalloc((void**)&gS, (size_t)world * 2 * B * sizeof(T)));
      if (o.want_v) CK(hipMalloc((void**)&gV, (size_t)world * 2 * B * n_v * sizeof(T)));
    }
    NK(ncclGroupStart());
    if (rank == 0) {
      for (int r = 1; r < world; ++r) {
        NK(ncclRecv(dh + 2 * r, 2, ncclInt32, r, nc, sa));
        NK(ncclRecv(gA + (size_t)r * 2 * B * m_pad, (size_t)2 * B * m_pad, nt, r, nc, sa));
        NK(ncclRecv(gS + (size_t)r * 2 * B, (size_t)2 * B, nt, r, nc, sa));
        if (o.want_v) NK(ncclRecv(gV + (size_t)r * 2 * B * n_v, (size_t)2 * B * n_v, nt, r, nc, sa));
      }
    } else {
      NK(ncclSend(dh + 2 * rank, 2, ncclInt32, 0, nc, sa));
      NK(ncclSend(dA, (size_t)2 * B * m_pad, nt, 0, nc, sa));
      NK(ncclSend(dS, (size_t)2 * B, nt, 0, nc, sa));
      if (o.want_v) NK(ncclSend(dV, (size_t)2 * B * n_v, nt, 0, nc, sa));
    }
    NK(ncclGroupEnd());
    CK(hipStreamSynchronize(sa));
    if (rank == 0) {
      CK(hipMemcpy(gA, dA, (size_t)2 * B * m_pad * sizeof(T), hipMemcpyDeviceToDevice));
      CK(hipMemcpy(gS, dS, (size_t)2 * B * sizeof(T), hipMemcpyDeviceToDevice));
      if (o.want_v) CK(hipMemcpy(gV, dV, (size_t)2 * B * n_v * sizeof(T), hipMemcpyDeviceToDevice));
      std::vector<int32_t> hh(2 * world);
      std::vector<T> hU((size_t)world * 2 * B * m_pad), hS((size_t)world * 2 * B),
          hV(o.want_v ? (size_t)world * 2 * B * n_v : 0);
      CK(hipMemcpy(hh.data(), dh, hh.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
      CK(hipMemcpy(hU.data(), gA, hU.size() * sizeof(T), hipMemcpyDeviceToHost));
      CK(hipMemcpy(hS.data(), gS, hS.size() * sizeof(T), hipMemcpyDeviceToHost));
      if (o.want_v) CK(hipMemcpy(hV.data(), gV, hV.size() * sizeof(T), hipMemcpyDeviceToHost));
      // local slot (r, s) holds global columns [hh[2r+s] B, +B)
      std::vector<double> U((size_t)n * m), S(n), V(o.want_v ? (size_t)n * n : 0);
      std::vector<int> seen(2 * world, 0);
      for (int r = 0; r < world; ++r)
        for (int s = 0; s < 2; ++s) {
          const int sb = hh[2 * r + s];
          if (sb < 0 || sb >= 2 * world || seen[sb]++) {
            std::fprintf(stderr, "bad final placement: super-block %d\n", sb);
            rc = 4;
          }
          for (int c = 0; c < B && rc == 0; ++c) {
            const int j = sb * B + c;
            if (j >= n) break;
            const size_t src = (size_t)(r * 2 + s) * B + c;
            S[j] = hS[src];
            for (int i = 0; i < m; ++i) U[(size_t)j * m + i] = hU[src * m_pad + i];
            if (o.want_v)
              for (int i = 0; i < n; ++i) V[(size_t)j * n + i] = hV[src * n_v + i];
          }
        }
      if (rc == 0) {
        double anorm = 0;
        for (double x : A) anorm += x * x;
        anorm = std::sqrt(anorm);
        const double ou = svdj_cpu_orth_f64(m, n, U.data(), m, 0);
        std::printf("||U^TU-I||_F: %.3e\n", ou);
        if (o.want_v) {
          const double resid = svdj_cpu_residual_f64(m, n, n, A.data(), m, U.data(), m, S.data(),
                                                     V.data(), n, 0);
          const double ov = svdj_cpu_orth_f64(n, n, V.data(), n, 0);
          std::printf("||A-USVt||_F: %.6e\n||A-USVt||_F/||A||_F: %.3e\n||V^TV-I||_F: %.3e\n", resid,
                      resid / anorm, ov);
          const double lim = dtype ? 1e-10 : 1e-4;
          if (!(resid / anorm < lim)) {
            std::fprintf(stderr, "verification failed: relative residual %.3e >= %.1e\n",
                         resid / anorm, lim);
            rc = 5;
          }
        }
      }
      (void)hipFree(gA);
      (void)hipFree(gS);
      (void)hipFree(gV);
    }
    (void)hipFree(dh);
  }
  if (rank == 0 && !p.converged) std::printf("warning: not converged in %d sweeps\n", p.sweeps);
  (void)hipFree(dA);
  (void)hipFree(dV);
  (void)hipFree(dD);
  (void)hipFree(dS);
  (void)hipFree(dt);
  svdj_dist_handle_destroy(p.handle);
  svdj_dist_comm_destroy(comm);
  return rc;
}

int rank_main(const Opts& o, int rank, int world, int local) {
  if (o.shared) {
    const std::string host = "svdj-shared-gpu-rank" + std::to_string(rank);
    setenv("NCCL_HOSTID", host.c_str(), 1);
    setenv("NCCL_SOCKET_IFNAME", "lo", 0);
    setenv("NCCL_IB_DISABLE", "1", 0);
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    std::fprintf(stderr, "[rank %d] no GPU\n", rank);
    return 2;
  }
  const int device = o.shared ? 0 : local % ndev;
  if (!o.shared && world > ndev) {
    std::fprintf(stderr, "%d ranks but %d GPUs (use --shared-gpu to rehearse on one)\n", world, ndev);
    return 1;
  }
  return o.f32 ? run_rank<float>(o, rank, world, device) : run_rank<double>(o, rank, world, device);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s N --np P [--m M] [--dtype f32|f64] [--block W (default: per-GPU size)] [--shared-gpu] [--verify] ...\n",
                 argv[0]);
    return 1;
  }
  Opts o;
  o.n = std::atoi(argv[1]);
  std::string mma = "auto";
  for (int i = 2; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--m") o.m = std::atoi(next());
    else if (a == "--np") o.np = std::atoi(next());
    else if (a == "--input") o.dense = std::string(next()) == "dense";
    else if (a == "--seed") o.seed = (unsigned)std::strtoul(next(), nullptr, 10);
    else if (a == "--dtype") o.f32 = std::string(next()) == "f32";
    else if (a == "--block") o.W = std::atoi(next());
    else if (a == "--max-sweeps") o.max_sweeps = std::atoi(next());
    else if (a == "--tol") o.tol = std::atof(next());
    else if (a == "--abs-tol") o.abs_tol = true;
    else if (a == "--mma") mma = next();
    else if (a == "--no-v") o.want_v = false;
    else if (a == "--shared-gpu") o.shared = true;
    else if (a == "--verify") o.verify = true;
    else if (a == "--timeout") o.timeout = std::atof(next());
    else if (a == "--warmup") o.warmup = std::atoi(next());
    else if (a == "--exchange") {
      const std::string v = next();
      o.exchange = v == "spread" ? 2 : (v == "direct" ? 1 : 0);
    } else if (a == "--inner") {
      const std::string v = next();
      o.inner = v == "auto" ? 3 : (v == "cross" ? 2 : (v == "bipartite" ? 1 : 0));
    }
    else if (a == "--id-file") o.id_file = next();
    else if (a == "--comm-timing") o.comm_timing = true;
    else if (a == "--progress") o.progress = true;
    else if (a == "--stop-rule") o.stop_rule = std::string(next()) == "no_rotation" ? 0 : 1;
    else if (a == "--quad") {
      const std::string v = next();
      o.quad = v == "on" ? 1 : (v == "off" ? 2 : 0);
    }
    else if (a == "--keep-going") o.keep_going = true;
    else if (a == "--inject-fault") {
      const std::string v = next();
      const size_t c = v.find(':');
      if (c == std::string::npos) {
        std::fprintf(stderr, "--inject-fault RANK:SWEEP\n");
        return 1;
      }
      o.fault_rank = std::atoi(v.substr(0, c).c_str());
      o.fault_sweep = std::atoi(v.substr(c + 1).c_str());
    }
    else {
      std::fprintf(stderr, "unknown option %s\n", a.c_str());
      return 1;
    }
  }
  if (o.m == 0) o.m = o.n;
  if (o.n < 1 || o.m < o.n) {
    std::fprintf(stderr, "N >= 1 and m >= N required\n");
    return 1;
  }
  // -1 = auto: svdj_choose_mma once the block width is known (run_rank)
  if (o.f32) o.mma = mma == "auto" ? -1 : (mma == "bf16x6" ? 1 : (mma == "bf16x3" ? 2 : 0));

  const char* env_rank = std::getenv("RANK");
  const char* env_world = std::getenv("WORLD_SIZE");
  if (o.np == 0 && env_rank && env_world) {  // external launcher: this process is one rank
    if (o.id_file.empty()) {
      const char* e = std::getenv("SVDJ_DIST_ID");
      const char* port = std::getenv("MASTER_PORT");
      const char* run = std::getenv("TORCHELASTIC_RUN_ID");  // unique per torchrun job
      o.id_file = e ? e : std::string("/tmp/svdj_dist_") + (port ? port : "0") +
                              (run && std::strcmp(run, "none") ? std::string("_") + run : "") + ".id";
    }
    const char* lr = std::getenv("LOCAL_RANK");
    const int rank = std::atoi(env_rank);
    const int rc = rank_main(o, rank, std::atoi(env_world), lr ? std::atoi(lr) : rank);
    if (rank == 0) std::remove(o.id_file.c_str());
    return rc;
  }
  if (o.np < 1) o.np = 1;
  if (o.id_file.empty()) o.id_file = "/tmp/svdj_dist_" + std::to_string(getpid()) + ".id";
  std::remove(o.id_file.c_str());
  // one job token for the ranks forked below (svdj_dist_comm_init accepts
  // only an id file carrying it)
  const std::string tok = std::to_string(getpid()) + "-" + std::to_string((long long)time(nullptr));
  setenv("SVDJ_JOB_TOKEN", tok.c_str(), 1);
  std::fflush(stdout);
  // fork every rank before anything touches the GPU; the parent only waits
  std::vector<pid_t> pids;
  for (int r = 0; r < o.np; ++r) {
    const pid_t pid = fork();
    if (pid < 0) {
      std::perror("fork");
      for (pid_t q : pids) kill(q, SIGKILL);
      return 2;
    }
    if (pid == 0) {
      const int rc = rank_main(o, r, o.np, r);
      std::fflush(stdout);
      std::fflush(stderr);
      _exit(rc);
    }
    pids.push_back(pid);
  }
  int worst = 0, alive = o.np;
  std::vector<char> done(o.np, 0);
  auto stop_others = [&](int sig) {  // only children not yet reaped (their pids are ours)
    for (int r = 0; r < o.np; ++r)
      if (!done[r]) kill(pids[r], sig);
  };
  const auto t0 = std::chrono::steady_clock::now();
  while (alive > 0) {
    int st = 0;
    const pid_t pid = waitpid(-1, &st, WNOHANG);
    if (pid > 0) {
      --alive;
      int who = -1;
      for (int r = 0; r < o.np; ++r)
        if (pids[r] == pid) who = r;
      if (who >= 0) done[who] = 1;
      const int code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
      if (code != 0) {
        std::fprintf(stderr, "rank %d exited with %d; stopping the job\n", who, code);
        if (!worst) {
          worst = code;
          if (!o.keep_going) stop_others(SIGTERM);
        }
      }
      continue;
    }
    if (pid < 0) break;
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > o.timeout + 30) {
      std::fprintf(stderr, "job exceeded %.0f s; stopping the ranks\n", o.timeout);
      stop_others(SIGKILL);
      worst = 124;
      o.timeout = 1e30;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  std::remove(o.id_file.c_str());
  return worst;
}
