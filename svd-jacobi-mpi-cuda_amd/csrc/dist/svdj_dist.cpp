// Native distributed block one-sided Jacobi (svdj_dist.h): RCCL + the HIP
// block kernels of libsvdj_hip, no Python.
//
// Per sweep on GPU g (slots 0 and 1 hold super-blocks of k = B/W blocks,
// each split in halves 0|1 of k/2 blocks):
//   round 0: round robin inside each slot        (chain a: slot 0, b: slot 1)
//   every round r: cross pairs between the slots as four half tasks
//       phase 1: I0 x S0 (a) || I1 x S1 (b)
//       phase 2: I0 x S1 (a) || I1 x S0 (b)      (I = incoming slot, S = other)
//   between rounds: the slot named by the tournament is sent to one peer and
//   replaced by the block received from another (one grouped
//   ncclSend/ncclRecv, reference scatter/gather main.cu:582-680, 854-936).
// Each phase is one svdj_block_steps2 call (chain b's step s starts when
// chain a's EVD of step s is done); the two streams meet at phase ends.  The
// stop test is an RCCL all-reduce (max of the float-ordered uint32
// convergence value, sum of rotated pairs) per sweep: the value the
// reference computes and discards (main.cu:710).
#include "svdj_dist.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#include "svdj_cpu.h"
#include "svdj_hip.h"

namespace {

thread_local char g_err[512] = {0};

int fail(int rc, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return rc;
}

#define HIPC(x)                                                                    \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) return fail(-100, "%s:%d %s: %s", __FILE__, __LINE__, #x, \
                                      hipGetErrorString(e_));                      \
  } while (0)
#define NCCLC(x)                                                                   \
  do {                                                                             \
    ncclResult_t r_ = (x);                                                         \
    if (r_ != ncclSuccess) return fail(-200, "%s:%d %s: %s", __FILE__, __LINE__, #x, \
                                       ncclGetErrorString(r_));                    \
  } while (0)
#define SVDJC(x)                                                                   \
  do {                                                                             \
    int rc_ = (x);                                                                 \
    if (rc_ < 0) return fail(rc_, "%s:%d %s: %s", __FILE__, __LINE__, #x,           \
                             svdj_hip_last_error());                               \
  } while (0)

int rup(int a, int b) { return (a + b - 1) / b * b; }

struct Tour {
  int P, R;
  std::vector<int32_t> held, xslot, send_to, recv_from;
  explicit Tour(int P_) : P(P_), R(2 * P_ - 1), held(R * P_ * 2), xslot(R * P_), send_to(R * P_),
                          recv_from(R * P_) {
    svdj_tournament(P, held.data(), xslot.data(), send_to.data(), recv_from.data());
  }
  int h(int r, int g, int s) const { return held[(r * P + g) * 2 + s]; }
  int x(int r, int g) const { return xslot[r * P + g]; }
  int to(int r, int g) const { return send_to[r * P + g]; }
  int from(int r, int g) const { return recv_from[r * P + g]; }
};

// One chain of block steps: device pairs (steps, npairs, 2) + host modes.
struct Task {
  int32_t* pairs = nullptr;
  int steps = 0, npairs = 0;
  std::vector<int32_t> modes;
};

int upload(Task& t, const std::vector<int32_t>& host, int steps, int npairs,
           std::vector<int32_t> modes, hipStream_t st) {
  t.steps = steps;
  t.npairs = npairs;
  t.modes = std::move(modes);
  HIPC(hipMalloc((void**)&t.pairs, host.size() * sizeof(int32_t)));
  HIPC(hipMemcpyAsync(t.pairs, host.data(), host.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
  return 0;
}

}  // namespace

extern "C" const char* svdj_dist_last_error(void) { return g_err; }

extern "C" int svdj_dist_comm_init(int rank, int world, const char* id_path, double timeout_s,
                                   void** comm) {
  ncclUniqueId id;
  const std::string path(id_path);
  if (rank == 0) {
    NCCLC(ncclGetUniqueId(&id));
    const std::string tmp = path + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f || fwrite(&id, sizeof(id), 1, f) != 1) return fail(-1, "cannot write %s", tmp.c_str());
    fclose(f);
    if (rename(tmp.c_str(), path.c_str()) != 0) return fail(-1, "cannot publish %s", path.c_str());
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      FILE* f = fopen(path.c_str(), "rb");
      if (f) {
        const size_t got = fread(&id, sizeof(id), 1, f);
        fclose(f);
        if (got == 1) break;
      }
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s) return fail(-2, "rank %d: no unique id at %s after %.0f s", rank, path.c_str(), el);
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
  }
  ncclComm_t c;
  NCCLC(ncclCommInitRank(&c, world, id, rank));
  *comm = c;
  return 0;
}

extern "C" int svdj_dist_comm_destroy(void* comm) {
  if (comm) NCCLC(ncclCommDestroy((ncclComm_t)comm));
  return 0;
}

extern "C" int svdj_dist_geometry(int world, int m, int n, int W, int* B, int* ncols, int* m_pad,
                                  int* n_v) {
  if (world < 1 || m < n || n < 1 || (W != 32 && W != 64)) return fail(-2, "bad geometry args");
  const int q = 4 * world * W;  // B/W even: super-blocks split in halves
  const int nc = rup(n > q ? n : q, q);
  *ncols = nc;
  *B = nc / (2 * world);
  *m_pad = rup(m, SVDJ_ROW_ALIGN);
  *n_v = rup(nc, SVDJ_ROW_ALIGN);
  return 0;
}

extern "C" int svdj_dist_initial_held(int world, int rank, int32_t held[2]) {
  Tour t(world);
  held[0] = t.h(0, rank, 0);
  held[1] = t.h(0, rank, 1);
  return 0;
}

extern "C" int svdj_dist_solve(svdj_dist_problem* p, void* sigma) {
  const int P = p->world, g = p->rank, W = p->W, B = p->B;
  const int k = B / W, hk = k / 2;
  if (B % W || k < 2 || k % 2) return fail(-2, "B=%d must hold an even number of W=%d blocks", B, W);
  if (p->stream_a == p->stream_b) return fail(-2, "two distinct streams needed");
  const size_t es = p->dtype == 1 ? 8 : 4;
  hipStream_t sa = (hipStream_t)p->stream_a, sb = (hipStream_t)p->stream_b;
  ncclComm_t comm = (ncclComm_t)p->comm;
  const ncclDataType_t nt = p->dtype == 1 ? ncclFloat64 : ncclFloat32;
  Tour tour(P);

  // ---- plans (local block ids: slot s holds blocks [s k, (s+1) k))
  std::vector<int32_t> rr((size_t)(k - 1) * (k / 2) * 2);
  svdj_round_robin(k, rr.data());
  Task rr_task[2], cross[2][2][2];  // cross[incoming slot][I half][S half]
  std::vector<int32_t> rr_modes(k - 1, 0);
  rr_modes[0] = 1;  // the first step of a sweep re-measures the diagonal (full Gram)
  for (int s = 0; s < 2; ++s) {
    std::vector<int32_t> h = rr;
    for (auto& v : h) v += s * k;
    if (int rc = upload(rr_task[s], h, k - 1, k / 2, rr_modes, sa)) return rc;
  }
  for (int inc = 0; inc < 2; ++inc)
    for (int ih = 0; ih < 2; ++ih)
      for (int sh = 0; sh < 2; ++sh) {
        const int stay = 1 - inc;
        std::vector<int32_t> h((size_t)hk * hk * 2);
        for (int t = 0; t < hk; ++t)
          for (int a = 0; a < hk; ++a) {
            h[(t * hk + a) * 2] = inc * k + ih * hk + a;
            h[(t * hk + a) * 2 + 1] = stay * k + sh * hk + (a + t) % hk;
          }
        if (int rc = upload(cross[inc][ih][sh], h, hk, hk, std::vector<int32_t>(hk, 0), sa)) return rc;
      }

  // ---- workspaces, metric, exchange buffers, cross-stream events
  const size_t wsb = svdj_block_workspace_bytes(p->dtype, W, k / 2, p->m_pad);
  void *ws_a = nullptr, *ws_b = nullptr, *rA = nullptr, *rV = nullptr, *rD = nullptr;
  uint32_t* metric = nullptr;
  HIPC(hipMalloc(&ws_a, wsb));
  HIPC(hipMalloc(&ws_b, wsb));
  HIPC(hipMalloc((void**)&metric, 2 * sizeof(uint32_t)));
  HIPC(hipMalloc(&rA, (size_t)B * p->m_pad * es));
  HIPC(hipMalloc(&rD, (size_t)B * es));
  if (p->Vt) HIPC(hipMalloc(&rV, (size_t)B * p->n_v * es));
  hipEvent_t ea, eb;
  HIPC(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
  HIPC(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
  auto join = [&]() -> int {  // both streams wait for each other
    HIPC(hipEventRecord(ea, sa));
    HIPC(hipEventRecord(eb, sb));
    HIPC(hipStreamWaitEvent(sa, eb, 0));
    HIPC(hipStreamWaitEvent(sb, ea, 0));
    return 0;
  };
  auto phase = [&](const Task& a, const Task& b) -> int {
    SVDJC(svdj_block_steps2(p->dtype, W, p->m_pad, p->At, p->m_pad, p->Vt, p->n_v, p->n_v, p->D,
                            a.pairs, a.npairs, a.steps, a.modes.data(), ws_a, wsb, sa, b.pairs,
                            b.npairs, b.steps, b.modes.data(), ws_b, wsb, sb, p->tol, p->tol_mode,
                            1, metric, p->mma));
    return join();
  };

  // placement of every GPU's slots (all ranks simulate the whole table)
  std::vector<int32_t> phys(2 * P);
  for (int h = 0; h < P; ++h) {
    phys[2 * h] = tour.h(0, h, 0);
    phys[2 * h + 1] = tour.h(0, h, 1);
  }
  if (p->held[0] != phys[2 * g] || p->held[1] != phys[2 * g + 1])
    return fail(-2, "rank %d holds (%d, %d), the tournament starts from (%d, %d)", g, p->held[0],
                p->held[1], phys[2 * g], phys[2 * g + 1]);
  int rc = 0;
  p->sweeps = 0;
  p->converged = 0;
  for (int sw = 0; sw < p->max_sweeps && !rc; ++sw) {
    HIPC(hipMemsetAsync(metric, 0, 2 * sizeof(uint32_t), sa));
    if ((rc = join())) break;
    if ((rc = phase(rr_task[0], rr_task[1]))) break;
    for (int r = 0; r < tour.R && !rc; ++r) {
      const int inc = r == 0 ? 0 : tour.x(r, g);
      if ((rc = phase(cross[inc][0][0], cross[inc][1][1]))) break;
      if ((rc = phase(cross[inc][0][1], cross[inc][1][0]))) break;
      if (r + 1 < tour.R) {  // exchange before round r+1, on stream a (b waits below)
        const int x = tour.x(r + 1, g), dst = tour.to(r + 1, g), src = tour.from(r + 1, g);
        char* A0 = (char*)p->At + (size_t)x * B * p->m_pad * es;
        char* D0 = (char*)p->D + (size_t)x * B * es;
        NCCLC(ncclGroupStart());
        NCCLC(ncclSend(A0, (size_t)B * p->m_pad, nt, dst, comm, sa));
        NCCLC(ncclSend(D0, (size_t)B, nt, dst, comm, sa));
        NCCLC(ncclRecv(rA, (size_t)B * p->m_pad, nt, src, comm, sa));
        NCCLC(ncclRecv(rD, (size_t)B, nt, src, comm, sa));
        if (p->Vt) {
          char* V0 = (char*)p->Vt + (size_t)x * B * p->n_v * es;
          NCCLC(ncclSend(V0, (size_t)B * p->n_v, nt, dst, comm, sa));
          NCCLC(ncclRecv(rV, (size_t)B * p->n_v, nt, src, comm, sa));
        }
        NCCLC(ncclGroupEnd());
        HIPC(hipMemcpyAsync(A0, rA, (size_t)B * p->m_pad * es, hipMemcpyDeviceToDevice, sa));
        HIPC(hipMemcpyAsync(D0, rD, (size_t)B * es, hipMemcpyDeviceToDevice, sa));
        if (p->Vt)
          HIPC(hipMemcpyAsync((char*)p->Vt + (size_t)x * B * p->n_v * es, rV,
                              (size_t)B * p->n_v * es, hipMemcpyDeviceToDevice, sa));
        if ((rc = join())) break;
        std::vector<int32_t> old = phys;
        for (int h = 0; h < P; ++h) {
          const int sh = tour.from(r + 1, h);
          phys[2 * h + tour.x(r + 1, h)] = old[2 * sh + tour.x(r + 1, sh)];
        }
      }
    }
    if (rc) break;
    // ---- stop test: global max convergence value (positive floats order as
    // uint32) and total rotated pairs
    NCCLC(ncclAllReduce(metric, metric, 1, ncclUint32, ncclMax, comm, sa));
    NCCLC(ncclAllReduce(metric + 1, metric + 1, 1, ncclUint32, ncclSum, comm, sa));
    uint32_t hm[2];
    HIPC(hipMemcpyAsync(hm, metric, sizeof(hm), hipMemcpyDeviceToHost, sa));
    HIPC(hipStreamSynchronize(sa));
    float mx;
    memcpy(&mx, &hm[0], sizeof(float));
    if (p->hist) p->hist[sw] = mx;
    p->sweeps = sw + 1;
    if (hm[1] == 0) {
      p->converged = 1;
      break;
    }
  }
  if (!rc) {
    p->held[0] = phys[2 * g];
    p->held[1] = phys[2 * g + 1];
    if (sigma) {
      const int r2 = svdj_finalize(p->dtype, p->At, p->m_pad, p->m_pad, 2 * B, sigma, 1, sa);
      if (r2 < 0) rc = fail(r2, "finalize: %s", svdj_hip_last_error());
    }
    if (!rc && hipStreamSynchronize(sa) != hipSuccess) rc = fail(-100, "final sync failed");
  }
  (void)hipEventDestroy(ea);
  (void)hipEventDestroy(eb);
  for (auto* t : {&rr_task[0], &rr_task[1]}) (void)hipFree(t->pairs);
  for (auto& a : cross)
    for (auto& b : a)
      for (auto& c : b) (void)hipFree(c.pairs);
  (void)hipFree(ws_a);
  (void)hipFree(ws_b);
  (void)hipFree(metric);
  (void)hipFree(rA);
  (void)hipFree(rD);
  (void)hipFree(rV);
  return rc;
}
