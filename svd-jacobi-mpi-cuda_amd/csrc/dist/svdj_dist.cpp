// Native distributed block one-sided Jacobi (svdj_dist.h): RCCL + the HIP
// block kernels of libsvdj_hip, no Python.  Same plan as the Python executor
// (parallel/pipeline.py, parallel/distributed.py):
//
// Per sweep on GPU g (slots 0 and 1 hold super-blocks of k = B/W blocks,
// each split in halves 0|1 of k/2 blocks; I = incoming slot, S = the other):
//   round 0 : round robin inside each slot            (chain 0: slot 0, 1: slot 1)
//   round r : I0xS0 (0), I0xS1 (0), I1xS0 (1), send half 0 of the slot
//             replaced next, I1xS1 (1), send half 1   (last round: no sends)
// Tasks on different chains touching disjoint halves are issued as one
// staggered svdj_block_steps2 pair; every dependency (half -> task, task ->
// send, arrival -> consumer) is a HIP event, so exchanges overlap the compute
// of the other halves (reference main.cu:582-680, 854-936 sends whole blocks
// with blocking MPI between rounds).  The stop test is an RCCL all-reduce (max
// of the float-ordered uint32 convergence value, sum of rotated pairs) per
// sweep: the value the reference computes and discards (main.cu:710).
#include "svdj_dist.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdlib.h>
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
           std::vector<int32_t> modes) {
  t.steps = steps;
  t.npairs = npairs;
  t.modes = std::move(modes);
  HIPC(hipMalloc((void**)&t.pairs, host.size() * sizeof(int32_t)));
  HIPC(hipMemcpy(t.pairs, host.data(), host.size() * sizeof(int32_t), hipMemcpyHostToDevice));
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

extern "C" int svdj_dist_choose_block(int dtype, int world, int m, int n) {
  // models/block.py choose_block (measurements there)
  const int per_gpu = n / (world > 0 ? world : 1);
  if (dtype == 1) return (m >= 12288 && per_gpu >= 4096) ? 64 : 32;
  return (m >= 8192 && per_gpu >= 2048) ? 64 : 32;
}

extern "C" int svdj_dist_initial_held(int world, int rank, int32_t held[2]) {
  Tour t(world);
  held[0] = t.h(0, rank, 0);
  held[1] = t.h(0, rank, 1);
  return 0;
}

namespace {

// ---- sweep plan of one GPU (parallel/pipeline.py sweep_plan / issue_groups)
// Halves are keyed slot*2 + half.  Tasks carry their device pairs and the
// stream (chain) they run on; a Send moves one half of one slot.
struct Item {
  bool send = false;
  const Task* task = nullptr;
  int stream = 0, hv[2] = {0, 0};  // task: chain and the two halves it touches
  int round = 0, slot = 0, half = 0;  // send
};

std::vector<Item> sweep_items(const Tour& t, int g, const Task rr[2], const Task cross[2][2][2]) {
  std::vector<Item> it;
  auto task = [&](const Task* tk, int stream, int h0, int h1) {
    Item x;
    x.task = tk;
    x.stream = stream;
    x.hv[0] = h0;
    x.hv[1] = h1;
    it.push_back(x);
  };
  auto send = [&](int r, int slot, int half) {
    Item x;
    x.send = true;
    x.round = r;
    x.slot = slot;
    x.half = half;
    it.push_back(x);
  };
  task(&rr[0], 0, 0, 1);
  task(&rr[1], 1, 2, 3);
  for (int r = 0; r < t.R; ++r) {
    const int inc = r ? t.x(r, g) : 0, stay = 1 - inc;
    auto T = [&](int ih, int sh, int stream) {
      task(&cross[inc][ih][sh], stream, inc * 2 + ih, stay * 2 + sh);
    };
    if (r + 1 == t.R) {  // nothing to send: two fully parallel phases
      T(0, 0, 0), T(1, 1, 1), T(0, 1, 0), T(1, 0, 1);
      continue;
    }
    const int nxt = t.x(r + 1, g);
    T(0, 0, 0), T(0, 1, 0), T(1, 0, 1);
    send(r + 1, nxt, 0);
    T(1, 1, 1);
    send(r + 1, nxt, 1);
  }
  return it;
}

// Issue order: a task is paired with the next task (at most one Send in
// between) when they run on different chains, touch disjoint halves and the
// Send concerns neither half of the second; the Send is issued after the pair.
struct Group {
  int a = -1, b = -1;  // item indices (b = -1: single task; a is a Send if items[a].send)
};

std::vector<Group> issue_groups(const std::vector<Item>& it) {
  std::vector<Group> out;
  const int n = (int)it.size();
  int i = 0;
  while (i < n) {
    if (!it[i].send) {
      int j = i + 1;
      while (j < n && it[j].send) ++j;
      if (j < n && j - i - 1 <= 1) {
        const Item &x = it[i], &y = it[j];
        bool ok = y.stream != x.stream;
        for (int u : x.hv)
          for (int v : y.hv) ok = ok && u != v;
        for (int s = i + 1; s < j; ++s)
          for (int v : y.hv) ok = ok && it[s].slot * 2 + it[s].half != v;
        if (ok) {
          out.push_back({i, j});
          for (int s = i + 1; s < j; ++s) out.push_back({s, -1});
          i = j + 1;
          continue;
        }
      }
    }
    out.push_back({i, -1});
    ++i;
  }
  return out;
}

}  // namespace

extern "C" int svdj_dist_plan(int world, int rank, int32_t* out, int cap) {
  if (world < 1 || rank < 0 || rank >= world) return fail(-2, "bad plan args");
  Tour tour(world);
  Task rr[2], cross[2][2][2];
  const std::vector<Item> items = sweep_items(tour, rank, rr, cross);
  const std::vector<Group> groups = issue_groups(items);
  if ((int)groups.size() > cap) return fail(-2, "plan has %zu groups, cap %d", groups.size(), cap);
  for (size_t i = 0; i < groups.size(); ++i) {
    int32_t* o = out + 7 * i;
    const Item& a = items[groups[i].a];
    for (int j = 0; j < 7; ++j) o[j] = -1;
    if (a.send) {
      o[0] = 2, o[1] = a.round, o[2] = a.slot, o[3] = a.half;
      continue;
    }
    o[0] = groups[i].b < 0 ? 0 : 1;
    o[1] = a.stream, o[2] = a.hv[0], o[3] = a.hv[1];
    if (groups[i].b >= 0) {
      const Item& b = items[groups[i].b];
      o[4] = b.stream, o[5] = b.hv[0], o[6] = b.hv[1];
    }
  }
  return (int)groups.size();
}

// Two chains of a group: issued independently (default) or offset by an EVD
// (svdj_block_steps2, SVDJ_DIST_STAGGER=1) -- the Python executor's
// SolverConfig.stagger; independent issue measured faster since the
// bipartite EVD and the round-2 apply geometry (profiles/r2_stag2).
static bool stagger_on() {
  static const bool on = [] {
    const char* e = getenv("SVDJ_DIST_STAGGER");
    return e && e[0] == '1';
  }();
  return on;
}

extern "C" int svdj_dist_solve(svdj_dist_problem* p, void* sigma) {
  const int P = p->world, g = p->rank, W = p->W, B = p->B;
  const int k = B / W, hk = k / 2, hB = hk * W;
  if (B % W || k < 2 || k % 2) return fail(-2, "B=%d must hold an even number of W=%d blocks", B, W);
  if (p->stream_a == p->stream_b) return fail(-2, "two distinct streams needed");
  const size_t es = p->dtype == 1 ? 8 : 4;
  hipStream_t st[2] = {(hipStream_t)p->stream_a, (hipStream_t)p->stream_b};
  hipStream_t sa = st[0];
  ncclComm_t comm = (ncclComm_t)p->comm;
  const ncclDataType_t nt = p->dtype == 1 ? ncclFloat64 : ncclFloat32;
  Tour tour(P);

  // ---- plans (local block ids: slot s holds blocks [s k, (s+1) k))
  std::vector<int32_t> rr((size_t)(k - 1) * (k / 2) * 2);
  svdj_round_robin(k, rr.data());
  Task rr_task[2], cross[2][2][2];  // cross[incoming slot][I half][S half]
  const int cross_mode = p->inner_order ? 2 : 0;  // svdj_block_steps mode of a cross step
  std::vector<int32_t> rr_modes(k - 1, cross_mode);
  rr_modes[0] = 1;  // the first step of a sweep re-measures the diagonal (full Gram)
  int rc = 0;
  for (int s = 0; s < 2 && !rc; ++s) {
    std::vector<int32_t> h = rr;
    for (auto& v : h) v += s * k;
    rc = upload(rr_task[s], h, k - 1, k / 2, rr_modes);
  }
  for (int inc = 0; inc < 2; ++inc)
    for (int ih = 0; ih < 2; ++ih)
      for (int sh = 0; sh < 2 && !rc; ++sh) {
        const int stay = 1 - inc;
        std::vector<int32_t> h((size_t)hk * hk * 2);
        for (int t = 0; t < hk; ++t)
          for (int a = 0; a < hk; ++a) {
            h[(t * hk + a) * 2] = inc * k + ih * hk + a;
            h[(t * hk + a) * 2 + 1] = stay * k + sh * hk + (a + t) % hk;
          }
        rc = upload(cross[inc][ih][sh], h, hk, hk, std::vector<int32_t>(hk, cross_mode));
      }
  const std::vector<Item> items = sweep_items(tour, g, rr_task, cross);
  const std::vector<Group> groups = issue_groups(items);

  // ---- workspaces (one per chain), metric, per-half receive buffers, events
  const size_t wsb = svdj_block_workspace_bytes(p->dtype, W, k / 2, p->m_pad);
  void* ws[2] = {nullptr, nullptr};
  void *rA[2] = {nullptr, nullptr}, *rV[2] = {nullptr, nullptr}, *rD[2] = {nullptr, nullptr};
  uint32_t* metric = nullptr;
  hipStream_t sc = (hipStream_t)p->stream_comm;
  const bool own_sc = sc == nullptr && P > 1;
  std::vector<hipEvent_t> ev(items.size() + 4, nullptr);  // per item + ready, join, copied[2]
  auto alloc = [&](void** q, size_t bytes) {
    if (!rc && hipMalloc(q, bytes) != hipSuccess) rc = fail(-100, "hipMalloc(%zu) failed", bytes);
  };
  for (int c = 0; c < 2; ++c) alloc(&ws[c], wsb);
  alloc((void**)&metric, 2 * sizeof(uint32_t));
  if (P > 1)
    for (int h = 0; h < 2; ++h) {
      alloc(&rA[h], (size_t)hB * p->m_pad * es);
      alloc(&rD[h], (size_t)hB * es);
      if (p->Vt) alloc(&rV[h], (size_t)hB * p->n_v * es);
    }
  if (!rc && own_sc && hipStreamCreateWithFlags(&sc, hipStreamNonBlocking) != hipSuccess)
    rc = fail(-100, "comm stream creation failed");
  for (auto& e : ev)
    if (!rc && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      rc = fail(-100, "event creation failed");
  hipEvent_t ev_ready = ev[items.size()], ev_join = ev[items.size() + 1];
  hipEvent_t* ev_copied = &ev[items.size() + 2];

  // placement of every GPU's slots (all ranks simulate the whole table)
  std::vector<int32_t> phys(2 * P);
  for (int h = 0; h < P; ++h) {
    phys[2 * h] = tour.h(0, h, 0);
    phys[2 * h + 1] = tour.h(0, h, 1);
  }
  if (!rc && (p->held[0] != phys[2 * g] || p->held[1] != phys[2 * g + 1]))
    rc = fail(-2, "rank %d holds (%d, %d), the tournament starts from (%d, %d)", g, p->held[0],
              p->held[1], phys[2 * g], phys[2 * g + 1]);

  auto rows = [&](int slot, int half) { return (size_t)slot * B + (size_t)half * hB; };
  // One sweep: every dependency is an event; the host never waits.
  auto sweep = [&]() -> int {
    std::vector<hipEvent_t> last[4];   // task events on each half since its last exchange
    hipEvent_t pending[4] = {nullptr, nullptr, nullptr, nullptr};  // arrived, not copied in
    bool copied_used[2] = {false, false};
    int halves_sent = 0;
    HIPC(hipMemsetAsync(metric, 0, 2 * sizeof(uint32_t), sa));
    HIPC(hipEventRecord(ev_ready, sa));
    HIPC(hipStreamWaitEvent(st[1], ev_ready, 0));
    if (sc) HIPC(hipStreamWaitEvent(sc, ev_ready, 0));
    auto consume = [&](int hv, hipStream_t s) -> int {
      if (!pending[hv]) return 0;
      HIPC(hipStreamWaitEvent(s, pending[hv], 0));
      pending[hv] = nullptr;
      const int slot = hv / 2, half = hv % 2;
      const size_t r0 = rows(slot, half);
      HIPC(hipMemcpyAsync((char*)p->At + r0 * p->m_pad * es, rA[half], (size_t)hB * p->m_pad * es,
                          hipMemcpyDeviceToDevice, s));
      HIPC(hipMemcpyAsync((char*)p->D + r0 * es, rD[half], (size_t)hB * es, hipMemcpyDeviceToDevice, s));
      if (p->Vt)
        HIPC(hipMemcpyAsync((char*)p->Vt + r0 * p->n_v * es, rV[half], (size_t)hB * p->n_v * es,
                            hipMemcpyDeviceToDevice, s));
      HIPC(hipEventRecord(ev_copied[half], s));  // the next receive into rV[half] waits on it
      copied_used[half] = true;
      return 0;
    };
    for (const Group& gr : groups) {
      const Item& a = items[gr.a];
      if (a.send) {  // one half of slot a.slot to send_to, its replacement from recv_from
        const int key = a.slot * 2 + a.half, dst = tour.to(a.round, g), src = tour.from(a.round, g);
        for (hipEvent_t e : last[key]) HIPC(hipStreamWaitEvent(sc, e, 0));
        last[key].clear();
        if (copied_used[a.half]) HIPC(hipStreamWaitEvent(sc, ev_copied[a.half], 0));
        const size_t r0 = rows(a.slot, a.half);
        NCCLC(ncclGroupStart());
        NCCLC(ncclSend((char*)p->At + r0 * p->m_pad * es, (size_t)hB * p->m_pad, nt, dst, comm, sc));
        NCCLC(ncclSend((char*)p->D + r0 * es, (size_t)hB, nt, dst, comm, sc));
        NCCLC(ncclRecv(rA[a.half], (size_t)hB * p->m_pad, nt, src, comm, sc));
        NCCLC(ncclRecv(rD[a.half], (size_t)hB, nt, src, comm, sc));
        if (p->Vt) {
          NCCLC(ncclSend((char*)p->Vt + r0 * p->n_v * es, (size_t)hB * p->n_v, nt, dst, comm, sc));
          NCCLC(ncclRecv(rV[a.half], (size_t)hB * p->n_v, nt, src, comm, sc));
        }
        NCCLC(ncclGroupEnd());
        hipEvent_t arrived = ev[gr.a];
        HIPC(hipEventRecord(arrived, sc));
        pending[key] = arrived;
        if (++halves_sent % 2 == 0) {  // both halves of round a.round issued: new placement
          std::vector<int32_t> old = phys;
          for (int h = 0; h < P; ++h) {
            const int sh = tour.from(a.round, h);
            phys[2 * h + tour.x(a.round, h)] = old[2 * sh + tour.x(a.round, sh)];
          }
        }
        continue;
      }
      const int n_t = gr.b < 0 ? 1 : 2;
      const Item* t[2] = {&a, gr.b < 0 ? nullptr : &items[gr.b]};
      for (int q = 0; q < n_t; ++q) {
        hipStream_t s = st[t[q]->stream];
        for (int hv : t[q]->hv) {
          for (hipEvent_t e : last[hv]) HIPC(hipStreamWaitEvent(s, e, 0));
          if (int r2 = consume(hv, s)) return r2;
        }
      }
      const Task &x = *t[0]->task;
      if (n_t == 2 && stagger_on()) {
        const Task& y = *t[1]->task;
        const int cx = t[0]->stream, cy = t[1]->stream;
        SVDJC(svdj_block_steps2(p->dtype, W, p->m_pad, p->At, p->m_pad, p->Vt, p->n_v, p->n_v, p->D,
                                x.pairs, x.npairs, x.steps, x.modes.data(), ws[cx], wsb, st[cx],
                                y.pairs, y.npairs, y.steps, y.modes.data(), ws[cy], wsb, st[cy],
                                p->tol, p->tol_mode, 1, metric, p->mma));
      } else {
        for (int q = 0; q < n_t; ++q) {  // one chain, or two issued independently
          const Task& z = *t[q]->task;
          const int cz = t[q]->stream;
          SVDJC(svdj_block_steps(p->dtype, W, p->m_pad, p->At, p->m_pad, p->Vt, p->n_v, p->n_v, p->D,
                                 z.pairs, z.npairs, z.steps, z.modes.data(), p->tol, p->tol_mode, 1,
                                 ws[cz], wsb, metric, p->mma, st[cz]));
        }
      }
      for (int q = 0; q < n_t; ++q) {
        hipEvent_t e = ev[q == 0 ? gr.a : gr.b];
        HIPC(hipEventRecord(e, st[t[q]->stream]));
        for (int hv : t[q]->hv) last[hv].push_back(e);
      }
    }
    HIPC(hipEventRecord(ev_join, st[1]));
    HIPC(hipStreamWaitEvent(sa, ev_join, 0));
    return 0;
  };

  if (!rc) {
    p->sweeps = 0;
    p->converged = 0;
  }
  for (int sw = 0; sw < p->max_sweeps && !rc; ++sw) {
    if ((rc = sweep())) break;
    // ---- stop test: global max convergence value (positive floats order as
    // uint32) and total rotated pairs
    uint32_t hm[2] = {0, 0};
    auto reduce = [&]() -> int {
      NCCLC(ncclAllReduce(metric, metric, 1, ncclUint32, ncclMax, comm, sa));
      NCCLC(ncclAllReduce(metric + 1, metric + 1, 1, ncclUint32, ncclSum, comm, sa));
      HIPC(hipMemcpyAsync(hm, metric, sizeof(hm), hipMemcpyDeviceToHost, sa));
      HIPC(hipStreamSynchronize(sa));
      return 0;
    };
    if ((rc = reduce())) break;
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
  } else {
    (void)hipDeviceSynchronize();  // nothing of this call may still run on its buffers
  }
  for (auto& e : ev)
    if (e) (void)hipEventDestroy(e);
  if (own_sc && sc) (void)hipStreamDestroy(sc);
  for (auto* t : {&rr_task[0], &rr_task[1]}) (void)hipFree(t->pairs);
  for (auto& a : cross)
    for (auto& b : a)
      for (auto& c : b) (void)hipFree(c.pairs);
  for (int h = 0; h < 2; ++h) {
    (void)hipFree(ws[h]);
    (void)hipFree(rA[h]);
    (void)hipFree(rD[h]);
    (void)hipFree(rV[h]);
  }
  (void)hipFree(metric);
  return rc;
}
