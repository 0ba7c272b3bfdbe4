// Native distributed block one-sided Jacobi (svdj_dist.h): RCCL + the HIP
// block kernels of libsvdj_hip, no Python.  Same plan as the Python executor
// (parallel/pipeline.py, parallel/distributed.py):
//
// Per sweep on GPU g (slots 0 and 1 hold super-blocks of k = B/W blocks,
// each split in halves 0|1 of k/2 blocks; I = incoming slot, S = the other;
// one GPU from 64 pairs per chain step: the task pairs merged into single
// launches of twice the pairs and quad steps, as the Python engine):
//   round 0 : round robin inside each slot            (chain 0: slot 0, 1: slot 1)
//   round r : I0xS0 (0), I0xS1 (0), I1xS0 (1), send half 0 of the slot
//             replaced next, I1xS1 (1), send half 1   (last round: no sends)
// Tasks on different chains touching disjoint halves form one issue group
// (one GPU: merged into single launches); every dependency (half -> task, task ->
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
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "svdj_cpu.h"
#include "svdj_debug.h"
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

}  // namespace

extern "C" const char* svdj_dist_last_error(void) { return g_err; }

// The id file carries a job token next to the RCCL id, so a rank accepts
// only the file of its own job attempt: SVDJ_JOB_TOKEN (svdj_dist_main --np
// sets a fresh one before forking) or torchrun's TORCHELASTIC_RUN_ID joined
// with TORCHELASTIC_RESTART_COUNT (an elastic restart, or a reused
// --rdzv-id after a crash, must not pick up the dead attempt's id).  The
// file's age is checked in every case, against the start of the reading
// process: with a token it must be younger than that minus timeout_s (a
// leftover of an older job with the same token is refused), without one
// than that minus 30 s (tokenless launchers start their ranks together and
// remove the file before their rendezvous, as bench.py does).
namespace {
struct IdFile {
  char magic[8];
  char token[64];
  ncclUniqueId id;
};
constexpr char kIdMagic[8] = {'S', 'V', 'D', 'J', 'I', 'D', '2', 0};
std::string job_token() {
  const char* t = std::getenv("SVDJ_JOB_TOKEN");
  if (t && *t) return std::string(t).substr(0, 63);
  const char* r = std::getenv("TORCHELASTIC_RUN_ID");
  if (r && *r && std::strcmp(r, "none")) {
    const char* c = std::getenv("TORCHELASTIC_RESTART_COUNT");
    return (std::string(r).substr(0, 48) + "#" + (c && *c ? c : "0")).substr(0, 63);
  }
  return std::string();
}
}  // namespace

// Wall-clock start of this process (Linux /proc), or now if unavailable.
static time_t process_start_time() {
  static const time_t t = [] {
    const time_t now = time(nullptr);
    long long btime = -1;
    if (FILE* f = fopen("/proc/stat", "r")) {
      char line[256];
      while (fgets(line, sizeof(line), f))
        if (!strncmp(line, "btime ", 6)) btime = atoll(line + 6);
      fclose(f);
    }
    unsigned long long start_ticks = 0;
    bool ok = false;
    if (FILE* f = fopen("/proc/self/stat", "r")) {
      char buf[1024];
      const size_t k = fread(buf, 1, sizeof(buf) - 1, f);
      fclose(f);
      buf[k] = 0;
      // field 22 (starttime) counts from the field after the ')' of comm
      if (const char* p = strrchr(buf, ')')) {
        int field = 2;
        for (const char* q = p + 1; *q && !ok; ++q)
          if (*q == ' ' && ++field == 22) ok = sscanf(q + 1, "%llu", &start_ticks) == 1;
      }
    }
    const long hz = sysconf(_SC_CLK_TCK);
    if (btime < 0 || !ok || hz <= 0) return now;
    const time_t s = (time_t)(btime + (long long)(start_ticks / (unsigned long long)hz));
    return s <= now ? s : now;
  }();
  return t;
}

// Host part of the bootstrap (no RCCL, no GPU; CPU-tested under ASan):
// rank 0 publishes `n` bytes at `path` (written to path.tmp, then renamed),
// every other rank waits for a fresh file of this job's token and reads them.
extern "C" int svdj_dist_id_file(int rank, const char* id_path, double timeout_s, void* blob,
                                 size_t n) {
  IdFile rec;
  if (n != sizeof(rec.id)) return fail(-2, "id blob of %zu bytes, expected %zu", n, sizeof(rec.id));
  std::memset(&rec, 0, sizeof(rec));
  const std::string path(id_path), token = job_token();
  if (rank == 0) {
    std::memcpy(&rec.id, blob, n);
    std::memcpy(rec.magic, kIdMagic, sizeof(kIdMagic));
    std::memcpy(rec.token, token.data(), token.size());
    const std::string tmp = path + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return fail(-1, "cannot write %s", tmp.c_str());
    const bool ok = fwrite(&rec, sizeof(rec), 1, f) == 1;
    fclose(f);
    if (!ok) return fail(-1, "cannot write %s", tmp.c_str());
    if (rename(tmp.c_str(), path.c_str()) != 0) return fail(-1, "cannot publish %s", path.c_str());
    return 0;
  }
  // freshness is measured from this process's start, not from this call: the
  // ranks of one launch start together, and a peer that reaches here late
  // (slow GPU init or data load) must still accept the file its rank 0
  // published after the launch
  const double window = token.empty() ? 30.0 : (timeout_s > 30 ? timeout_s : 30.0);
  const time_t not_before = process_start_time() - (time_t)window;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    struct stat sb;
    const bool fresh = stat(path.c_str(), &sb) == 0 && sb.st_mtime >= not_before;
    FILE* f = fresh ? fopen(path.c_str(), "rb") : nullptr;
    if (f) {
      IdFile got;
      const size_t k = fread(&got, sizeof(got), 1, f);
      fclose(f);
      if (k == 1 && !std::memcmp(got.magic, kIdMagic, sizeof(kIdMagic)) &&
          !std::strncmp(got.token, token.c_str(), sizeof(got.token))) {
        std::memcpy(blob, &got.id, n);
        return 0;
      }
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > timeout_s)
      return fail(-2, "rank %d: no unique id of this job (token '%s') at %s after %.0f s", rank,
                  token.c_str(), path.c_str(), el);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

extern "C" int svdj_dist_comm_init(int rank, int world, const char* id_path, double timeout_s,
                                   void** comm) {
  ncclUniqueId id;
  std::memset(&id, 0, sizeof(id));
  if (rank == 0) NCCLC(ncclGetUniqueId(&id));
  if (int r = svdj_dist_id_file(rank, id_path, timeout_s, &id, sizeof(id))) return r;
  ncclComm_t c;
  NCCLC(ncclCommInitRank(&c, world, id, rank));
  *comm = c;
  return 0;
}

extern "C" int svdj_dist_comm_destroy(void* comm) {
  if (comm) NCCLC(ncclCommDestroy((ncclComm_t)comm));
  return 0;
}

// Size rule of the quad steps (hk = pairs per chain step), shared by the
// geometry's padding and svdj_dist_issue_rules (models/block.py quad_size_rule).
static bool quad_size_rule(int hk, int m_pad, int world) {
  (void)m_pad;  // round 6: no row condition since the shared-GPU apply grid (profiles/r6_rule)
  return hk >= 16 || (hk >= 12 && world > 1);
}

extern "C" int svdj_dist_geometry(int world, int m, int n, int W, int dtype, int* B, int* ncols,
                                  int* m_pad, int* n_v) {
  if (world < 1 || m < n || n < 1 || (W != 32 && W != 64) || dtype < 0 || dtype > 2)
    return fail(-2, "bad geometry args");
  const int q = 4 * world * W;  // B/W even: super-blocks split in halves
  int nc = rup(n > q ? n : q, q);
  const int mp = rup(m, SVDJ_ROW_ALIGN);
  // quad steps need k = B/W % 4 == 0: a column count that lands on k % 4 == 2
  // where the quad rule would hold takes one more q of zero columns (<= 6 %
  // more columns at the sizes the rule admits; quad vs single steps is 20-25 %
  // per solve).  Not for fp64 (no quad steps).  distributed.py geometry.
  if (dtype != 1 && W == 64 && svdj_debug_knob("quad_pad", 1) != 0) {
    const int k = nc / (2 * world * W);
    if (k % 4 == 2 && quad_size_rule((k + 2) / 2, mp, world)) nc += q;
  }
  *ncols = nc;
  *B = nc / (2 * world);
  *m_pad = mp;
  *n_v = rup(nc, SVDJ_ROW_ALIGN);
  return 0;
}

extern "C" int svdj_dist_choose_block(int dtype, int world, int m, int n) {
  // models/block.py choose_block (measurements there)
  const int per_gpu = n / (world > 0 ? world : 1);
  if (dtype == 1) return (m >= 6144 && per_gpu >= 2048) ? 64 : 32;
  return per_gpu >= 1024 ? 64 : 32;
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

extern "C" int svdj_dist_storage_cols(int world, int B) { return (world > 1 ? 3 : 2) * B; }

namespace {

// ---- where the resident halves live (parallel/pipeline.py HalfLayout).
// Half buffers of hB columns: loc[slot][half] holds (slot, half); spare[h] is
// the free buffer the next exchange of a half h receives into.  Buffers
// {h, 2+h, 4+h} always hold (slot 0, h), (slot 1, h), spare.
struct Layout {
  int loc[2][2] = {{0, 1}, {2, 3}};
  int spare[2] = {4, 5};
};

// Moves (src buffer, dst buffer) that bring every half home to buffer
// 2 slot + half, parking one half in the spare when two sit in each other's
// home (same rule as HalfLayout.moves_to_canonical).
std::vector<std::pair<int, int>> moves_to_canonical(Layout& L) {
  std::vector<std::pair<int, int>> mv;
  for (int h = 0; h < 2; ++h) {
    int where[2] = {L.loc[0][h], L.loc[1][h]}, free_b = L.spare[h];
    for (int it = 0; it < 4; ++it) {
      int todo[2], nt = 0;
      for (int s = 0; s < 2; ++s)
        if (where[s] != 2 * s + h) todo[nt++] = s;
      if (!nt) break;
      int pick = todo[0];
      for (int q = 0; q < nt; ++q)
        if (2 * todo[q] + h == free_b) pick = todo[q];
      mv.push_back({where[pick], free_b});
      const int old = where[pick];
      where[pick] = free_b;
      free_b = old;
    }
    L.loc[0][h] = where[0];
    L.loc[1][h] = where[1];
    L.spare[h] = free_b;
  }
  return mv;
}

// Interval measure of union(waits) minus union(busy) (pipeline.exposed_time).
double exposed_time(std::vector<std::pair<double, double>> w, std::vector<std::pair<double, double>> b) {
  auto merge = [](std::vector<std::pair<double, double>>& v) {
    std::sort(v.begin(), v.end());
    std::vector<std::pair<double, double>> o;
    for (auto& x : v) {
      if (x.second <= x.first) continue;
      if (!o.empty() && x.first <= o.back().second)
        o.back().second = std::max(o.back().second, x.second);
      else
        o.push_back(x);
    }
    v.swap(o);
  };
  merge(w);
  merge(b);
  double total = 0;
  size_t j = 0;
  for (auto& x : w) {
    double t = x.first;
    while (j < b.size() && b[j].second <= t) ++j;
    size_t k = j;
    while (t < x.second) {
      if (k < b.size() && b[k].first <= t) {
        t = std::max(t, b[k].second);
        ++k;
        continue;
      }
      const double nxt = k < b.size() ? std::min(b[k].first, x.second) : x.second;
      total += nxt - t;
      t = nxt;
    }
  }
  return total;
}

// A chain template: host pairs in canonical local block ids (slot*k +
// half*hk + j) and the two halves it touches; one device copy per placement
// of those halves (buffers bA, bB), built when the handle is created.
struct Template {
  std::vector<int32_t> host;
  int steps = 0, npairs = 0;
  std::vector<int32_t> modes;
  int hv[2] = {0, 0};                 // halves touched (slot*2 + half)
  int32_t* dev[6][6] = {};            // [buffer of hv[0]][buffer of hv[1]] -> device pairs
};

// Fail-fast watchdog: a thread polls the RCCL async
// error and the time since the last finished sweep.  On a fault it takes the
// NCCL lock (the solve holds it around every group of RCCL calls, so the
// communicator is never freed under an enqueue), sets `fired` and calls
// ncclCommAbort, which releases RCCL kernels spinning on the dead peer so
// the streams drain; the solve returns -300 at its next check.  If the lock
// cannot be had for 5 s (an enqueue itself is stuck), the process exits 3.
struct Watchdog {
  std::atomic<bool> stop{false}, fired{false};
  std::mutex mu;  // held by the solve around RCCL calls
  std::atomic<long long> last_ns{0};
  char why[256] = {0};
  std::thread th;
  static long long now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  void progress() { last_ns = now_ns(); }
  void start(ncclComm_t comm, double timeout_s, int rank) {
    progress();
    th = std::thread([this, comm, timeout_s, rank]() {
      while (!stop.load()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        ncclResult_t ae = ncclSuccess;
        const ncclResult_t q = ncclCommGetAsyncError(comm, &ae);
        const double idle = (now_ns() - last_ns.load()) * 1e-9;
        if (q != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress)) {
          snprintf(why, sizeof(why), "rank %d: RCCL async error: %s", rank,
                   ncclGetErrorString(q != ncclSuccess ? q : ae));
        } else if (idle > timeout_s) {
          snprintf(why, sizeof(why), "rank %d: no sweep finished for %.0f s (peer dead or hung)",
                   rank, idle);
        } else {
          continue;
        }
        fprintf(stderr, "[svdj_dist watchdog] %s: aborting the communicator\n", why);
        fflush(stderr);
        const long long t_lock = now_ns();
        while (!mu.try_lock()) {
          if ((now_ns() - t_lock) * 1e-9 > 5.0) {
            fprintf(stderr, "[svdj_dist watchdog] rank %d: RCCL call stuck, exiting\n", rank);
            fflush(stderr);
            _exit(3);
          }
          std::this_thread::sleep_for(std::chrono::milliseconds(5));
        }
        fired = true;
        (void)ncclCommAbort(comm);
        mu.unlock();
        return;
      }
    });
  }
  void join() {
    stop = true;
    if (th.joinable()) th.join();
  }
};

}  // namespace

struct svdj_dist_handle_t {
  int rank, world, dtype, W, m_pad, n_v, B, k, hk, hB, has_v, timing;
  bool spread = false;           // exchanges relayed over all links (parallel/spread.py)
  int io = 0;                    // resolved EVD order of the cross steps (0 cyclic, 1 bip, 2 cross)
  void* relay[2] = {nullptr, nullptr};  // A / V relay chunks, one row per source rank
  size_t relay_n[2] = {0, 0};           // elements per row
  ncclComm_t comm;
  hipStream_t st[2], sc;
  bool own_sc = false;
  size_t es, wsb;
  void* ws[2] = {nullptr, nullptr};
  uint32_t* metric = nullptr;
  int32_t* pairs_pool = nullptr;
  Template rr[2], cross[2][2][2];
  bool quad = false;    // quad steps (two cross steps fused) in every template
  bool merged = false;  // one GPU: each parallel task pair issued as one launch of twice the pairs
  int32_t* merged_pairs = nullptr;  // [rr0+rr1 | T00+T11 | T01+T10], device
  size_t merged_off[3] = {0, 0, 0};
  int merged_steps[3] = {0, 0, 0}, merged_np[3] = {0, 0, 0};
  std::vector<int32_t> merged_modes[3];
  double calib_ms[2] = {0, 0};  // exchange calibration: direct, spread (0: not run)
  std::vector<Item> items;
  std::vector<Group> groups;
  // per item: end event (task) / arrival (send); timing: start (task) / issue
  // (send), consumer-ready events (two per task); plus sweep start and join
  std::vector<hipEvent_t> ev, ev_start, ev_ready;
  hipEvent_t ev_t0 = nullptr, ev_join = nullptr;
  Layout L;
};

namespace {

// Host part of the plan's pair lists: every template's pairs and modes and,
// on one GPU, the merged lists (mp).  No device call (svdj_dist_merged_lists
// exposes it to the CPU tests).
void template_hosts(svdj_dist_handle_t* h, int cross_mode, std::vector<int32_t>& mp) {
  const int k = h->k, hk = h->hk;
  std::vector<int32_t> rr((size_t)(k - 1) * (k / 2) * 2);
  std::vector<int32_t> rr_modes(k - 1, cross_mode);
  if (h->quad) {  // quad order (block.hip "quad step"): modes 4 / 5 in pairs
    svdj_quad_round_robin(k, rr.data());
    for (int s = 1; s < k - 1; ++s) rr_modes[s] = (s & 1) ? 4 : 5;
  } else {
    svdj_round_robin(k, rr.data());
  }
  rr_modes[0] = 1;  // the first step of a sweep re-measures the diagonal (full Gram)
  for (int s = 0; s < 2; ++s) {
    Template& t = h->rr[s];
    t.host = rr;
    for (auto& v : t.host) v += s * k;
    t.steps = k - 1;
    t.npairs = k / 2;
    t.modes = rr_modes;
    t.hv[0] = 2 * s;
    t.hv[1] = 2 * s + 1;
  }
  for (int inc = 0; inc < 2; ++inc)
    for (int ih = 0; ih < 2; ++ih)
      for (int sh = 0; sh < 2; ++sh) {
        const int stay = 1 - inc;
        Template& t = h->cross[inc][ih][sh];
        t.host.assign((size_t)hk * hk * 2, 0);
        if (h->quad) {
          std::vector<int32_t> xs(hk), ys(hk);
          for (int a = 0; a < hk; ++a) {
            xs[a] = inc * k + ih * hk + a;
            ys[a] = stay * k + sh * hk + a;
          }
          svdj_quad_bipartite(hk, xs.data(), ys.data(), t.host.data());
          t.modes.assign(hk, 4);
          for (int s = 1; s < hk; s += 2) t.modes[s] = 5;
        } else {
          for (int q = 0; q < hk; ++q)
            for (int a = 0; a < hk; ++a) {
              t.host[(q * hk + a) * 2] = inc * k + ih * hk + a;
              t.host[(q * hk + a) * 2 + 1] = stay * k + sh * hk + (a + q) % hk;
            }
          t.modes.assign(hk, cross_mode);
        }
        t.steps = hk;
        t.npairs = hk;
        t.hv[0] = inc * 2 + ih;
        t.hv[1] = stay * 2 + sh;
      }
  mp.clear();
  if (h->merged) {
    // one GPU (canonical buffers: a local block id is its buffer block):
    // the parallel task pairs of the sweep -- rr0 + rr1, then the last round's
    // [T00 || T11] and [T01 || T10] -- concatenated step by step, the order
    // of pipeline.run_merged
    const Template* grp[3][2] = {{&h->rr[0], &h->rr[1]},
                                 {&h->cross[0][0][0], &h->cross[0][1][1]},
                                 {&h->cross[0][0][1], &h->cross[0][1][0]}};
    for (int m = 0; m < 3; ++m) {
      const Template &x = *grp[m][0], &y = *grp[m][1];
      h->merged_off[m] = mp.size();
      h->merged_steps[m] = x.steps;
      h->merged_np[m] = x.npairs + y.npairs;
      h->merged_modes[m] = x.modes;
      for (int st = 0; st < x.steps; ++st) {
        mp.insert(mp.end(), x.host.begin() + (size_t)st * x.npairs * 2,
                  x.host.begin() + (size_t)(st + 1) * x.npairs * 2);
        mp.insert(mp.end(), y.host.begin() + (size_t)st * y.npairs * 2,
                  y.host.begin() + (size_t)(st + 1) * y.npairs * 2);
      }
    }
  }
}

int build_templates(svdj_dist_handle_t* h, int cross_mode) {
  const int k = h->k, hk = h->hk;
  std::vector<int32_t> mp;
  template_hosts(h, cross_mode, mp);
  // every placement of each template's two halves: half h lives in one of
  // buffers {h, 2+h, 4+h} (only the canonical ones on one GPU)
  std::vector<Template*> all = {&h->rr[0], &h->rr[1]};
  for (auto& a : h->cross)
    for (auto& b : a)
      for (auto& c : b) all.push_back(&c);
  const int nopt = h->world > 1 ? 3 : 1;
  std::vector<int32_t> pool;
  std::vector<std::tuple<Template*, int, int, size_t>> where;
  for (Template* t : all)
    for (int ia = 0; ia < nopt; ++ia)
      for (int ib = 0; ib < nopt; ++ib) {
        const int ha = t->hv[0] % 2, hb = t->hv[1] % 2;
        const int ba = (ia == 0 ? t->hv[0] : (ia == 1 ? 2 * (1 - t->hv[0] / 2) + ha : 4 + ha));
        const int bb = (ib == 0 ? t->hv[1] : (ib == 1 ? 2 * (1 - t->hv[1] / 2) + hb : 4 + hb));
        if (ba == bb) continue;
        where.emplace_back(t, ba, bb, pool.size());
        for (int32_t v : t->host) {
          const int slot = v / k, rem = v % k, half = rem / hk, off = rem % hk;
          const int hvv = slot * 2 + half;
          const int buf = hvv == t->hv[0] ? ba : bb;
          pool.push_back(buf * hk + off);
        }
      }
  HIPC(hipMalloc((void**)&h->pairs_pool, pool.size() * sizeof(int32_t)));
  HIPC(hipMemcpy(h->pairs_pool, pool.data(), pool.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  for (auto& w : where) std::get<0>(w)->dev[std::get<1>(w)][std::get<2>(w)] = h->pairs_pool + std::get<3>(w);
  if (h->merged) {
    HIPC(hipMalloc((void**)&h->merged_pairs, mp.size() * sizeof(int32_t)));
    HIPC(hipMemcpy(h->merged_pairs, mp.data(), mp.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  return 0;
}

}  // namespace

extern "C" int svdj_dist_issue_rules(int world, int dtype, int W, int mma, int k, int m_pad,
                                     int quad_mode, int* quad, int* merged) {
  const bool quad_ok = dtype == 0 && W == 64 && (mma == 1 || mma == 2) && k % 4 == 0;
  if (quad_mode < 0 || quad_mode > 2) return fail(-2, "quad %d (0 auto, 1 on, 2 off)", quad_mode);
  if (quad_mode == 1 && !quad_ok)
    return fail(-2, "quad steps need fp32, W = 64, a split-bf16 apply and k %% 4 == 0");
  // models/block.py choose_quad, parallel/distributed.py choose_merged
  const int hk = k / 2;
  *quad = quad_ok && (quad_mode == 1 || (quad_mode == 0 && quad_size_rule(hk, m_pad, world)));
  const int force = svdj_debug_knob("merge", -1);  // A/B only (svdj_debug.h), world 1 only
  *merged = world == 1 && (force >= 0 ? force == 1 : *quad ? (hk >= 16 && hk < 32) : hk >= 64);
  return 0;
}

extern "C" int svdj_dist_merged_lists(int k, int quad, int cross_mode, int32_t* pairs, int pcap,
                                      int32_t* modes, int mcap, int32_t* meta) {
  if (k < 4 || k % 2 || (quad && k % 4)) return fail(-2, "bad merged-list args");
  svdj_dist_handle_t h{};
  h.rank = 0;
  h.world = 1;
  h.k = k;
  h.hk = k / 2;
  h.quad = quad != 0;
  h.merged = true;
  std::vector<int32_t> mp;
  template_hosts(&h, cross_mode, mp);
  size_t nm = 0;
  for (int m = 0; m < 3; ++m) nm += h.merged_modes[m].size();
  if (mp.size() > (size_t)pcap || nm > (size_t)mcap) return fail(-3, "merged lists: buffer too small");
  std::copy(mp.begin(), mp.end(), pairs);
  for (int m = 0, at = 0; m < 3; ++m) {
    meta[m * 3] = (int32_t)h.merged_off[m];
    meta[m * 3 + 1] = h.merged_steps[m];
    meta[m * 3 + 2] = h.merged_np[m];
    for (int32_t v : h.merged_modes[m]) modes[at++] = v;
  }
  return (int)mp.size();
}

namespace {

void handle_free(svdj_dist_handle_t* h) {
  if (!h) return;
  for (auto* v : {&h->ev, &h->ev_start, &h->ev_ready})
    for (auto& e : *v)
      if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : {h->ev_t0, h->ev_join})
    if (e) (void)hipEventDestroy(e);
  if (h->own_sc && h->sc) (void)hipStreamDestroy(h->sc);
  (void)hipFree(h->pairs_pool);
  (void)hipFree(h->merged_pairs);
  (void)hipFree(h->relay[0]);
  (void)hipFree(h->relay[1]);
  (void)hipFree(h->ws[0]);
  (void)hipFree(h->ws[1]);
  (void)hipFree(h->metric);
  delete h;
}


// One half exchange of tournament round `round` on stream sc (grouped RCCL):
// each message goes to send_to and arrives from recv_from, directly, or
// (spread, a message with a relay buffer) cut into P-1 near-equal chunks --
// chunk 0 direct, chunk j >= 1 via the j-th rank not in {sender, receiver}
// -- in two grouped phases (parallel/spread.py).  The data that arrives is
// the same bit for bit.
struct XMsg {
  char *out, *in;
  size_t n;
  char* relay;  // non-null: relayed (spread)
  size_t relay_n;
};
int exchange_ops(const Tour& tour, int round, int g, const XMsg* msgs, int nm, bool spread,
                 ncclDataType_t nt, size_t es, ncclComm_t comm, hipStream_t sc) {
  const int P = tour.P, dst = tour.to(round, g), src = tour.from(round, g);
  auto piece = [&](size_t n, int j, size_t& a, size_t& len) {
    const size_t base = n / (P - 1), rem = n % (P - 1);
    a = j * base + ((size_t)j < rem ? (size_t)j : rem);
    len = base + ((size_t)j < rem ? 1 : 0);
  };
  auto relay_index = [&](int s, int d, int q) {
    int j = 0;
    for (int x = 0; x < P; ++x) {
      if (x == s || x == d) continue;
      ++j;
      if (x == q) return j;
    }
    return -1;
  };
  size_t a0, ln;
  NCCLC(ncclGroupStart());  // direct messages / phase 1
  for (int i = 0; i < nm; ++i) {
    const XMsg& M = msgs[i];
    if (!spread || !M.relay) {
      NCCLC(ncclSend(M.out, M.n, nt, dst, comm, sc));
      NCCLC(ncclRecv(M.in, M.n, nt, src, comm, sc));
      continue;
    }
    piece(M.n, 0, a0, ln);
    NCCLC(ncclSend(M.out + a0 * es, ln, nt, dst, comm, sc));
    for (int q = 0, j = 0; q < P; ++q) {
      if (q == g || q == dst) continue;
      piece(M.n, ++j, a0, ln);
      NCCLC(ncclSend(M.out + a0 * es, ln, nt, q, comm, sc));
    }
    piece(M.n, 0, a0, ln);
    NCCLC(ncclRecv(M.in + a0 * es, ln, nt, src, comm, sc));
    for (int s = 0; s < P; ++s) {  // sources this rank relays for
      if (s == g || s == src) continue;
      piece(M.n, relay_index(s, tour.to(round, s), g), a0, ln);
      NCCLC(ncclRecv(M.relay + (size_t)s * M.relay_n * es, ln, nt, s, comm, sc));
    }
  }
  NCCLC(ncclGroupEnd());
  if (spread) {  // phase 2: forward the relayed chunks, receive ours
    NCCLC(ncclGroupStart());
    for (int i = 0; i < nm; ++i) {
      const XMsg& M = msgs[i];
      if (!M.relay) continue;
      for (int s = 0; s < P; ++s) {
        if (s == g || s == src) continue;
        const int d = tour.to(round, s);
        piece(M.n, relay_index(s, d, g), a0, ln);
        NCCLC(ncclSend(M.relay + (size_t)s * M.relay_n * es, ln, nt, d, comm, sc));
      }
      for (int q = 0, j = 0; q < P; ++q) {
        if (q == src || q == g) continue;
        piece(M.n, ++j, a0, ln);
        NCCLC(ncclRecv(M.in + a0 * es, ln, nt, q, comm, sc));
      }
    }
    NCCLC(ncclGroupEnd());
  }
  return 0;
}

// Wait for stream s without blocking forever.  Handle creation runs before
// the solve's watchdog exists, so its collectives are polled here: an RCCL
// async error or timeout_s without completion aborts the communicator (the
// RCCL kernels spinning on a dead peer are released and the stream drains)
// and returns -300, as a watchdog abort in svdj_dist_solve does.
int poll_stream(hipStream_t s, ncclComm_t comm, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return fail(-100, "stream error: %s", hipGetErrorString(q));
    ncclResult_t ae = ncclSuccess;
    const ncclResult_t r = ncclCommGetAsyncError(comm, &ae);
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (r != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress) || el > timeout_s) {
      (void)ncclCommAbort(comm);
      (void)hipStreamSynchronize(s);
      return fail(-300, "handle creation: %s; communicator aborted",
                  el > timeout_s ? "collective timed out" : "RCCL async error");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// Exchange calibration (pipeline.calibrate_exchange, ADVICE r3 / VERDICT r4):
// at handle creation, from 4 ranks with exchange auto, one half exchange of
// the first tournament round is timed both ways on this job's links (real
// half-buffer sizes of A, the norms and V; one warm-up, the best of 3; every
// timing the max over ranks), and spread is kept only if it is >= 10 %
// faster.  Every rank takes the same decision (the times are all-reduced).
int calibrate_exchange(svdj_dist_handle_t* h, double timeout_s) {
  const int P = h->world, g = h->rank;
  Tour tour(P);
  const size_t es = h->es;
  const ncclDataType_t nt = h->dtype == 1 ? ncclFloat64 : ncclFloat32;
  const size_t n[3] = {(size_t)h->hB * h->m_pad, (size_t)h->hB, h->has_v ? (size_t)h->hB * h->n_v : 0};
  char* buf[3][2] = {{nullptr, nullptr}, {nullptr, nullptr}, {nullptr, nullptr}};
  double* dt = nullptr;
  int rc = 0;
  for (int i = 0; i < 3 && !rc; ++i)
    for (int j = 0; j < 2 && !rc && n[i]; ++j)
      if (hipMalloc((void**)&buf[i][j], n[i] * es) != hipSuccess || hipMemset(buf[i][j], 0, n[i] * es) != hipSuccess)
        rc = fail(-100, "calibration buffers: hipMalloc failed");
  if (!rc && hipMalloc((void**)&dt, sizeof(double)) != hipSuccess) rc = fail(-100, "hipMalloc failed");
  double best[2] = {1e30, 1e30};
  for (int v = 0; v < 2 && !rc; ++v) {
    const bool spread = v == 1;
    XMsg msgs[3];
    int nm = 0;
    msgs[nm++] = {buf[0][0], buf[0][1], n[0], spread ? (char*)h->relay[0] : nullptr, h->relay_n[0]};
    msgs[nm++] = {buf[1][0], buf[1][1], n[1], nullptr, 0};
    if (n[2]) msgs[nm++] = {buf[2][0], buf[2][1], n[2], spread ? (char*)h->relay[1] : nullptr, h->relay_n[1]};
    for (int it = 0; it < 4 && !rc; ++it) {
      // line the ranks up (a tiny all-reduce), then time one exchange
      if (ncclAllReduce(dt, dt, 1, ncclFloat64, ncclMax, h->comm, h->sc) != ncclSuccess) {
        rc = fail(-200, "calibration barrier failed");
        break;
      }
      if ((rc = poll_stream(h->sc, h->comm, timeout_s))) break;
      const auto t0 = std::chrono::steady_clock::now();
      if ((rc = exchange_ops(tour, 1, g, msgs, nm, spread, nt, es, h->comm, h->sc))) break;
      if ((rc = poll_stream(h->sc, h->comm, timeout_s))) break;
      double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (hipMemcpy(dt, &t, sizeof(t), hipMemcpyHostToDevice) != hipSuccess ||
          ncclAllReduce(dt, dt, 1, ncclFloat64, ncclMax, h->comm, h->sc) != ncclSuccess) {
        rc = fail(-200, "calibration max over ranks failed");
        break;
      }
      if ((rc = poll_stream(h->sc, h->comm, timeout_s))) break;
      if (hipMemcpy(&t, dt, sizeof(t), hipMemcpyDeviceToHost) != hipSuccess) {
        rc = fail(-100, "calibration copy failed");
        break;
      }
      if (it) best[v] = std::min(best[v], t);
    }
  }
  for (auto& b : buf)
    for (char* x : b) (void)hipFree(x);
  (void)hipFree(dt);
  if (rc) return rc;
  h->calib_ms[0] = best[0] * 1e3;
  h->calib_ms[1] = best[1] * 1e3;
  h->spread = best[1] < 0.9 * best[0];
  if (!h->spread)
    for (void*& r : h->relay) {
      (void)hipFree(r);
      r = nullptr;
    }
  return 0;
}

}  // namespace

extern "C" int svdj_dist_handle_create(const svdj_dist_problem* p, void** out) {
  *out = nullptr;
  const int W = p->W, B = p->B;
  if (W <= 0 || B % W || (B / W) < 2 || (B / W) % 2)
    return fail(-2, "B=%d must hold an even number of W=%d blocks", B, W);
  if (p->stream_a == p->stream_b) return fail(-2, "two distinct streams needed");
  auto* h = new svdj_dist_handle_t();
  h->rank = p->rank, h->world = p->world, h->dtype = p->dtype, h->W = W, h->m_pad = p->m_pad;
  h->n_v = p->n_v, h->B = B, h->k = B / W, h->hk = h->k / 2, h->hB = h->hk * W;
  h->has_v = p->Vt != nullptr, h->timing = p->comm_timing != 0;
  h->comm = (ncclComm_t)p->comm;
  h->st[0] = (hipStream_t)p->stream_a;
  h->st[1] = (hipStream_t)p->stream_b;
  h->sc = (hipStream_t)p->stream_comm;
  h->es = p->dtype == 1 ? 8 : 4;
  int rc = 0;
  auto guard = [&](int r) {
    if (r < 0 && !rc) rc = r;
  };
  // 3 = auto: by the pairs of a cross step (half super-blocks)
  const int io = p->inner_order == 3 ? svdj_choose_inner_order(p->dtype, W, h->hk) : p->inner_order;
  h->io = io;
  // quad steps from 32 pairs per chain step on any number of GPUs, merged
  // issue on one GPU from 64 pairs (32 with quad steps) -- the Python
  // engine's rules: models/block.py choose_quad, distributed.py merged
  int quad = 0, merged = 0;
  const int dr = svdj_dist_issue_rules(p->world, p->dtype, W, p->mma, h->k, p->m_pad, p->quad,
                                       &quad, &merged);
  if (dr < 0) rc = dr;
  h->quad = quad != 0;
  h->merged = merged != 0;
  if (!rc) guard(build_templates(h, io == 2 ? 3 : (io ? 2 : 0)));
  h->wsb = svdj_block_workspace_bytes(p->dtype, W, h->merged ? h->k : h->k / 2, p->m_pad,
                                      h->quad ? 1 : 0);
  for (int c = 0; c < 2 && !rc; ++c)
    if (hipMalloc(&h->ws[c], h->wsb) != hipSuccess) rc = fail(-100, "hipMalloc(ws %zu) failed", h->wsb);
  if (!rc && hipMalloc((void**)&h->metric, SVDJ_METRIC_WORDS * sizeof(uint32_t)) != hipSuccess)
    rc = fail(-100, "hipMalloc(metric) failed");
  if (p->exchange < 0 || p->exchange > 2) rc = rc ? rc : fail(-2, "exchange %d (0 auto, 1 direct, 2 spread)", p->exchange);
  h->spread = h->world > 2 && (p->exchange == 2 || (p->exchange == 0 && h->world >= 4));
  if (h->spread) {  // chunk rows: ceil(message / (P - 1)) elements
    const size_t msg[2] = {(size_t)h->hB * h->m_pad, h->has_v ? (size_t)h->hB * h->n_v : 0};
    for (int i = 0; i < 2 && !rc; ++i) {
      h->relay_n[i] = (msg[i] + h->world - 2) / (h->world - 1);
      if (msg[i] && hipMalloc(&h->relay[i], h->relay_n[i] * h->world * h->es) != hipSuccess)
        rc = fail(-100, "hipMalloc(relay %zu) failed", h->relay_n[i] * h->world * h->es);
    }
  }
  if (!rc && !h->sc && h->world > 1) {
    if (hipStreamCreateWithFlags(&h->sc, hipStreamNonBlocking) != hipSuccess)
      rc = fail(-100, "comm stream creation failed");
    else
      h->own_sc = true;
  }
  // Measured exchange choice: a collective, so first a go/no-go over ALL
  // ranks (max of the local failure flags; a rank that failed above still
  // takes part), then every rank calibrates or every rank gives up -- a rank
  // that skipped calibration alone would leave its peers blocked in it.
  if (h->world >= 4 && p->exchange == 0 && h->sc) {
    const double tmo = p->timeout_s > 0 ? p->timeout_s : 600.0;
    int32_t* flag = nullptr;
    int32_t any = rc ? 1 : 0;
    if (hipMalloc((void**)&flag, sizeof(int32_t)) != hipSuccess ||
        hipMemcpy(flag, &any, sizeof(any), hipMemcpyHostToDevice) != hipSuccess) {
      rc = rc ? rc : fail(-100, "go/no-go flag: hipMalloc failed");
    } else if (ncclAllReduce(flag, flag, 1, ncclInt32, ncclMax, h->comm, h->sc) != ncclSuccess) {
      rc = rc ? rc : fail(-200, "go/no-go all-reduce failed");
    } else if (int r = poll_stream(h->sc, h->comm, tmo)) {
      rc = rc ? rc : r;
    } else if (hipMemcpy(&any, flag, sizeof(any), hipMemcpyDeviceToHost) != hipSuccess) {
      rc = rc ? rc : fail(-100, "go/no-go flag copy failed");
    } else if (any && !rc) {
      rc = fail(-2, "handle creation failed on another rank: exchange calibration skipped");
    }
    (void)hipFree(flag);
    if (!rc) guard(calibrate_exchange(h, tmo));
  }
  if (rc) {
    handle_free(h);
    return rc;
  }
  *out = h;
  return 0;
}

extern "C" int svdj_dist_handle_destroy(void* handle) {
  handle_free((svdj_dist_handle_t*)handle);
  return 0;
}

namespace {

// The issue plan of one rank on templates (same items / groups as
// sweep_items / issue_groups, which tests compare with the Python plan).
struct TItem {
  bool send = false;
  Template* t = nullptr;
  int stream = 0;
  int round = 0, slot = 0, half = 0;
};

std::vector<TItem> template_items(const Tour& tour, int g, svdj_dist_handle_t* h,
                                  const std::vector<Item>& items) {
  // sweep_items was built on dummy Tasks at fixed addresses: map them back
  std::vector<TItem> out;
  out.reserve(items.size());
  for (const Item& x : items) {
    TItem y;
    y.send = x.send;
    y.stream = x.stream;
    y.round = x.round, y.slot = x.slot, y.half = x.half;
    if (!x.send) {
      // decode the halves: rr tasks touch (s,0),(s,1); cross (inc,ih),(stay,sh)
      const int a = x.hv[0], b = x.hv[1];
      if (a / 2 == b / 2) {
        y.t = &h->rr[a / 2];
      } else {
        y.t = &h->cross[a / 2][a % 2][b % 2];
      }
    }
    out.push_back(y);
  }
  (void)tour;
  (void)g;
  return out;
}

}  // namespace

extern "C" int svdj_dist_solve(svdj_dist_problem* p, void* sigma) {
  svdj_dist_handle_t* h = (svdj_dist_handle_t*)p->handle;
  bool own = false;
  if (!h) {
    void* hh = nullptr;
    if (int r = svdj_dist_handle_create(p, &hh)) return r;
    h = (svdj_dist_handle_t*)hh;
    own = true;
  }
  struct Own {
    svdj_dist_handle_t* h;
    bool own;
    ~Own() {
      if (own) handle_free(h);
    }
  } own_guard{h, own};
  if (h->rank != p->rank || h->world != p->world || h->dtype != p->dtype || h->W != p->W ||
      h->m_pad != p->m_pad || h->n_v != p->n_v || h->B != p->B || h->has_v != (p->Vt != nullptr) ||
      h->comm != (ncclComm_t)p->comm)
    return fail(-2, "handle does not match the problem geometry");
  const int P = h->world, g = h->rank, W = h->W, B = h->B, hB = h->hB;
  const size_t es = h->es;
  hipStream_t* st = h->st;
  hipStream_t sa = st[0], sc = h->sc;
  ncclComm_t comm = h->comm;
  const ncclDataType_t nt = h->dtype == 1 ? ncclFloat64 : ncclFloat32;
  Tour tour(P);

  // issue plan (cached in the handle after the first solve)
  if (h->items.empty()) {
    Task rr_d[2], cross_d[2][2][2];
    h->items = sweep_items(tour, g, rr_d, cross_d);
    h->groups = issue_groups(h->items);
    const unsigned flags = h->timing ? 0 : hipEventDisableTiming;
    h->ev.assign(h->items.size(), nullptr);
    for (auto& e : h->ev) HIPC(hipEventCreateWithFlags(&e, flags));
    if (h->timing) {
      h->ev_start.assign(h->items.size(), nullptr);
      h->ev_ready.assign(2 * h->items.size(), nullptr);
      for (auto* v : {&h->ev_start, &h->ev_ready})
        for (auto& e : *v) HIPC(hipEventCreateWithFlags(&e, 0));
      HIPC(hipEventCreateWithFlags(&h->ev_t0, 0));
    }
    HIPC(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
  }
  const std::vector<TItem> titems = template_items(tour, g, h, h->items);
  const std::vector<Item>& items = h->items;
  const std::vector<Group>& groups = h->groups;
  Layout& L = h->L;
  L = Layout();
  if (P == 1) L.spare[0] = L.spare[1] = -1;

  // placement of every GPU's slots (all ranks simulate the whole table)
  std::vector<int32_t> phys(2 * P);
  for (int r = 0; r < P; ++r) {
    phys[2 * r] = tour.h(0, r, 0);
    phys[2 * r + 1] = tour.h(0, r, 1);
  }
  if (p->held[0] != phys[2 * g] || p->held[1] != phys[2 * g + 1])
    return fail(-2, "rank %d holds (%d, %d), the tournament starts from (%d, %d)", g, p->held[0],
                p->held[1], phys[2 * g], phys[2 * g + 1]);

  Watchdog wd;
  const double timeout = p->timeout_s > 0 ? p->timeout_s : 600.0;
  if (P > 1) wd.start(comm, timeout, g);
  // Wait for stream sa without blocking forever: poll, and give up when the
  // watchdog fired (a dead peer leaves RCCL kernels spinning; the abort
  // releases them and the stream drains).
  auto wait_sa = [&]() -> int {
    for (;;) {
      const hipError_t q = hipStreamQuery(sa);
      if (q == hipSuccess) return 0;
      if (q != hipErrorNotReady) return fail(-100, "stream error: %s", hipGetErrorString(q));
      if (wd.fired.load()) return fail(-300, "%s", wd.why);
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  };
  auto buf_ptr = [&](void* base, size_t ld, int b) { return (char*)base + (size_t)b * hB * ld * es; };
  std::vector<std::pair<double, double>> busy, waits;
  double comm_ms = 0, sweep_base_ms = 0;
  long long n_exch = 0, n_bytes = 0;
  int mma_sweep = p->mma;  // the apply's mode, | 256 for a 2-part quad Gram (below)
  // One sweep: every dependency is an event; the host never waits.
  auto sweep = [&]() -> int {
    std::vector<hipEvent_t> last[4];   // task events on each half since its last exchange
    hipEvent_t pending[4] = {nullptr, nullptr, nullptr, nullptr};  // arrived, not yet waited
    int halves_sent = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> sp_busy, sp_wait, sp_span;
    if (svdj_reset_metric(h->metric, sa) != 0) return fail(-100, "metric reset failed");
    if (h->merged) {  // one GPU: three merged launches on one stream, nothing to wait for
      for (int m = 0; m < 3; ++m)
        SVDJC(svdj_block_steps(h->dtype, W, h->m_pad, p->At, h->m_pad, p->Vt, h->n_v, h->n_v, p->D,
                               h->merged_pairs + h->merged_off[m], h->merged_np[m],
                               h->merged_steps[m], h->merged_modes[m].data(), p->tol, p->tol_mode,
                               1, h->ws[0], h->wsb, h->metric, mma_sweep, sa));
      return 0;
    }
    if (h->timing) HIPC(hipEventRecord(h->ev_t0, sa));
    HIPC(hipEventRecord(h->ev_join, sa));
    HIPC(hipStreamWaitEvent(st[1], h->ev_join, 0));
    if (sc) HIPC(hipStreamWaitEvent(sc, h->ev_join, 0));
    for (const Group& gr : groups) {
      const Item& a = items[gr.a];
      if (a.send) {  // one half of slot a.slot to send_to, its replacement from recv_from
        const int key = a.slot * 2 + a.half;
        const int out_b = L.loc[a.slot][a.half], in_b = L.spare[a.half];
        for (hipEvent_t e : last[key]) HIPC(hipStreamWaitEvent(sc, e, 0));
        last[key].clear();
        if (h->timing) HIPC(hipEventRecord(h->ev_start[gr.a], sc));
        std::unique_lock<std::mutex> lk(wd.mu);
        if (wd.fired.load()) return fail(-300, "%s", wd.why);
        // messages in the order of pipeline.py: A half, norms, V half
        XMsg msgs[3];
        int nm = 0;
        msgs[nm++] = {buf_ptr(p->At, h->m_pad, out_b), buf_ptr(p->At, h->m_pad, in_b),
                      (size_t)hB * h->m_pad, h->spread ? (char*)h->relay[0] : nullptr, h->relay_n[0]};
        msgs[nm++] = {(char*)p->D + (size_t)out_b * hB * es, (char*)p->D + (size_t)in_b * hB * es,
                      (size_t)hB, nullptr, 0};
        if (p->Vt)
          msgs[nm++] = {buf_ptr(p->Vt, h->n_v, out_b), buf_ptr(p->Vt, h->n_v, in_b),
                        (size_t)hB * h->n_v, h->spread ? (char*)h->relay[1] : nullptr,
                        h->relay_n[1]};
        ++n_exch;
        for (int i = 0; i < nm; ++i) n_bytes += (long long)msgs[i].n * (long long)es;
        if (int r = exchange_ops(tour, a.round, g, msgs, nm, h->spread, nt, es, comm, sc)) return r;
        lk.unlock();
        // received in place: from here on (issue order) the half lives in in_b;
        // in_b's last readers were waited for by the exchange that freed it
        L.loc[a.slot][a.half] = in_b;
        L.spare[a.half] = out_b;
        hipEvent_t arrived = h->ev[gr.a];
        HIPC(hipEventRecord(arrived, sc));
        if (h->timing) sp_span.push_back({h->ev_start[gr.a], arrived});
        pending[key] = arrived;
        if (++halves_sent % 2 == 0) {  // both halves of round a.round issued: new placement
          std::vector<int32_t> old = phys;
          for (int r = 0; r < P; ++r) {
            const int sh = tour.from(a.round, r);
            phys[2 * r + tour.x(a.round, r)] = old[2 * sh + tour.x(a.round, sh)];
          }
        }
        continue;
      }
      const int n_t = gr.b < 0 ? 1 : 2;
      const int idx[2] = {gr.a, gr.b};
      for (int q = 0; q < n_t; ++q) {
        const Item& x = items[idx[q]];
        hipStream_t s = st[x.stream];
        int nready = 0;
        for (int hv : x.hv) {
          for (hipEvent_t e : last[hv]) HIPC(hipStreamWaitEvent(s, e, 0));
          if (pending[hv]) {
            if (h->timing) {
              hipEvent_t r = h->ev_ready[2 * idx[q] + nready++];
              HIPC(hipEventRecord(r, s));
              sp_wait.push_back({r, pending[hv]});
            }
            HIPC(hipStreamWaitEvent(s, pending[hv], 0));
            pending[hv] = nullptr;
          }
        }
        if (h->timing) HIPC(hipEventRecord(h->ev_start[idx[q]], s));
      }
      auto dev_pairs = [&](const TItem& ti) {
        const Template& t = *ti.t;
        const int ba = L.loc[t.hv[0] / 2][t.hv[0] % 2], bb = L.loc[t.hv[1] / 2][t.hv[1] % 2];
        return t.dev[ba][bb];
      };
      for (int q = 0; q < n_t; ++q) {  // one chain, or two issued independently
        const TItem& z = titems[idx[q]];
        const int cz = z.stream;
        SVDJC(svdj_block_steps(h->dtype, W, h->m_pad, p->At, h->m_pad, p->Vt, h->n_v, h->n_v, p->D,
                               dev_pairs(z), z.t->npairs, z.t->steps, z.t->modes.data(), p->tol,
                               p->tol_mode, 1, h->ws[cz], h->wsb, h->metric,
                               mma_sweep | (h->quad ? 512 : 0), st[cz]));  // bit 9: chains share the GPU
      }
      for (int q = 0; q < n_t; ++q) {
        const Item& x = items[idx[q]];
        hipEvent_t e = h->ev[idx[q]];
        HIPC(hipEventRecord(e, st[x.stream]));
        if (h->timing) sp_busy.push_back({h->ev_start[idx[q]], e});
        for (int hv : x.hv) last[hv].push_back(e);
      }
    }
    HIPC(hipEventRecord(h->ev_join, st[1]));
    HIPC(hipStreamWaitEvent(sa, h->ev_join, 0));
    if (sc) {
      HIPC(hipEventRecord(h->ev_join, sc));
      HIPC(hipStreamWaitEvent(sa, h->ev_join, 0));
    }
    if (h->timing) {  // diagnostics: resolve this sweep's events now
      if (int r = wait_sa()) return r;
      auto t = [&](hipEvent_t e) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, h->ev_t0, e);
        return (double)ms;
      };
      for (auto& x : sp_busy) busy.push_back({t(x.first) + sweep_base_ms, t(x.second) + sweep_base_ms});
      for (auto& x : sp_wait) waits.push_back({t(x.first) + sweep_base_ms, t(x.second) + sweep_base_ms});
      for (auto& x : sp_span) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, x.first, x.second);
        comm_ms += ms;
      }
      sweep_base_ms += 1e7;  // sweeps never overlap: keep their intervals apart
    }
    return 0;
  };

  int rc = 0;
  p->sweeps = 0;
  p->converged = 0;
  // negligible-column floor of the block EVDs (block.hip needs_rotation),
  // relative to the largest squared column norm: local value, then the max
  // over ranks (the floor is monotone in that norm)
  if (svdj_set_norm_floor_scaled(h->dtype, h->m_pad, p->D, 2 * p->B, h->metric, sa) < 0)
    return fail(-100, "norm floor: %s", svdj_hip_last_error());
  if (P > 1 &&
      ncclAllReduce(h->metric + 2, h->metric + 2, 1, ncclFloat64, ncclMax, comm, sa) != ncclSuccess)
    return fail(-200, "norm floor all-reduce failed");
  p->inner_order_used = h->io;
  p->exchange_used = P > 1 ? (h->spread ? 2 : 1) : 0;
  p->quad_used = h->quad ? 1 : 0;
  p->merged_used = h->merged ? 1 : 0;
  p->calib_direct_ms = h->calib_ms[0];
  p->calib_spread_ms = h->calib_ms[1];
  const auto t_solve = std::chrono::steady_clock::now();
  // Quad Gram precision per sweep (parallel/distributed.py, the same rule):
  // 2 bf16 parts (svdj_block_steps' mma bit 8) while the previous sweep
  // rotated every pair; SVDJ_DEBUG gram2=0/1 forces it off / on (A/B).
  const long long nbt = 2LL * P * h->k, all_pairs = nbt * (nbt - 1) / 2;
  const int gram2 = svdj_debug_knob("gram2", -1);
  bool prev_all = true;
  for (int sw = 0; sw < p->max_sweeps && !rc; ++sw) {
    mma_sweep = p->mma | ((h->quad && (gram2 < 0 ? prev_all : gram2 == 1)) ? 256 : 0);
    if ((rc = sweep())) break;
    // ---- stop test (svdj_stop.h): global max convergence value and largest
    // applied |sin| (positive floats order as uint32), total rotated pairs
    uint32_t hm[6] = {0, 0, 0, 0, 0, 0};
    auto reduce = [&]() -> int {
      {
        std::lock_guard<std::mutex> lk(wd.mu);
        if (wd.fired.load()) return fail(-300, "%s", wd.why);
        if (P > 1) {  // one GPU (comm may be NULL): the local words are the global ones
          NCCLC(ncclAllReduce(h->metric, h->metric, 1, ncclUint32, ncclMax, comm, sa));
          NCCLC(ncclAllReduce(h->metric + 1, h->metric + 1, 1, ncclUint32, ncclSum, comm, sa));
          NCCLC(ncclAllReduce(h->metric + 4, h->metric + 4, 1, ncclUint32, ncclMax, comm, sa));
          NCCLC(ncclAllReduce(h->metric + 5, h->metric + 5, 1, ncclUint32, ncclSum, comm, sa));
        }
      }
      HIPC(hipMemcpyAsync(hm, h->metric, sizeof(hm), hipMemcpyDeviceToHost, sa));
      return wait_sa();
    };
    if ((rc = reduce())) break;
    if (wd.fired.load()) {
      rc = fail(-300, "%s", wd.why);
      break;
    }
    wd.progress();
    float mx, ms;
    memcpy(&mx, &hm[0], sizeof(float));
    memcpy(&ms, &hm[4], sizeof(float));
    prev_all = (long long)hm[1] >= all_pairs;
    if (p->hist) p->hist[sw] = mx;
    p->sweeps = sw + 1;
    if (p->progress && g == 0) {
      const double el =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t_solve).count();
      fprintf(stderr,
              "[svdj_dist] sweep %d: off %.3e, eff sin %.3e, rotated pairs %u, rotations %u, %.2f s\n",
              sw + 1, (double)mx, (double)ms, hm[1], hm[5], el);
      fflush(stderr);
    }
    if (p->fault_rank == g && p->fault_sweep == sw + 1) {
      fprintf(stderr, "[svdj_dist] fault injection: rank %d exits after sweep %d\n", g, sw + 1);
      fflush(stderr);
      _exit(17);
    }
    const int conv =
        svdj_sweep_converged_inline(mx, ms, hm[1], hm[5], p->tol, p->tol_mode, p->stop_rule);
    if (conv) {
      p->converged = conv;
      break;
    }
  }
  if (!rc) {
    // halves back home (rows [sB, (s+1)B) = slot s), then U and sigma
    for (auto& mv : moves_to_canonical(L)) {
      const size_t src = (size_t)mv.first, dst = (size_t)mv.second;
      rc = rc ? rc : (hipMemcpyAsync(buf_ptr(p->At, h->m_pad, dst), buf_ptr(p->At, h->m_pad, src),
                                     (size_t)hB * h->m_pad * es, hipMemcpyDeviceToDevice, sa) != hipSuccess
                          ? fail(-100, "canonicalise copy failed") : 0);
      if (!rc && p->Vt &&
          hipMemcpyAsync(buf_ptr(p->Vt, h->n_v, dst), buf_ptr(p->Vt, h->n_v, src),
                         (size_t)hB * h->n_v * es, hipMemcpyDeviceToDevice, sa) != hipSuccess)
        rc = fail(-100, "canonicalise copy failed");
      if (!rc && hipMemcpyAsync((char*)p->D + dst * hB * es, (char*)p->D + src * hB * es, hB * es,
                                hipMemcpyDeviceToDevice, sa) != hipSuccess)
        rc = fail(-100, "canonicalise copy failed");
    }
    p->held[0] = phys[2 * g];
    p->held[1] = phys[2 * g + 1];
    if (!rc && sigma) {
      const int r2 = svdj_finalize(h->dtype, p->At, h->m_pad, h->m_pad, 2 * B, sigma, 1, sa);
      if (r2 < 0) rc = fail(r2, "finalize: %s", svdj_hip_last_error());
    }
    if (!rc) rc = wait_sa();
  }
  wd.join();
  if (rc == -300 || wd.fired.load()) {
    p->comm = nullptr;  // aborted: the caller must not destroy it
    if (!rc) rc = fail(-300, "%s", wd.why);
  } else if (rc) {
    (void)hipDeviceSynchronize();  // nothing of this call may still run on its buffers
  }
  p->exchanges = n_exch;
  p->bytes_sent = n_bytes;
  if (h->timing) {
    p->comm_ms = comm_ms;
    p->exposed_comm_ms = exposed_time(waits, busy);
  }
  return rc;
}
