// Native distributed solver (C ABI): one process per GPU, RCCL over xGMI.
//
// The reference's distributed solver is a C++ entry point driven by its
// native binary (reference main.cu:440-448 omp_mpi_cuda_dgesvd_local_matrices,
// driven from main.cu:1587; lib/JacobiMethods.cuh:44-52).  This is the
// MI355X-native equivalent without Python: the super-block tournament of
// svdj_tournament (2P super-blocks, 2P-1 rounds, one super-block exchanged
// per GPU per round), the block steps of libsvdj_hip on two chains, and an
// RCCL all-reduce of the sweep's convergence value and rotation count as the
// stop test.  The exchange is pipelined as in parallel/pipeline.py: each
// super-block moves in two halves with grouped ncclSend/ncclRecv on a comm
// stream as soon as the tasks touching that half are done, received in place
// into a spare half buffer (from 4 GPUs relayed over all xGMI links), and
// consumers wait on the arrival event -- the host never blocks inside a sweep.  A watchdog thread aborts the
// communicator on an RCCL async error or when no sweep finishes in time.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Communicator bootstrap through a file (the role of the reference's
// MPI_Init / MPI_Comm_rank, main.cu:1680-1694): rank 0 creates the RCCL
// unique id and publishes it at `id_path` (atomic rename); the other ranks
// wait for it (up to timeout_s).  The caller has selected the rank's device first.
// *comm receives an ncclComm_t.  Returns 0 or <0.
int svdj_dist_comm_init(int rank, int world, const char* id_path, double timeout_s, void** comm);
// Its host part (no RCCL): rank 0 publishes the n-byte id (n = sizeof
// ncclUniqueId) with this job's token (SVDJ_JOB_TOKEN, or TORCHELASTIC_RUN_ID
// + TORCHELASTIC_RESTART_COUNT); other ranks accept only a fresh file (younger
// than timeout_s with a token, 30 s without) carrying the same token.
int svdj_dist_id_file(int rank, const char* id_path, double timeout_s, void* blob, size_t n);
int svdj_dist_comm_destroy(void* comm);

// Geometry of an m x n problem (m >= n) on `world` GPUs with block width W:
// n is padded to ncols = a multiple of 4*world*W columns, cut into 2*world
// super-blocks of B columns (B/W even); row counts padded to 128.  dtype 0
// fp32, 1 fp64, 2 bf16: outside fp64, at W = 64, a count that would give
// k = B/W % 4 == 2 where the quad-step size rule holds is padded by one more
// 4*world*W so that quad steps (k % 4 == 0) can run.
int svdj_dist_geometry(int world, int m, int n, int W, int dtype, int* B, int* ncols, int* m_pad,
                       int* n_v);

// Default block width (models/block.py choose_block): fp32 64 when a GPU
// holds >= 1024 columns, fp64 64 when m >= 6144 and >= 2048 columns per GPU,
// else 32.
int svdj_dist_choose_block(int dtype, int world, int m, int n);

// Super-block ids held by `rank` at the start of a sweep (round 0 placement).
int svdj_dist_initial_held(int world, int rank, int32_t held[2]);

// Rows of At / Vt / entries of D a rank allocates for super-blocks of B
// columns: 2B on one GPU, 3B with exchanges -- the two extra half buffers
// are the receive spares (exchanges receive in place, no copy-in).  Rows
// [0, 2B) hold slot 0 | slot 1 before and after svdj_dist_solve.
int svdj_dist_storage_cols(int world, int B);

typedef struct {
  int rank, world;
  void* comm;                 // ncclComm_t (svdj_dist_comm_init)
  int dtype;                  // 0 fp32, 1 fp64
  int W, m_pad, n_v, B;       // from svdj_dist_geometry
  void* At;                   // (svdj_dist_storage_cols, m_pad) transposed columns:
                              // slot s = rows [sB, (s+1)B) on entry and on return
  void* Vt;                   // (svdj_dist_storage_cols, n_v) or NULL (no V)
  void* D;                    // (svdj_dist_storage_cols) squared column norms
  int32_t held[2];            // in: svdj_dist_initial_held (the data must be placed so);
                              // out: super-blocks in the two slots after the last sweep
  double tol;
  int tol_mode;               // 0 relative, 1 absolute
  int max_sweeps;
  int mma;                    // matrix-core mode of the apply (svdj_block_steps)
  int inner_order;            // EVD of the cross steps: 0 cyclic, 1 bipartite (mode 2),
                              // 2 cross-only bipartite (mode 3), 3 auto
                              // (svdj_choose_inner_order of the half super-block pairs)
  int exchange;               // half super-block transfer: 0 auto (from 4 ranks both are
                              // timed on the job's links when the handle is created and
                              // spread is kept only if >= 10 % faster, as
                              // pipeline.calibrate_exchange), 1 direct (one grouped
                              // send/recv, one xGMI link), 2 spread (P-1 chunks relayed over
                              // all links in two grouped phases, parallel/spread.py)
  void* stream_a;             // two compute streams (distinct)
  void* stream_b;
  void* stream_comm;          // exchange stream, or NULL (created by the handle).  HIP maps
                              // streams onto GPU_MAX_HW_QUEUES hardware queues as they
                              // are created: make the three streams first, before RCCL's
                              // own, or two of them may share a queue and serialise.
  double timeout_s;           // watchdog: no finished sweep for this long, or an RCCL
                              // async error -> ncclCommAbort and return -300 (<= 0: 600 s)
  int comm_timing;            // 1: timing events on every exchange and task
  int fault_rank, fault_sweep;  // test hook: that rank _exit(17)s after that sweep (-1: off)
  void* handle;               // svdj_dist_handle_create, or NULL (one per call)
  double* hist;               // host [max_sweeps]: per-sweep global max convergence value
  int sweeps;                 // out
  int converged;              // out
  double comm_ms;             // out (comm_timing): sum of exchange spans
  double exposed_comm_ms;     // out (comm_timing): time some compute stream waited for an
                              // arrival while no task ran on either compute stream
  long long exchanges;        // out: half exchanges issued by this rank (timing or not)
  long long bytes_sent;       // out: bytes this rank sent in them (relay hops excluded)
  int progress;               // 1: rank 0 prints one line per sweep on stderr
  int inner_order_used;       // out: the resolved EVD order (0 cyclic, 1 bipartite, 2 cross)
  int exchange_used;          // out: the resolved exchange (1 direct, 2 spread)
  int stop_rule;              // 1: a sweep also ends the iteration by the second-order rule
                              // (svdj_stop.h; relative mode); 0: only a sweep without
                              // rotations does.  converged (out) = 1 (no rotation) or 2
  int quad;                   // quad steps (two cross steps fused, fp32 W = 64 split-bf16
                              // apply): 0 auto (>= 32 pairs per chain step, 16 on columns of
                              // >= 16384 rows, any number of GPUs: models/block.py
                              // choose_quad), 1 on, 2 off
  int quad_used;              // out
  int merged_used;            // out: 1 = one GPU, the two chains issued as single launches of
                              // twice the pairs (pipeline.run_merged; >= 64 pairs per chain step)
  double calib_direct_ms;     // out: exchange calibration (exchange auto from 4 GPUs, at
  double calib_spread_ms;     // handle creation): max over ranks of one half exchange, or 0
} svdj_dist_problem;

// Persistent per-rank state for repeated solves of one geometry: workspaces,
// metric, every device pair list of the plan (for each placement of the
// halves), events and the comm stream -- allocated once, so a solve
// allocates nothing.  Reads rank, world, comm, dtype, W, m_pad, n_v, B,
// Vt (NULL or not), the streams and comm_timing from *p.  On one GPU comm may
// be NULL (no RCCL call is made at world 1).  From 4 ranks with exchange auto
// it is collective (go/no-go flag, then the exchange calibration, both
// polled against timeout_s); -300: a peer died or hung and the communicator
// was aborted -- it must not be destroyed.
int svdj_dist_handle_create(const svdj_dist_problem* p, void** handle);
int svdj_dist_handle_destroy(void* handle);

// Runs sweeps until one applies no rotation anywhere (or max_sweeps), then
// normalises U in place (At rows) and writes sigma[2B] (device, data type).
// Collective: every rank calls it.  Returns 0 or <0 (svdj_dist_last_error());
// -300: the watchdog aborted the communicator (a peer died or hung) -- the
// communicator is then unusable and must not be destroyed.
int svdj_dist_solve(svdj_dist_problem* p, void* sigma);

// Issue order of one sweep on `rank` (host only, for tests): per group 7 ints
// {kind, ...}: kind 0 = one task {stream, half, half}, 1 = a joint pair
// {stream, half, half, stream, half, half}, 2 = a half exchange {round, slot,
// half}; halves are slot*2 + half.  Returns the group count (<= cap) or <0.
int svdj_dist_plan(int world, int rank, int32_t* out, int cap);

// Issue rules of a rank with k W-blocks per super-block (host only): quad
// steps (quad_mode 0 auto / 1 on / 2 off; auto = from 32 pairs per chain
// step, or 16 on columns of >= 16384 rows; fp32 W = 64 split-bf16 apply,
// k % 4 == 0) and, on one GPU, the
// merged issue (from 64 pairs per chain step, 32 with quad steps;
// SVDJ_DEBUG merge=0/1 overrides, svdj_debug.h) -- models/block.py choose_quad and
// parallel/distributed.py choose_merged.  Returns 0 or <0.
int svdj_dist_issue_rules(int world, int dtype, int W, int mma, int k, int m_pad, int quad_mode,
                          int* quad, int* merged);

// One-GPU merged issue (host only, for tests): the pair lists of the three
// merged task groups of a sweep with k blocks per super-block (rr0+rr1,
// T00+T11, T01+T10; local block ids), concatenated step by step; modes[] the
// step modes of each group in turn, meta[3][3] {offset, steps, pairs/step}.
// Returns the number of ints written to pairs, or <0.
int svdj_dist_merged_lists(int k, int quad, int cross_mode, int32_t* pairs, int pcap,
                           int32_t* modes, int mcap, int32_t* meta);

// Message of the calling thread's last failure.
const char* svdj_dist_last_error(void);

#ifdef __cplusplus
}
#endif
