// Native distributed solver (C ABI): one process per GPU, RCCL over xGMI.
//
// The reference's distributed solver is a C++ entry point driven by its
// native binary (reference main.cu:440-448 omp_mpi_cuda_dgesvd_local_matrices,
// driven from main.cu:1587; lib/JacobiMethods.cuh:44-52).  This is the
// MI355X-native equivalent without Python: the super-block tournament of
// svdj_tournament (2P super-blocks, 2P-1 rounds, one super-block exchanged
// per GPU per round), the block steps of libsvdj_hip on two staggered chains,
// and an RCCL all-reduce of the sweep's convergence value and rotation count
// as the stop test.  The exchange is pipelined as in parallel/pipeline.py:
// each super-block moves in two halves with grouped ncclSend/ncclRecv on a
// comm stream as soon as the tasks touching that half are done, and consumers
// wait on the arrival event -- the host never blocks inside a sweep.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Communicator bootstrap through a file: rank 0 creates the RCCL unique id
// and publishes it at `id_path` (atomic rename); the other ranks wait for it
// (up to timeout_s).  The caller has selected the rank's device first.
// *comm receives an ncclComm_t.  Returns 0 or <0.
int svdj_dist_comm_init(int rank, int world, const char* id_path, double timeout_s, void** comm);
int svdj_dist_comm_destroy(void* comm);

// Geometry of an m x n problem (m >= n) on `world` GPUs with block width W:
// n is padded to ncols = a multiple of 4*world*W columns, cut into 2*world
// super-blocks of B columns (B/W even); row counts padded to 128.
int svdj_dist_geometry(int world, int m, int n, int W, int* B, int* ncols, int* m_pad, int* n_v);

// Default block width (models/block.py choose_block): fp32 64 when m >= 8192
// and a GPU holds >= 2048 columns, fp64 64 when m >= 12288 and >= 4096
// columns per GPU, else 32.
int svdj_dist_choose_block(int dtype, int world, int m, int n);

// Super-block ids held by `rank` at the start of a sweep (round 0 placement).
int svdj_dist_initial_held(int world, int rank, int32_t held[2]);

typedef struct {
  int rank, world;
  void* comm;                 // ncclComm_t (svdj_dist_comm_init)
  int dtype;                  // 0 fp32, 1 fp64
  int W, m_pad, n_v, B;       // from svdj_dist_geometry
  void* At;                   // (2B, m_pad) transposed columns: slot s = rows [sB, (s+1)B)
  void* Vt;                   // (2B, n_v) or NULL (no V)
  void* D;                    // (2B) squared column norms (svdj_col_norms2)
  int32_t held[2];            // in: svdj_dist_initial_held (the data must be placed so);
                              // out: super-blocks in the two slots after the last sweep
  double tol;
  int tol_mode;               // 0 relative, 1 absolute
  int max_sweeps;
  int mma;                    // matrix-core mode of the apply (svdj_block_steps)
  int inner_order;            // EVD of the cross steps: 0 cyclic, 1 bipartite (mode 2)
  void* stream_a;             // two compute streams (distinct)
  void* stream_b;
  void* stream_comm;          // exchange stream, or NULL (created per call).  HIP maps
                              // streams onto GPU_MAX_HW_QUEUES hardware queues as they
                              // are created: make the three streams first, before RCCL's
                              // own, or two of them may share a queue and serialise.
  double* hist;               // host [max_sweeps]: per-sweep global max convergence value
  int sweeps;                 // out
  int converged;              // out
} svdj_dist_problem;

// Runs sweeps until one applies no rotation anywhere (or max_sweeps), then
// normalises U in place (At rows) and writes sigma[2B] (device, data type).
// Collective: every rank calls it.  Returns 0 or <0 (svdj_dist_last_error()).
int svdj_dist_solve(svdj_dist_problem* p, void* sigma);

// Issue order of one sweep on `rank` (host only, for tests): per group 7 ints
// {kind, ...}: kind 0 = one task {stream, half, half}, 1 = a staggered pair
// {stream, half, half, stream, half, half}, 2 = a half exchange {round, slot,
// half}; halves are slot*2 + half.  Returns the group count (<= cap) or <0.
int svdj_dist_plan(int world, int rank, int32_t* out, int cap);

// Message of the calling thread's last failure.
const char* svdj_dist_last_error(void);

#ifdef __cplusplus
}
#endif
