"""Distributed block one-sided Jacobi (one process per GPU).

Reference: ``omp_mpi_cuda_dgesvd_local_matrices`` (reference main.cu:440-1423)
splits every Sameh step's pairs across MPI ranks and has rank 0 scatter the
needed columns of A and V to every worker and gather them back EVERY step
(main.cu:582-680, 854-936; 2 TB of host-staged traffic per sweep at n=5000).

MI355X design:

* owner-computes: the n columns are cut into 2P super-blocks of B columns;
  GPU g permanently holds two of them (A and V columns + tracked squared
  norms) in HBM;
* a sweep is a 2P-1 round tournament over super-blocks (every pair meets
  once); between rounds each GPU sends exactly ONE super-block to one peer
  and receives one (grouped RCCL send/recv over xGMI) -- see
  ``schedule.tournament``;
* inside a round, the GPU orthogonalises its two resident super-blocks with
  the MFMA block kernels: round 0 runs a full round robin over its 2k
  W-blocks (covering all within-super-block pairs once per sweep), later
  rounds run the k-step bipartite cross schedule;
* the stop test is an all-reduce (max off value, sum of rotations) per sweep.

Input is root-owned like the reference (rank 0 passes A, which is scattered
once), or generated in place per rank (``generator``) for large synthetic
benchmarks.  Output is gathered to rank 0 (``gather=True``) in the
reference's layout, or left distributed.
"""
from __future__ import annotations

import os
import sys
import time

import torch

from ..config import SolverConfig, SVDOptions, debug_knob
from ..models.base import SVDResult, Solver
from ..models import precondition as pre
from ..models.block import (choose_block, choose_mma, quad_size_rule, resolve_inner_order,
                            resolve_quad)
from ..ops import kernels as K
from ..utils import checkpoint as ckpt
from ..utils.layout import pad_rows, round_up
from ..utils.tracing import trace_range
from .comm import Communicator
from .pipeline import PipelineExecutor, sweep_plan
from .schedule import distributed_sweep_plan, tournament


def choose_merged(P: int, k: int, quad: bool) -> bool:
    """One-GPU merged issue (PipelineExecutor.run_merged) for k W-blocks per
    super-block: from 64 pairs per chain step; with quad steps from 16 to 31
    pairs (measured: see the comment at its use in
    DistributedBlockJacobi._solve).  The
    reference's single-process path rotates one pair per launch
    (main.cu:727-758); this is the opposite end: all of a step's pairs of
    both chains in one launch.
    On one GPU only, in both engines; SVDJ_DEBUG merge=0/1 overrides there
    (config.debug_knob).  libsvdj_dist: svdj_dist_issue_rules."""
    if P != 1:
        return False
    force = debug_knob("merge")
    if force is not None:
        return force == 1
    hk = k // 2
    return 16 <= hk < 32 if quad else hk >= 64


class DistributedBlockJacobi(Solver):
    name = "distributed-block"

    def __init__(self, config: SolverConfig | None = None, comm: Communicator | None = None):
        super().__init__(config)
        if self.config.chains not in (1, 2):
            raise ValueError(f"SolverConfig.chains must be 1 (blocking exchange) or 2 "
                             f"(pipelined), got {self.config.chains}")
        self.comm = comm or Communicator()
        self._ws = {}  # this solver's kernel workspaces (never shared with another solver)

    # ------------------------------------------------------------ geometry
    def geometry(self, m: int, n: int, dtype: torch.dtype):
        P = self.comm.world
        W = self.config.block or choose_block(dtype, max(n // max(P, 1), 1), m)
        K.check_block(dtype, W)
        # pipelined sweeps split super-blocks in halves: k = B/W must be even
        parts = 2 if self.config.chains == 2 else 1
        q = 2 * parts * P * W
        ncols = round_up(max(n, q), q)
        m_pad = pad_rows(m)
        # quad steps need k % 4 == 0: a pipelined fp32/bf16 W = 64 count that
        # lands on k % 4 == 2 where the quad rule holds takes one more q of
        # zero columns (<= 6 % more columns there; quad steps save 20-25 % of
        # a solve).  Same rule as libsvdj_dist's svdj_dist_geometry.
        k = ncols // (2 * P * W)
        if parts == 2 and dtype != torch.float64 and W == 64 and k % 4 == 2 \
                and quad_size_rule((k + 2) // 2, m_pad, P) and debug_knob("quad_pad", 1) != 0:
            ncols += q
        B = ncols // (2 * P)
        return {"P": P, "W": W, "ncols": ncols, "B": B, "k": B // W, "m_pad": m_pad,
                "n_v": pad_rows(ncols)}

    # --------------------------------------------------------------- solve
    _DT_CODE = {torch.float32: 0, torch.float64: 1, torch.bfloat16: 2}

    def solve(self, A: torch.Tensor | None = None, jobu=SVDOptions.AllVec,
              jobv=SVDOptions.AllVec, m: int | None = None, n: int | None = None,
              dtype: torch.dtype | None = None, generator=None, gather: bool = True,
              time_only: bool = False) -> SVDResult:
        """Distributed SVD.  ``dtype`` is the problem precision (fp32, fp64 or
        bf16 = bf16 data on fp32 master copies and bf16 matrix cores).  Tall
        inputs (m >= qr_ratio n, or precondition="qr") are QR-preconditioned
        with a row-distributed CholeskyQR2 (``precondition.dist_qr``: local
        Gram, RCCL all-reduce, replicated Cholesky, local TRSM); the sweeps
        then run on the replicated R (n x n) and U = Q U_R is a local GEMM
        per row block.  That path returns U as this rank's row block
        (``info["u_rows"]``) with sigma and V complete on every rank, or U
        complete on rank 0 with ``gather``."""
        comm, cfg = self.comm, self.config
        dev = comm.device
        jobu, jobv = SVDOptions.parse(jobu), SVDOptions.parse(jobv)
        # ---- problem description (root-owned input is broadcast as shape)
        if A is not None:
            m, n = A.shape
            dtype = dtype or cfg.dtype or A.dtype
        dtype = dtype or cfg.dtype or torch.float32
        if dtype not in self._DT_CODE:
            dtype = torch.float32
        hdr = torch.tensor([m or 0, n or 0, self._DT_CODE[dtype]], dtype=torch.int64, device=dev)
        if generator is None and comm.distributed:
            comm.broadcast(hdr, 0)
        m, n = int(hdr[0]), int(hdr[1])
        dtype = {0: torch.float32, 1: torch.float64, 2: torch.bfloat16}[int(hdr[2])]
        if m < n:
            raise ValueError("distributed path expects m >= n")
        work = torch.float64 if dtype == torch.float64 else torch.float32
        if not pre.use_qr(cfg, m, n):
            res = self._solve(A, jobu, jobv, m, n, dtype, generator, gather, time_only)
            res.info["flops"] = pre.flops(m, n, res.sweeps, False)
            return res
        # ---- QR-preconditioned tall-skinny solve, row-distributed: rank g
        # owns rows [r0, r1) of A and of U; R (n x n) is replicated
        P, g = comm.world, comm.rank
        r0, r1 = g * m // P, (g + 1) * m // P
        t_qr = time.perf_counter()
        if generator is not None:
            A_loc = torch.cat([generator(c0, min(c0 + 1024, n))[r0:r1].to(device=dev, dtype=work)
                               for c0 in range(0, n, 1024)], dim=1)
        else:
            A_loc = self._scatter_rows(A, m, n, work)
        out = pre.dist_qr(A_loc, work, comm)
        if out is None:  # too ill-conditioned for CholeskyQR2: replicated Householder
            Qf, R = pre.qr(self._allgather_rows(A_loc, m, n), work, method="householder")
            Q_loc, Lt = Qf[r0:r1].contiguous(), None
            del Qf
        else:
            Q_loc, R, Lt = out
        del A_loc
        if cfg.comm_timing and dev.type == "cuda":  # phase timing costs a sync
            torch.cuda.synchronize(dev)
        t_qr = time.perf_counter() - t_qr
        res = self._solve(None, jobu, jobv, n, n, dtype, lambda c0, c1: R[:, c0:c1], False,
                          time_only)
        want_u = jobu != SVDOptions.NoVec
        U_R, S, V = self._allgather_columns(res, n, want_u, jobv != SVDOptions.NoVec)
        U_loc = pre.apply_q(Q_loc, Lt, U_R).to(U_R.dtype) if want_u else None
        res.S, res.V = S, V
        res.info.update(precondition="qr", flops=pre.flops(m, n, res.sweeps, True),
                        qr_seconds=round(t_qr, 4),
                        distributed_output="rows" if P > 1 and not gather else False,
                        u_rows=(r0, r1))
        if gather and P > 1 and want_u:
            U_loc = self._gather_rows(U_loc, m, n)
        res.U = U_loc
        if dtype == torch.bfloat16 and (gather or P == 1):
            res.U = res.U.to(torch.bfloat16) if res.U is not None else None
            res.V = res.V.to(torch.bfloat16) if res.V is not None else None
        return res

    # -------------------------------------------------- row-distributed QR I/O
    def _row_range(self, h: int, m: int):
        P = self.comm.world
        return h * m // P, (h + 1) * m // P

    def _scatter_rows(self, A, m, n, dtype):
        """Root-owned A: rank 0 sends every rank its row block (one grouped batch)."""
        comm = self.comm
        r0, r1 = self._row_range(comm.rank, m)
        if not comm.distributed:
            return A.to(device=comm.device, dtype=dtype)
        if comm.rank == 0:
            Ad = A.to(device=comm.device, dtype=dtype)
            sends = [(Ad[self._row_range(h, m)[0]:self._row_range(h, m)[1]].contiguous(), h)
                     for h in range(1, comm.world)]
            comm.sendrecv(sends, [])
            return Ad[r0:r1].contiguous()
        out = torch.empty(r1 - r0, n, dtype=dtype, device=comm.device)
        comm.sendrecv([], [(out, 0)])
        return out

    def _allgather_rows(self, A_loc, m, n):
        """Every rank's row block, assembled on every rank (Householder fallback)."""
        comm = self.comm
        if not comm.distributed:
            return A_loc
        rows = max(self._row_range(h, m)[1] - self._row_range(h, m)[0] for h in range(comm.world))
        buf = torch.zeros(rows, n, dtype=A_loc.dtype, device=A_loc.device)
        buf[:A_loc.shape[0]] = A_loc
        allr = comm.allgather(buf)
        return torch.cat([allr[h, :self._row_range(h, m)[1] - self._row_range(h, m)[0]]
                          for h in range(comm.world)])

    def _gather_rows(self, U_loc, m, n):
        """Row blocks of U to rank 0 (one grouped batch); None on other ranks."""
        comm = self.comm
        if comm.rank != 0:
            comm.sendrecv([(U_loc.contiguous(), 0)], [])
            return None
        parts = [U_loc]
        recvs = []
        for h in range(1, comm.world):
            a, b = self._row_range(h, m)
            t = torch.empty(b - a, n, dtype=U_loc.dtype, device=U_loc.device)
            parts.append(t)
            recvs.append((t, h))
        comm.sendrecv([], recvs)
        return torch.cat(parts)

    def _allgather_columns(self, res, n, want_u, want_v):
        """All of U_R (n x n), sigma (n) and V (n x n) on every rank, from each
        rank's resident super-block columns (transposed layout)."""
        comm = self.comm
        geo = res.info["geometry"]
        B = geo["B"]
        held = torch.tensor(res.info["held"], dtype=torch.int64, device=res.S.device)
        ids = comm.allgather(held).cpu()
        S_all = comm.allgather(res.S)
        U_all = comm.allgather(res.U) if want_u else None
        V_all = comm.allgather(res.V) if want_v else None
        ncols = 2 * B * comm.world
        S = torch.zeros(ncols, dtype=res.S.dtype, device=res.S.device)
        Ut = torch.zeros(ncols, n, dtype=res.S.dtype, device=res.S.device) if want_u else None
        Vt = torch.zeros(ncols, n, dtype=res.S.dtype, device=res.S.device) if want_v else None
        for h in range(comm.world):
            for s_ in range(2):
                sb = int(ids[h, s_])
                dst, src = slice(sb * B, (sb + 1) * B), slice(s_ * B, (s_ + 1) * B)
                S[dst] = S_all[h, src]
                if want_u:
                    Ut[dst] = U_all[h, src, :n]
                if want_v:
                    Vt[dst] = V_all[h, src, :n]
        return (Ut[:n].t() if want_u else None), S[:n], (Vt[:n].t() if want_v else None)

    def _solve(self, A, jobu, jobv, m, n, pdtype, generator, gather, time_only) -> SVDResult:
        comm, cfg = self.comm, self.config
        dev = comm.device
        dtype = torch.float64 if pdtype == torch.float64 else torch.float32
        bf16 = pdtype == torch.bfloat16
        geo = self.geometry(m, n, dtype)
        P, W, B, k, m_pad, n_v, ncols = (geo[x] for x in ("P", "W", "B", "k", "m_pad", "n_v", "ncols"))
        mma = cfg.mma if cfg.mma != "auto" else ("bf16x3" if bf16 else choose_mma(dtype, W))
        g = comm.rank
        tour = tournament(P)
        pipelined = cfg.chains == 2
        quad = pipelined and resolve_quad(cfg.quad, dtype, W, mma, k, P, m_pad)
        if pipelined:
            splan = sweep_plan(P, k, tour.xslot[:, g], quad=quad)
        else:
            plans = distributed_sweep_plan(P, k)
            dev_pairs = [torch.from_numpy(p.pairs).to(dev) for p in plans]
        streams = self._chain_streams(dev) if (pipelined and dev.type == "cuda") else None

        # ---- resident state: slot s holds super-block held[s]
        # phys[h][s] = super-block physically resident in slot s of GPU h; every
        # rank simulates the whole table (exchanges are deterministic).
        phys = [[int(tour.held[0, h, 0]), int(tour.held[0, h, 1])] for h in range(P)]
        held = phys[g]
        # pipelined multi-rank storage carries one spare half buffer per half
        # index (the exchanges receive in place, pipeline.HalfLayout); rows
        # [0, 2B) are the canonical slots at the start and after the solve
        ncol_store = PipelineExecutor.storage_columns(B, comm.distributed) if pipelined else 2 * B
        At = torch.zeros(ncol_store, m_pad, dtype=dtype, device=dev)
        want_v = jobv != SVDOptions.NoVec
        Vt = torch.zeros(ncol_store, n_v, dtype=dtype, device=dev) if want_v else None
        self._distribute(A, generator, At, held, m, n, B, dtype)
        if want_v:
            for s in range(2):
                K.set_identity(Vt[s * B:(s + 1) * B], B, held[s] * B)
        D = K.col_norms2(At, m_pad)
        tol = self.tolerance(pdtype, m)
        # pairs per cross step: half super-blocks (pipelined) or whole ones
        inner = resolve_inner_order(cfg.inner_order, W, k // 2 if pipelined else k, dtype)
        if pipelined:
            rA = rV = rD = None
        else:  # blocking exchange (chains=1) receives into a staging block
            rA = torch.empty(B, m_pad, dtype=dtype, device=dev)
            rV = torch.empty(B, n_v, dtype=dtype, device=dev) if want_v else None
            rD = torch.empty(B, dtype=dtype, device=dev)
        metric = K.new_metric(dev)
        # scale of the negligible-column floor: the largest squared column norm
        # of the whole matrix (one all-reduce at setup)
        dmax = float(D[:2 * B].max()) if D.numel() else 1.0
        if comm.distributed:
            dmax = comm.max_over_ranks(dmax)
        K.set_norm_floor(metric, dtype, m_pad, dmax)
        comm.barrier()

        hist, t_comm, t_total = [], 0.0, 0.0
        sweeps = 0
        stop_reason = None
        start = 0
        sig = {"m": m, "n": n, "dtype": str(dtype), "P": P, "W": W, "B": B, "rank": g,
               "want_v": want_v}
        if cfg.checkpoint_dir:
            st = ckpt.load(cfg.checkpoint_dir, g, dev)
            if st is not None and ckpt.compatible(st, sig):
                At[:2 * B].copy_(st["At"])
                D[:2 * B].copy_(st["D"])
                if want_v:
                    Vt[:2 * B].copy_(st["Vt"])
                phys = [list(x) for x in st["phys"]]
                held = phys[g]
                hist = list(st["hist"])
                start = sweeps = int(st["sweep"])
        sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
        sync()
        t0 = time.perf_counter()
        converged = False
        bufs = (rA, rV, rD)
        # work actually done by the quad kernels (bench.py's executed-MFMA and
        # HBM estimates): device counters of the apply, summed per sweep without
        # a host sync, and the quad Grams issued
        work = {"gram_quads": 0, "gram_quads2": 0}
        gram_parts = [3]  # bf16 parts of this sweep's quad Grams (set per sweep below)
        shared_gpu = [False]  # two chains issued concurrently (set with `merged` below)
        work_acc = torch.zeros(2, dtype=torch.float64, device=metric.device)
        if pipelined:
            ex = PipelineExecutor(comm, streams, At, Vt, D, k, W, tour, timing=cfg.comm_timing,
                                  parts=splan.parts, exchange=cfg.exchange)

            def run_steps(pairs, modes, slot):
                # quads of the quad steps issued (each runs the quad Gram): host count
                nq = sum(1 for x in modes if int(x) == 4) * (pairs.shape[1] // 2)
                work["gram_quads"] += nq
                work["gram_quads2"] += nq if gram_parts[0] == 2 else 0
                K.block_steps(At, Vt, D, m_pad, pairs, W, modes, tol, cfg.max_inner_sweeps,
                              metric, slot, mma=mma, pool=self._ws, tol_mode=cfg.tol_mode,
                              inner_order=inner, gram_parts=gram_parts[0],
                              shared_gpu=shared_gpu[0])
        # One rank, no exchanges, >= 64 pairs per chain step (>= 32 with quad
        # steps): the two chains' parallel tasks merged into single launches
        # of twice the pairs (PipelineExecutor.run_merged), the EVD latency
        # paid once per step (profiles/r4_merge; from 64 pairs bitwise the
        # two-chain solve, the Gram keeps the chunking).  Single steps of 32
        # pairs keep the overlapped chains (8192^2 merged +10 %); quad steps
        # of 32 pairs merge well (12288^2 1747 -> 1677 ms, 8192^2 per sweep
        # 39.4 -> 36.9 ms, profiles/r5_quad2), and so do quad steps of 16
        # pairs (4096^2 135.4 -> 123.5 ms, profiles/r6_issue).  Since the quad
        # apply leaves the concurrent chain CUs (profiles/r6_grid), the two
        # chains beat merging again from 32 quad pairs: 16384^2 3169-3187 ->
        # 3034 ms (same 19 sweeps, bitwise the same result), 8192^2 30.4 ->
        # 29.5 ms per sweep; 4096^2 (16 pairs) still merges, 110 vs 120 ms
        # (profiles/r6_merge).  SVDJ_DEBUG merge=0/1
        # overrides; with exchanges merging was slower at every P (round 6,
        # 16384^2 P = 8: 51.9 ms per sweep merged, 50.6 merged with quad
        # steps, 43.1 not merged; profiles/r6_issue/plan_p8).
        merged = pipelined and dev.type == "cuda" and choose_merged(P if comm.distributed else 1,
                                                                    k, quad)
        # the two chains on their own streams: the quad apply leaves the other
        # chain CUs (svdj_block_steps bit 9; libsvdj_dist the same)
        shared_gpu[0] = pipelined and quad and not (merged and not comm.distributed)
        # Quad Gram precision per sweep: while the previous sweep rotated
        # every pair (far from convergence: the first ~12 of 19 sweeps at
        # 16384^2), the couplings only steer rotation angles and the 2-part
        # Gram (~2^-16) does; later sweeps need the exact one
        # (profiles/r6_gram2; libsvdj_dist: the same rule in svdj_dist_solve).
        # SVDJ_DEBUG gram2=0/1 forces it off / on (A/B).
        nbt = 2 * P * k
        all_pairs = nbt * (nbt - 1) // 2
        gram2 = debug_knob("gram2")
        prev_all = start == 0
        for sw in range(start, cfg.max_sweeps):
            use2 = prev_all if gram2 is None else gram2 == 1
            gram_parts[0] = 2 if (quad and use2) else 3
            with trace_range(f"svdj.sweep{sw}"):
                K.reset_metric(metric)
                if pipelined and merged and not comm.distributed:
                    ex.run_merged(splan, run_steps)
                elif pipelined:
                    t_comm += ex.run(splan, run_steps, phys, merge=merged)
                    held = phys[g]
                for r in range(0 if not pipelined else tour.rounds, tour.rounds):
                    if r > 0 and P > 1:
                        tc = time.perf_counter()
                        with trace_range("svdj.exchange"):
                            self._exchange(tour, r, phys, At, Vt, D, bufs, B)
                        held = phys[g]
                        t_comm += time.perf_counter() - tc
                    with trace_range(f"svdj.round{r}"):
                        K.block_steps(At, Vt, D, m_pad, dev_pairs[r], W, plans[r].modes, tol,
                                      cfg.max_inner_sweeps, metric, mma=mma, pool=self._ws,
                                      tol_mode=cfg.tol_mode, inner_order=inner)
                mx, ms, nrot, ncr = self._reduce_metric(metric, dev)
                prev_all = int(nrot) >= all_pairs
                work_acc += K.metric_work(metric)
            hist.append(mx)
            sweeps = sw + 1
            if cfg.progress and g == 0:
                print(f"[svdj] sweep {sweeps}: off {mx:.3e}, eff sin {ms:.3e}, rotated pairs "
                      f"{int(nrot)}, rotations {int(ncr)}, {time.perf_counter() - t0:.2f} s",
                      file=sys.stderr, flush=True)
            # every rank sees the same all-reduced values: the same decision
            stop = K.sweep_converged(mx, ms, nrot, ncr, tol, cfg.tol_mode, cfg.stop_rule)
            if stop:
                converged = True
                stop_reason = "no_rotation" if stop == 1 else "second_order"
                break
            # The next sweep replays the same exchange pattern from the current
            # placement: the schedule only depends on positions, so every
            # physical pair still meets exactly once per sweep.
            if cfg.checkpoint_dir and cfg.checkpoint_every and sweeps % cfg.checkpoint_every == 0:
                if pipelined:
                    ex.canonicalize()
                ckpt.save(cfg.checkpoint_dir, g,
                          {**sig, "At": At[:2 * B], "Vt": Vt[:2 * B] if want_v else torch.empty(0),
                           "D": D[:2 * B], "phys": phys, "hist": hist, "sweep": sweeps})
            self._fault_point(sweeps)
        if converged and cfg.checkpoint_dir:
            ckpt.clear(cfg.checkpoint_dir, g)
        if pipelined:
            ex.canonicalize()
            At, D = At[:2 * B], D[:2 * B]
            Vt = Vt[:2 * B] if want_v else None
        sigma_loc = K.finalize(At, m_pad, scale_u=jobu != SVDOptions.NoVec)
        sync()
        t_total = time.perf_counter() - t0
        wa = work_acc.cpu()
        info_work = {"apply_mfma": int(wa[0]) * 24, "apply_tiles": int(wa[1]),
                     "gram_quads": int(work["gram_quads"]),
                     "gram_quads2": int(work["gram_quads2"]), "m_pad": m_pad}
        info = {"tol": tol, "converged": converged, "stop_reason": stop_reason, "work": info_work,
                "stop_rule": cfg.stop_rule, "dtype": str(pdtype), "geometry": geo, "mma": mma,
                "inner_order": inner, "quad": quad, "merged_chains": bool(pipelined and merged),
                "exchange": ex.exchange if pipelined else "direct",
                "comm_seconds": t_comm, "rank": g, "held": list(held)}
        if pipelined and P > 1:
            info["comm"] = ex.comm_summary()
        if time_only or not gather:
            return SVDResult(At if jobu != SVDOptions.NoVec else None, sigma_loc, Vt, sweeps, hist,
                             t_total, self.name, {**info, "distributed_output": True})
        U, S, V = self._gather(At, Vt, sigma_loc, held, m, n, B, dtype, want_v,
                               jobu != SVDOptions.NoVec)
        if bf16:  # bf16 in/out (sigma stays fp32)
            U = U.to(torch.bfloat16) if U is not None else None
            V = V.to(torch.bfloat16) if V is not None else None
        return SVDResult(U, S, V, sweeps, hist, t_total, self.name, info)

    def _fault_point(self, sweeps: int):
        """Fault injection for failure-detection tests: SolverConfig.extra
        ["fault_exit"] = (rank, sweep) makes that rank exit abruptly (no
        cleanup, exit status 17) after that sweep, like a crashed peer."""
        f = self.config.extra.get("fault_exit") if self.config.extra else None
        if f and int(f[0]) == self.comm.rank and int(f[1]) == sweeps:
            print(f"[svdj] fault injection: rank {self.comm.rank} exits after sweep {sweeps}",
                  file=sys.stderr, flush=True)
            import os
            os._exit(17)

    _STREAMS: dict = {}  # device -> the two chain streams, shared by every solver in the process

    def _chain_streams(self, dev):
        """The chain streams are created ONCE per device and process and
        reused by every solver (each svd() call builds a new one): torch
        hands out pool streams round robin, and HIP binds each new stream to
        one of GPU_MAX_HW_QUEUES (4) hardware queues, so fresh streams per
        solve can land on the same queue as each other and serialise.
        Solves in one process are sequential, so sharing is safe."""
        key = str(dev)
        if key not in DistributedBlockJacobi._STREAMS:
            DistributedBlockJacobi._STREAMS[key] = [torch.cuda.Stream(dev) for _ in range(2)]
        return DistributedBlockJacobi._STREAMS[key]

    # ------------------------------------------------------- data movement
    def _exchange(self, tour, r, phys, At, Vt, D, bufs, B):
        """Round r of the tournament: this GPU sends the super-block in slot
        xslot[r][g] (A columns, V columns, squared norms) to send_to[r][g] and
        receives its replacement from recv_from[r][g] -- one grouped RCCL
        send/recv.  ``phys`` (every GPU's placement) is updated in place."""
        g, P = self.comm.rank, self.comm.world
        rA, rV, rD = bufs
        x = int(tour.xslot[r, g])
        dst, src = int(tour.send_to[r, g]), int(tour.recv_from[r, g])
        sl = slice(x * B, (x + 1) * B)
        sends = [(At[sl], dst), (D[sl], dst)]
        recvs = [(rA, src), (rD, src)]
        if Vt is not None:
            sends.append((Vt[sl], dst))
            recvs.append((rV, src))
        # gloo on device tensors (rehearsal) is not stream-ordered, see pipeline.py
        host_sync = At.is_cuda and not getattr(self.comm, "async_device", False)
        if host_sync:
            torch.cuda.synchronize(At.device)
        self.comm.sendrecv(sends, recvs)
        if host_sync:
            torch.cuda.synchronize(At.device)
        At[sl].copy_(rA)
        D[sl].copy_(rD)
        if Vt is not None:
            Vt[sl].copy_(rV)
        old = [[phys[h][0], phys[h][1]] for h in range(P)]
        for h in range(P):
            src_h = int(tour.recv_from[r, h])
            phys[h][int(tour.xslot[r, h])] = old[src_h][int(tour.xslot[r, src_h])]

    def _reduce_metric(self, metric, dev):
        """Global (max off value, max effective sine, rotated pairs, column
        rotations) of the sweep (all-reduces instead of the reference's
        discarded convergence value, main.cu:710)."""
        v = K.metric_stop_values(metric)
        return self.comm.allreduce_stop(v[0], v[1], v[2], v[3])

    def _distribute(self, A, generator, At, held, m, n, B, dtype):
        comm = self.comm
        if generator is not None:
            for s in range(2):
                c0, c1 = held[s] * B, min((held[s] + 1) * B, n)
                if c1 > c0:
                    cols = generator(c0, c1)  # (m, c1-c0)
                    At[s * B:s * B + (c1 - c0), :m].copy_(cols.t())
            return
        if not comm.distributed:
            for s in range(2):
                c0, c1 = held[s] * B, min((held[s] + 1) * B, n)
                if c1 > c0:
                    At[s * B:s * B + (c1 - c0), :m].copy_(A[:, c0:c1].t())
            return
        # Root-owned input: rank 0 packs every rank's two super-blocks and
        # posts all P-1 sends as ONE grouped batch, so the transfers run
        # concurrently over the P-1 xGMI links (the reference's scatter is a
        # serial loop of blocking sends, main.cu:582-619).
        tour = tournament(comm.world)
        if comm.rank == 0:
            Ad = A.to(device=At.device, dtype=At.dtype)
            sends = []
            for dst in range(comm.world):
                buf = torch.zeros_like(At[:2 * B]) if dst != 0 else At
                for s in range(2):
                    sb = int(tour.held[0, dst, s])
                    c0, c1 = sb * B, min((sb + 1) * B, n)
                    if c1 > c0:
                        buf[s * B:s * B + (c1 - c0), :m].copy_(Ad[:, c0:c1].t())
                if dst != 0:
                    sends.append((buf, dst))
            comm.sendrecv(sends, [])
        else:
            comm.sendrecv([], [(At[:2 * B], 0)])

    def roundtrip(self, A: torch.Tensor | None, m: int, n: int, dtype=torch.float64):
        """Scatter root-owned A over the ranks' resident super-blocks and gather
        it back unchanged (rank 0 returns the (m, n) matrix, others None).

        The reference names this check ``test_local_matrix_distribution_*``
        and has the round-trip comparisons commented out
        (reference main.cu:630-643, 866-877, 1605-1609); here it is a method
        the tests call."""
        comm = self.comm
        geo = self.geometry(m, n, dtype)
        B, m_pad = geo["B"], geo["m_pad"]
        held = [int(tournament(comm.world).held[0, comm.rank, s]) for s in range(2)]
        At = torch.zeros(2 * B, m_pad, dtype=dtype, device=comm.device)
        self._distribute(A, None, At, held, m, n, B, dtype)
        sigma = torch.zeros(2 * B, dtype=dtype, device=comm.device)
        U, _, _ = self._gather(At, None, sigma, held, m, n, B, dtype, False, True)
        return U

    def _gather(self, At, Vt, sigma, held, m, n, B, dtype, want_v, want_u):
        comm = self.comm
        ids = torch.tensor(held, dtype=torch.int64, device=At.device)
        if not comm.distributed:
            parts = [(ids, At, Vt, sigma)]
        elif comm.rank == 0:
            # all P-1 ranks' blocks arrive in one grouped batch (concurrent
            # links; the reference gathers rank by rank, main.cu:854-936)
            parts = [(ids, At, Vt, sigma)]
            recvs = []
            for src in range(1, comm.world):
                rid = torch.empty_like(ids)
                rA, rS = torch.empty_like(At), torch.empty_like(sigma)
                rV = torch.empty_like(Vt) if want_v else None
                recvs += [(rid, src), (rA, src), (rS, src)] + ([(rV, src)] if want_v else [])
                parts.append((rid, rA, rV, rS))
            comm.sendrecv([], recvs)
        else:
            sends = [(ids, 0), (At, 0), (sigma, 0)] + ([(Vt, 0)] if want_v else [])
            comm.sendrecv(sends, [])
            return None, None, None
        ncols = 2 * B * comm.world
        Ut = torch.zeros(ncols, m, dtype=dtype, device=At.device)
        Vfull = torch.zeros(ncols, Vt.shape[1], dtype=dtype, device=At.device) if want_v else None
        S = torch.zeros(ncols, dtype=dtype, device=At.device)
        for rid, a, v, s_ in parts:
            for s in range(2):
                sb = int(rid[s])
                Ut[sb * B:(sb + 1) * B] = a[s * B:(s + 1) * B, :m]
                S[sb * B:(sb + 1) * B] = s_[s * B:(s + 1) * B]
                if want_v:
                    Vfull[sb * B:(sb + 1) * B] = v[s * B:(s + 1) * B]
        U = Ut[:n].t() if want_u else None
        V = Vfull[:n, :n].t() if want_v else None
        return U, S[:n], V
