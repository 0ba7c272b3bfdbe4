"""Single-device block one-sided Jacobi on MFMA (the performance path).

On a GPU the solve runs the distributed engine's plan at P = 1 (see
choose_engine); the "steps" engine is the plain form: per sweep a round
robin over nb = n/W column blocks, each step the gram -> LDS EVD -> apply
kernel chain of csrc/hip/block.hip on nb/2 disjoint block pairs.  Replaces the reference's per-pair host dot products + Givens
kernel (reference main.cu:685-852, 139-147) with matrix-core work on blocks
resident in HBM.
"""
from __future__ import annotations

import torch

from ..config import SVDOptions
from ..ops import kernels as K
from ..utils.layout import pack_columns, pad_rows, round_up
from .base import SVDResult, Solver, Timer


def choose_block(dtype: torch.dtype, n: int, m: int) -> int:
    """Block width W for ``n`` columns per GPU of ``m`` rows.

    W=64 halves the steps and the per-byte traffic of the Gram and the apply,
    but its EVD is slower and a step holds half as many pairs.  Since the
    low-latency cross EVD (choose_inner_order "cross" for W=64 steps,
    round 3) the W=64 EVD no longer dominates small problems, and
    W=64 wins almost everywhere.  Measured on MI355X, round 3
    (profiles/r3_blockw), W=32 / W=64:
      * fp32, 1 GPU n x n, ms per solve: 512 15.7 / 12.1, 1024 21.5 / 21.1,
        2048 50.3 / 41.6, 3072 102 / 92, 4096 162 / 149, 6144 454 / 390;
      * fp32 rank plans, ms per sweep: 8192^2 P=8 (1024 columns per GPU)
        20.0 / 15.2, P=4 23.0 / 22.3; 4096^2 P=2 10.9 / 8.6, P=8 (512
        columns) 10.0 / 12.4; 2048^2 P=4 (512) 4.9 / 4.4;
      * fp64, 1 GPU, ms per solve: 5000 516 / 559, 6144 926 / 884, 8192
        2420 / 2063, 10000 3917 / 3583; rank plans, ms per sweep: 5000^2
        P=2 (2500 columns) 22.9 / 25.1, 10000^2 P=2 147 / 126, 16384^2 P=8
        (2048 columns) 164 / 141.
    Rule: fp32 W=64 from 1024 columns per GPU; fp64 W=64 from m >= 6144 rows
    and 2048 columns per GPU (the fp64 W=64 EVD keeps a 2x larger G in LDS).
    """
    if dtype == torch.float64:
        return 64 if (m >= 6144 and n >= 2048) else 32
    return 64 if n >= 1024 else 32


def choose_inner_order(W: int, pairs_per_step: int, dtype: torch.dtype = torch.float32) -> str:
    """EVD ordering of the cross steps for ``pairs_per_step`` pairs of W-wide
    blocks per step (config inner_order="auto").

    "cross" (evd_cross_kernel + qbuild_kernel: a low-latency EVD that
    tracks only the cross couplings, Q built row-parallel by a second kernel)
    for fp32 W=64 steps and fp64 W=64 steps with more than 16 pairs;
    "bipartite" (one workgroup per pair, Q in registers) otherwise.  Measured on MI355X, 16384^2 fp32 rank plans, ms per sweep
    bipartite / cross, with the f32-MFMA apply (profiles/r3_evd): P=8 (8
    pairs) 59.1 / 51.0, P=4 (16) 112.5 / 108.1, P=2 (32) 201.5 / 202.4; with
    the split-bf16 apply, whose shorter steps expose the EVD more
    (profiles/r3_s3/inner): P=2 177.0 / 171.0, 1 GPU (64 pairs) 341.2 /
    341.1; 8192^2 P=2 27.8 / 25.7.  W=32: 8192^2 P=8 20.0 / 22.1.  fp64 (f64-MFMA
    apply, larger LDS image in the cross EVD): 16384^2 P=8 (16 pairs) 127.8 /
    140.3, 10000^2 P=2 (20 pairs) 126.0 / 121.4, 10000^2 1 GPU (39 pairs) 184 /
    175 ms per sweep."""
    if W != 64:
        return "bipartite"
    return "cross" if (dtype != torch.float64 or pairs_per_step > 16) else "bipartite"


def choose_mma(dtype: torch.dtype, W: int) -> str:
    """Matrix-core mode of the apply for mma="auto" (svdj_choose_mma).

    fp32 W=64 steps run on bf16 matrix cores with a 3-way operand split
    ("bf16x6": 6 exact bf16 products per fp32 product, dropped terms below
    2^-26, delta form Y = X + X(Q - I) with the identity added in fp32).
    Measured on MI355X against the f32 MFMA apply (profiles/r3_s3/bf16x6):
    the same residual, U/V orthogonality and sigma error at 512..16384, and
    per sweep 16384^2 1 GPU 392 -> 346 ms, 12288^2 2.57 -> 2.12 s per solve,
    rank plans P=4 108 -> 83 ms and P=2 200 -> 178 ms per sweep, P=8 equal.
    W=32 steps (small problems per GPU) keep the f32 MFMA: 4096^2 P=8 rank
    plan 8.55 vs 9.61 ms per sweep.  fp64 always uses f64 MFMA."""
    return "bf16x6" if (dtype == torch.float32 and W == 64) else "native"


def quad_supported(dtype: torch.dtype, W: int, mma: str, k: int) -> bool:
    """Quad steps exist for fp32 W=64 with the split-bf16 apply and k
    (blocks per super-block) a multiple of 4."""
    return dtype == torch.float32 and W == 64 and mma in ("bf16x6", "bf16x3") and k % 4 == 0


def quad_size_rule(hk: int, m_pad: int, P: int) -> bool:
    """Size part of choose_quad (hk = pairs per chain step), shared with the
    geometry's padding (DistributedBlockJacobi.geometry; libsvdj_dist
    quad_size_rule).  ``m_pad`` no longer enters (round 6, see choose_quad)."""
    del m_pad
    return hk >= 16 or (hk >= 12 and P > 1)


def choose_quad(dtype: torch.dtype, W: int, mma: str, k: int, P: int, m_pad: int = 0) -> bool:
    """Quad steps for config quad="auto", on any number of GPUs: when a chain
    step holds >= 16 pairs (k // 2 >= 16), or >= 12 on more than one GPU;
    off below (quad_size_rule).

    Measured on MI355X with the round-5 kernels (one-read split-bf16 quad
    Gram with a swizzled raw image, a wide chunk reduction when it has many
    row chunks, T-stationary persistent K = 256 apply, vectorised Gram-space
    update; profiles/r5_quad2, ms per solve or per full-work sweep, quad on
    vs off): 1 GPU 16384^2 3.44-3.62 vs 4.70 s, 8192^2 637 vs 685 ms; rank
    plans with 32 pairs per step: 16384^2 P=2 137 vs 165, 32768^2 P=4 449 vs
    596, 65536^2 P=8 1749 vs 2112; with 16 pairs: 16384^2 P=4 78.3 vs 85.0,
    32768^2 P=8 223 vs 324, but 8192^2 P=2 28.5 vs 27.7 and 4096^2 on one GPU
    158 vs 136 ms (short columns: the longer EVD chain is exposed); with 8
    pairs quad steps lose (16384^2 P=8 57 vs 43).  Round 6 (profiles/r6_issue):
    on ONE GPU with 16 pairs the quad steps win once the two chains are
    merged into single launches (choose_merged) -- 4096^2 123.5 ms merged quad
    vs 127.1 merged single steps vs 135.4 two chains -- so there the row rule
    does not apply; 16384^2 P=8 (8 pairs) stays without: 52.8 ms per sweep
    quad, 50.6 merged-with-exchanges quad, 51.9 merged single, 43.1 default.
    Round 6, after the quad apply left the concurrent chain CUs
    (profiles/r6_grid, profiles/r6_rule; simulated plans, ms per sweep, quad
    vs single): 8192^2 P=2 (16 pairs) 23.6 vs 26.6, 12288^2 P=2 (24) 55.4 vs
    73.8, 12288^2 P=4 (12) 34.7 vs 41.0 -- the row condition is gone; with 8
    pairs 16384^2 P=8 43.3 vs 43.1, 4096^2 P=2 9.05 vs 8.98, 8192^2 P=4 16.6
    vs 17.5: still off there."""
    if not quad_supported(dtype, W, mma, k):
        return False
    return quad_size_rule(k // 2, m_pad, P)


def resolve_quad(mode: str, dtype: torch.dtype, W: int, mma: str, k: int, P: int,
                 m_pad: int = 0) -> bool:
    if mode == "off":
        return False
    if mode == "on":
        if not quad_supported(dtype, W, mma, k):
            raise ValueError(f"quad steps need fp32, W=64, a split-bf16 apply and k % 4 == 0 "
                             f"(dtype={dtype}, W={W}, mma={mma}, k={k})")
        return True
    return choose_quad(dtype, W, mma, k, P, m_pad)


def resolve_inner_order(order: str, W: int, pairs_per_step: int,
                        dtype: torch.dtype = torch.float32) -> str:
    return choose_inner_order(W, pairs_per_step, dtype) if order == "auto" else order


def choose_engine(cfg, device: torch.device) -> str:
    """Single-device engine of :class:`BlockJacobi` (``SolverConfig.extra
    ["engine"]``, default "auto"):

    * "pipeline" -- the distributed engine's plan at P = 1
      (:class:`parallel.DistributedBlockJacobi` on a world-1
      ``Communicator.local``): two step chains on two streams, quad steps and
      the merged one-GPU issue where they pay.  This is what ``bench.py``
      times, so ``svd(A)`` gets the headline engine (the public
      entry point ran the older single-stream round robin, ~35 % slower at
      16384^2);
    * "steps" -- ``svdj_block_solve``: one stream, round-robin single steps
      (the reference's sweep structure, main.cu:685-852, on block kernels).

    "auto" is "pipeline" on a GPU and "steps" on the CPU (the CPU emulation
    of the kernels runs either; the pipeline plan is the one the multi-rank
    CPU tests rehearse)."""
    eng = (cfg.extra or {}).get("engine", "auto")
    if eng not in ("auto", "pipeline", "steps"):
        raise ValueError(f"engine must be auto, pipeline or steps, got {eng!r}")
    if eng == "auto":
        return "pipeline" if device.type == "cuda" else "steps"
    return eng


class BlockJacobi(Solver):
    name = "block"

    def _solve_pipeline(self, A, jobu, jobv, device) -> SVDResult:
        from dataclasses import replace

        from ..parallel.comm import Communicator
        from ..parallel.distributed import DistributedBlockJacobi

        cfg = self.config
        # api.svd has already QR-preconditioned tall inputs: the pipeline runs
        # on what it is given
        solver = DistributedBlockJacobi(replace(cfg, precondition="none"),
                                        Communicator.local(device))
        res = solver.solve(A, jobu, jobv)
        geo = res.info["geometry"]
        res.info.update(block=geo["W"], bf16=cfg.bf16_mode(A), device=str(device),
                        engine="pipeline")
        res.method = self.name
        return res

    def solve(self, A, jobu=SVDOptions.AllVec, jobv=SVDOptions.AllVec, device=None) -> SVDResult:
        cfg = self.config
        jobu, jobv = SVDOptions.parse(jobu), SVDOptions.parse(jobv)
        device = torch.device(device) if device is not None else A.device
        if A.shape[0] >= A.shape[1] and choose_engine(cfg, device) == "pipeline":
            return self._solve_pipeline(A, jobu, jobv, device)
        dtype = cfg.resolved_dtype(A)
        bf16 = cfg.bf16_mode(A)
        m, n = A.shape
        if m < n:
            raise ValueError("block path expects m >= n (api.svd transposes wide inputs)")
        W = cfg.block or choose_block(dtype, n, m)
        K.check_block(dtype, W)
        mma = cfg.resolved_mma(A, W)
        ncols = max(round_up(n, 2 * W), 2 * W)
        m_pad, n_v = pad_rows(m), pad_rows(ncols)
        At = pack_columns(A, dtype, device, ncols, m_pad)
        want_v = jobv != SVDOptions.NoVec
        Vt = torch.zeros(ncols, n_v, dtype=dtype, device=device) if want_v else None
        if want_v:
            K.set_identity(Vt, ncols)
        tol = self.tolerance(cfg.precision_dtype(A), m)
        with Timer(device) as tm:
            D = K.col_norms2(At, m_pad)
            inner = resolve_inner_order(cfg.inner_order, W, ncols // (2 * W), dtype)
            sweeps, hist = K.block_solve(At, Vt, D, m_pad, W, tol, cfg.max_inner_sweeps,
                                         cfg.max_sweeps, mma=mma, tol_mode=cfg.tol_mode,
                                         inner_order=inner, stop_rule=cfg.stop_rule)
            S = K.finalize(At, m_pad, scale_u=jobu != SVDOptions.NoVec)
        U = At[:n, :m].t() if jobu != SVDOptions.NoVec else None
        V = Vt[:n, :n].t() if want_v else None
        if bf16:  # bf16 in/out; sigma stays fp32
            U = U.to(torch.bfloat16) if U is not None else None
            V = V.to(torch.bfloat16) if V is not None else None
        conv = sweeps < cfg.max_sweeps or (hist and hist[-1] <= tol)
        return SVDResult(U, S[:n], V, sweeps, hist, tm.seconds, self.name,
                         {"tol": tol, "converged": bool(conv), "dtype": str(dtype), "block": W,
                          "mma": mma, "bf16": bf16,
                          "device": str(device), "engine": "steps"})
