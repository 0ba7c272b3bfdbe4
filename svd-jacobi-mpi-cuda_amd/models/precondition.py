"""QR preconditioning for tall-skinny problems (m >> n).

The reference only handles square input (main.cu:1452-1453, "we expect here
squared matrix" main.cu:1405); its sweep costs n(n-1)/2 (12m + 6n) flops, so
for m >> n the m-long column updates dominate every sweep.  The standard
remedy (LAPACK xGESVJ/xGEJSV practice) is A = Q R first, Jacobi on the n x n
R, then U = Q U_R: one QR (2mn^2 - 2n^3/3 flops) and one GEMM (2mn^2) buy
sweeps on n-long instead of m-long columns.  The factorisation and the GEMM
are plain library calls on the device (rocSOLVER geqrf / hipBLASLt through
torch); the Jacobi sweeps stay on the framework's kernels.
"""
from __future__ import annotations

import torch

from ..config import SolverConfig
from ..utils.metrics import algorithmic_flops_per_sweep


def use_qr(cfg: SolverConfig, m: int, n: int) -> bool:
    if cfg.precondition == "qr":
        return m > n
    if cfg.precondition == "none":
        return False
    return m >= cfg.qr_ratio * n and n >= 64


def qr(A: torch.Tensor, dtype: torch.dtype, method: str = "auto"):
    """Reduced QR in the working precision on A's device.

    ``cholqr2``: CholeskyQR2 -- twice (G = Q^T Q, G = L L^T, Q <- Q L^-T),
    R = L2^T L1^T.  Everything is GEMM / TRSM shaped (hipBLASLt, rocBLAS)
    and stable while kappa(A)^2 eps < 1.  ``householder``: torch.linalg.qr
    (rocSOLVER geqrf on the GPU, which made QR cost more than it saved at
    32768 x 8192).  ``auto``: CholeskyQR2 on the GPU, Householder if the Gram
    is not numerically positive definite (or on the CPU)."""
    A = A.to(dtype)
    if method in ("auto", "cholqr2") and (A.is_cuda or method == "cholqr2"):
        out = _cholqr2(A)
        if out is not None:
            return out
        if method == "cholqr2":
            raise RuntimeError("CholeskyQR2 failed: Gram not positive definite (ill-conditioned A)")
    Q, R = torch.linalg.qr(A, mode="reduced")
    return Q, R


def _cholqr2(A: torch.Tensor):
    """None when A is too ill-conditioned for CholeskyQR2 (kappa >~ eps^-1/2,
    estimated from the first Cholesky factor's pivots)."""
    eps = torch.finfo(A.dtype).eps
    Q, R = A, None
    for it in range(2):
        L, info = torch.linalg.cholesky_ex(Q.t() @ Q)
        if int(info) != 0 or not bool(torch.isfinite(L).all()):
            return None
        if it == 0:
            d = torch.diagonal(L).abs()
            if float(d.min()) <= eps ** 0.5 * float(d.max()):
                return None
        Q = torch.linalg.solve_triangular(L.t(), Q, upper=True, left=False)  # Q L^-T
        R = L.t() if R is None else L.t() @ R
    return Q, R


def dist_qr(A_loc: torch.Tensor, dtype: torch.dtype, comm):
    """Row-distributed CholeskyQR2: rank g holds rows A_g (m_g x n) of A.

    Twice: G = sum_g Q_g^T Q_g (local GEMM + one n x n all-reduce over
    RCCL), G = L L^T (redundant on every rank: every rank sees the same G),
    Q_g <- Q_g L^-T (local TRSM).  R = L2^T L1^T is replicated, so every rank
    can take its super-blocks of R with no further communication, and Q stays
    row-distributed (U = Q U_R is then a local GEMM per row block).  The QR
    cost is divided by P; the replicated m x n factorisation it replaces
    was redundant work on every rank.

    Returns (Q_g, R), or None when the Gram is not numerically positive
    definite (kappa(A) >~ eps^-1/2) -- the same decision on every rank."""
    Q = A_loc.to(dtype)
    eps = torch.finfo(dtype).eps
    R = None
    for it in range(2):
        G = Q.t() @ Q
        comm.allreduce_sum_(G)
        L, info = torch.linalg.cholesky_ex(G)
        if int(info) != 0 or not bool(torch.isfinite(L).all()):
            return None
        if it == 0:
            d = torch.diagonal(L).abs()
            if float(d.min()) <= eps ** 0.5 * float(d.max()):
                return None
        Q = torch.linalg.solve_triangular(L.t(), Q, upper=True, left=False)  # Q L^-T
        R = L.t() if R is None else L.t() @ R
    return Q, R


def flops(m: int, n: int, sweeps: int, qr_used: bool) -> float:
    """Algorithmic work of a solve: the reference-form sweep count on the
    matrix actually iterated on, plus QR and the U GEMM when preconditioned."""
    if not qr_used:
        return algorithmic_flops_per_sweep(m, n) * sweeps
    return (2.0 * m * n * n - 2.0 * n ** 3 / 3.0) + algorithmic_flops_per_sweep(n, n) * sweeps \
        + 2.0 * m * n * n
