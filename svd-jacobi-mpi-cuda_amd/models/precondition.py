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
    Q1, R, Lt = qr_deferred(A, dtype, method)
    return (Q1, R) if Lt is None else (
        torch.linalg.solve_triangular(Lt, Q1, upper=True, left=False), R)


def qr_deferred(A: torch.Tensor, dtype: torch.dtype, method: str = "auto"):
    """(Q1, R, Lt) with Q = Q1 Lt^-1 (Lt upper triangular n x n, or None when
    Q1 is Q itself).  The solvers never form Q: they only need U = Q U_R =
    Q1 (Lt^-1 U_R) (``apply_q``), so CholeskyQR2's second m x n TRSM becomes
    an n x n one.  Measured on MI355X at 32768 x 8192 fp32
    (tools/qr_breakdown.py, profiles/r3_fusion): the m x n TRSM is 17.5 ms,
    the Gram GEMMs and the U GEMM run at 153 TFLOP/s (97 % of the fp32
    matrix-core peak) in hipBLASLt, the two 8192 Choleskys take 28.8 ms each."""
    A = A.to(dtype)
    if method in ("auto", "cholqr2") and (A.is_cuda or method == "cholqr2"):
        out = _cholqr2(A)
        if out is not None:
            return out
        if method == "cholqr2":
            raise RuntimeError("CholeskyQR2 failed: Gram not positive definite (ill-conditioned A)")
    Q, R = torch.linalg.qr(A, mode="reduced")
    return Q, R, None


def apply_q(Q1: torch.Tensor, Lt, X: torch.Tensor) -> torch.Tensor:
    """Q X for Q = Q1 Lt^-1 (``qr_deferred`` / ``dist_qr``): one n x n
    triangular solve, then the m x n x n GEMM."""
    if Lt is not None:
        X = torch.linalg.solve_triangular(Lt, X.to(Lt.dtype), upper=True)
    return Q1 @ X.to(Q1.dtype)


def _cholqr2(A: torch.Tensor):
    """(Q1, R, L2^T), or None when A is too ill-conditioned for CholeskyQR2
    (kappa >~ eps^-1/2, estimated from the first Cholesky factor's pivots)."""
    eps = torch.finfo(A.dtype).eps
    L1, info = torch.linalg.cholesky_ex(A.t() @ A)
    if int(info) != 0 or not bool(torch.isfinite(L1).all()):
        return None
    d = torch.diagonal(L1).abs()
    if float(d.min()) <= eps ** 0.5 * float(d.max()):
        return None
    Q1 = torch.linalg.solve_triangular(L1.t(), A, upper=True, left=False)  # A L1^-T
    L2, info = torch.linalg.cholesky_ex(Q1.t() @ Q1)
    if int(info) != 0 or not bool(torch.isfinite(L2).all()):
        return None
    return Q1, L2.t() @ L1.t(), L2.t()


def _ordered_sum(G: torch.Tensor, comm) -> torch.Tensor:
    """sum_g G_g added in rank order on every rank (bitwise the same result
    whatever the backend); communicators without it (the one-GPU plan
    simulator's cost model) all-reduce."""
    f = getattr(comm, "ordered_sum_", None)
    return f(G) if f is not None else comm.allreduce_sum_(G)


def dist_qr(A_loc: torch.Tensor, dtype: torch.dtype, comm):
    """Row-distributed CholeskyQR2: rank g holds rows A_g (m_g x n) of A.

    G1 = sum_g A_g^T A_g (local GEMM + one n x n all-reduce over RCCL),
    G1 = L1 L1^T (redundant on every rank: every rank sees the same G1),
    Q1_g = A_g L1^-T (local TRSM), then G2 = sum_g Q1_g^T Q1_g = L2 L2^T the
    same way.  R = L2^T L1^T is replicated, so every rank can take its
    super-blocks of R with no further communication; Q = Q1 L2^-T stays
    row-distributed and unformed (U = Q U_R is ``apply_q`` per row block).
    The QR cost is divided by P; the replicated m x n factorisation it
    replaces was redundant work on every rank.

    The two Gram sums are rank-ordered (all-gather, then G_0 + G_1 + ... on
    every rank): a floating all-reduce adds in an order that depends on the
    backend and the ring (RCCL and gloo differ), which changes R's low bits
    and with them every later bit of the solve.  At BASELINE config 4
    (n = 8192, P = 4) that is 768 MB gathered per rank instead of 384 MB
    all-reduced -- a few ms over xGMI next to a ~180 ms QR.

    Returns (Q1_g, R, L2^T), or None when a Gram is not numerically positive
    definite (kappa(A) >~ eps^-1/2) -- the same decision on every rank."""
    A = A_loc.to(dtype)
    eps = torch.finfo(dtype).eps
    G = _ordered_sum(A.t() @ A, comm)
    L1, info = torch.linalg.cholesky_ex(G)
    if int(info) != 0 or not bool(torch.isfinite(L1).all()):
        return None
    d = torch.diagonal(L1).abs()
    if float(d.min()) <= eps ** 0.5 * float(d.max()):
        return None
    Q1 = torch.linalg.solve_triangular(L1.t(), A, upper=True, left=False)  # A L1^-T
    G = _ordered_sum(Q1.t() @ Q1, comm)
    L2, info = torch.linalg.cholesky_ex(G)
    if int(info) != 0 or not bool(torch.isfinite(L2).all()):
        return None
    return Q1, L2.t() @ L1.t(), L2.t()


def flops(m: int, n: int, sweeps: int, qr_used: bool) -> float:
    """Algorithmic work of a solve: the reference-form sweep count on the
    matrix actually iterated on, plus QR and the U GEMM when preconditioned."""
    if not qr_used:
        return algorithmic_flops_per_sweep(m, n) * sweeps
    return (2.0 * m * n * n - 2.0 * n ** 3 / 3.0) + algorithmic_flops_per_sweep(n, n) * sweeps \
        + 2.0 * m * n * n
