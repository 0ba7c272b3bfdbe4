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


def qr(A: torch.Tensor, dtype: torch.dtype):
    """Reduced QR in the working precision on A's device."""
    Q, R = torch.linalg.qr(A.to(dtype), mode="reduced")
    return Q, R


def flops(m: int, n: int, sweeps: int, qr_used: bool) -> float:
    """Algorithmic work of a solve: the reference-form sweep count on the
    matrix actually iterated on, plus QR and the U GEMM when preconditioned."""
    if not qr_used:
        return algorithmic_flops_per_sweep(m, n) * sweeps
    return (2.0 * m * n * n - 2.0 * n ** 3 / 3.0) + algorithmic_flops_per_sweep(n, n) * sweeps \
        + 2.0 * m * n * n
