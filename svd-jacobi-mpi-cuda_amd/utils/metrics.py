"""Verification metrics and flop accounting.

The reference checks only ||A - U S V^T||_F (reference main.cu:1641-1665),
which is vacuous for one-sided Jacobi (A V V^T = A for any orthogonal V,
SURVEY.md section 6.3).  :func:`verify` adds orthogonality of U and V and
sigma against an independent oracle.
"""
from __future__ import annotations

import math

import torch


def algorithmic_flops_per_sweep(m: int, n: int) -> float:
    """Work of one scalar sweep as the reference does it: n(n-1)/2 pairs x
    (6m dot triple + 6m A rotation + 6n V rotation)."""
    return n * (n - 1) / 2.0 * (12.0 * m + 6.0 * n)


def gflops(m: int, n: int, sweeps: int, seconds: float) -> float:
    return algorithmic_flops_per_sweep(m, n) * sweeps / max(seconds, 1e-12) / 1e9


def block_mfma_flops_per_sweep(m: int, n: int, W: int) -> float:
    """Matrix-core flops the block path issues per sweep (cross-Gram form):
    per block pair 2mW^2 (Gram) + 8mW^2 (apply A) + 8nW^2 (apply V)."""
    pairs = (n // W) * (n // W - 1) / 2.0
    return pairs * (2.0 * m * W * W + 8.0 * m * W * W + 8.0 * n * W * W)


@torch.no_grad()
def verify(A, U, S, V, sigma_ref=None) -> dict:
    """Accuracy report.  A (m,n), U (m,k), S (k,), V (n,k); computed in fp64."""
    A64 = A.double()
    out = {}
    if U is not None and V is not None:
        R = A64 - (U.double() * S.double()) @ V.double().t()
        out["residual_fro"] = float(R.norm())
        out["residual_rel"] = float(R.norm() / max(float(A64.norm()), 1e-300))
    if U is not None:
        k = U.shape[1]
        nz = S.double() > 0
        Uk = U.double()[:, nz]
        out["orth_u_fro"] = float((Uk.t() @ Uk - torch.eye(Uk.shape[1], dtype=torch.float64,
                                                             device=Uk.device)).norm())
        del k
    if V is not None:
        V64 = V.double()
        out["orth_v_fro"] = float((V64.t() @ V64 - torch.eye(V64.shape[1], dtype=torch.float64,
                                                              device=V64.device)).norm())
    if sigma_ref is not None:
        s = torch.sort(S.double().cpu(), descending=True).values
        r = torch.sort(sigma_ref.double().cpu(), descending=True).values
        k = min(s.numel(), r.numel())
        s, r = s[:k], r[:k]
        rel = (s - r).abs() / r.clamp(min=1e-300)
        out["sigma_max_rel_err"] = float(rel.max())
        out["sigma_max_abs_err_over_smax"] = float((s - r).abs().max() / max(float(r[0]), 1e-300))
    return out


def default_tol(dtype: torch.dtype, m: int) -> float:
    """Relative rotation threshold.  fp32 / fp64: sqrt(m) eps, the LAPACK
    xGESVJ value (computed dot products of length m carry ~sqrt(m) eps
    relative noise).  Round 1 needed 4 sqrt(m) eps while the split-K Gram
    slabs were summed in the data precision; with fp64 slab sums the tighter
    value converges at +1-2 % time and halves ||U^T U - I|| per factor of 2
    (16384^2 fp32: 0.40 -> 0.098, profiles/r2_tol).  bf16 problems: 4 sqrt(m)
    2^-21 -- above the 2-way bf16 split's product noise (~8 fp32 ulps per
    apply, tools/probe_apply.py), far below the bf16 output rounding, and
    tight enough that the last sweeps converge quadratically."""
    if dtype == torch.bfloat16:
        return 4.0 * math.sqrt(max(m, 1)) * 2.0 ** -21
    return math.sqrt(max(m, 1)) * torch.finfo(dtype).eps
