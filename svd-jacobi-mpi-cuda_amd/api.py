"""Public entry points.

``svd(A)`` -- functional API returning (U, S, V) (V, not V^T).
``gesvd(jobu, jobv, m, n, A, lda, s, V, ldv)`` -- the reference's in-place
signature (reference main.cu:440-448 ``omp_mpi_cuda_dgesvd_local_matrices``,
lib/JacobiMethods.cuh:44-62): column-major A (leading dimension lda) is
overwritten by U, ``s`` receives sigma (unsorted unless config.sort), V
(n x n, ldv) receives V.  With AllVec the reference's U is the thin m x n
factor stored in A (LAPACK jobu='O' semantics); SomeVec is the same here.
"""
from __future__ import annotations

import torch

from .config import SolverConfig, SVDOptions
from .models.base import SVDResult, sort_result
from .models.block import BlockJacobi
from .models import precondition as pre
from .models.oracle import OracleJacobi
from .models.scalar import ScalarJacobi

_METHODS = {"block": BlockJacobi, "scalar": ScalarJacobi, "oracle": OracleJacobi}


def _pick_method(cfg: SolverConfig, device: torch.device, n: int) -> str:
    if cfg.method != "auto":
        return cfg.method
    if device.type == "cpu":
        return "oracle"
    return "block" if n >= 64 else "scalar"


def svd(A: torch.Tensor, jobu=SVDOptions.AllVec, jobv=SVDOptions.AllVec,
        config: SolverConfig | None = None, device=None, **overrides) -> SVDResult:
    """One-sided Jacobi SVD of a dense (m x n) matrix.

    ``device`` defaults to A's device.  Keyword overrides update the config
    (e.g. ``svd(A, method="scalar", tol=1e-12)``).  Returns an
    :class:`SVDResult` that unpacks as ``U, S, V``.
    """
    cfg = config or SolverConfig()
    if overrides:
        cfg = SolverConfig(**{**cfg.__dict__, **overrides})
    if A.dim() != 2:
        raise ValueError("A must be 2-D")
    dev = torch.device(device) if device is not None else A.device
    jobu, jobv = SVDOptions.parse(jobu), SVDOptions.parse(jobv)
    m, n = A.shape
    transposed = m < n
    if transposed:  # A^T = U' S V'^T  =>  A = V' S U'^T
        A = A.t()
        jobu, jobv = jobv, jobu
    method = _pick_method(cfg, dev, A.shape[1])
    solver = _METHODS[method](cfg)
    mm, nn = A.shape
    Q = None
    if pre.use_qr(cfg, mm, nn):
        # tall-skinny: Jacobi on R (n x n), U = Q U_R (models/precondition.py)
        Q, R, Lt = pre.qr_deferred(A.to(dev), cfg.resolved_dtype(A))
        A = R.to(A.dtype) if cfg.bf16_mode(A) else R
    if method == "oracle":
        res = solver.solve(A, jobu, jobv)
    else:
        res = solver.solve(A, jobu, jobv, device=dev)
    if Q is not None:
        if res.U is not None:
            res.U = pre.apply_q(Q, Lt, res.U.to(Q.device)).to(res.U.dtype)
        res.info["precondition"] = "qr"
    res.info["flops"] = pre.flops(mm, nn, res.sweeps, Q is not None)
    if transposed:
        res.U, res.V = res.V, res.U
        res.info["transposed"] = True
    if cfg.sort:
        res = sort_result(res)
    return res


def gesvd(jobu, jobv, m: int, n: int, A: torch.Tensor, lda: int, s: torch.Tensor,
          V: torch.Tensor | None, ldv: int, config: SolverConfig | None = None) -> SVDResult:
    """Reference-shaped in-place API.

    A: buffer holding a column-major m x n matrix with leading dimension lda
    (a 1-D tensor of >= lda*n elements, or a 2-D tensor whose storage is
    that).  On return A holds U (if jobu != NoVec; otherwise A V), s[:min(m,n)]
    holds sigma and V[:, :n] (column-major, ldv) holds V.
    """
    if not A.is_contiguous():
        raise ValueError("A buffer must be contiguous storage")
    if m < n:
        raise ValueError("gesvd follows the reference (m >= n); use svd() for wide matrices")
    if lda < m:
        raise ValueError("lda < m")
    Acm = A.reshape(-1)[: lda * n].view(n, lda)[:, :m].t()  # (m, n) column-major view
    res = svd(Acm, jobu, jobv, config=config, device=A.device)
    s.reshape(-1)[:n].copy_(res.S[:n].to(s.dtype))
    if res.U is not None:
        Acm.copy_(res.U.to(A.dtype))
    if V is not None and res.V is not None:
        flatV = V.reshape(-1)
        Vcm = flatV[: ldv * n].view(n, ldv)[:, :n].t()
        Vcm.copy_(res.V[:n, :n].to(V.dtype))
    return res


def svd_on_the_fly(m: int, n: int, generator, comm=None, jobu=SVDOptions.AllVec,
                   jobv=SVDOptions.AllVec, dtype: torch.dtype = torch.float32,
                   config: SolverConfig | None = None, gather: bool = True) -> SVDResult:
    """Distributed SVD of a matrix that is never assembled on one rank:
    ``generator(c0, c1)`` returns columns c0..c1-1 (m x (c1-c0)) of a fixed
    matrix on the calling rank's device, and every rank generates only the
    super-blocks it owns.  The reference declares this entry point
    (``omp_mpi_dgesvd_on_the_fly_matrices``, lib/JacobiMethods.cuh:64-72) but
    never defines it.  ``comm`` defaults to a fresh Communicator (one process
    per GPU, RCCL; gloo on CPU)."""
    from .parallel import Communicator, DistributedBlockJacobi

    solver = DistributedBlockJacobi(config or SolverConfig(), comm or Communicator())
    return solver.solve(None, jobu, jobv, m=m, n=n, dtype=dtype, generator=generator,
                        gather=gather)
