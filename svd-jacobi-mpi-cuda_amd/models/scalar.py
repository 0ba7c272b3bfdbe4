"""Scalar column-pair Jacobi on one device (reference-parity path).

Same algorithm and ordering as the reference's sweep
(reference main.cu:496-1384 / cuda_dgesvd_kernel main.cu:163-437) but one
fused HIP launch per parallel step (csrc/hip/scalar.hip) with A and V
resident in HBM, and a real convergence loop.  Supports the reference's
parity knobs: Sameh ordering, absolute 1e-16 threshold, max_sweeps=1.
"""
from __future__ import annotations

import torch

from ..config import SVDOptions
from ..ops import kernels as K
from ..parallel.schedule import round_robin_padded, sameh
from ..utils.layout import pack_columns, pad_rows
from .base import SVDResult, Solver, Timer


class ScalarJacobi(Solver):
    name = "scalar"

    def solve(self, A, jobu=SVDOptions.AllVec, jobv=SVDOptions.AllVec, device=None) -> SVDResult:
        cfg = self.config
        jobu, jobv = SVDOptions.parse(jobu), SVDOptions.parse(jobv)
        device = torch.device(device) if device is not None else A.device
        dtype = cfg.resolved_dtype(A)
        m, n = A.shape
        if m < n:
            raise ValueError("scalar path expects m >= n (api.svd transposes wide inputs)")
        m_pad, n_v = pad_rows(m), pad_rows(n)
        At = pack_columns(A, dtype, device, n, m_pad)
        want_v = jobv != SVDOptions.NoVec
        Vt = torch.zeros(n, n_v, dtype=dtype, device=device) if want_v else None
        if want_v:
            K.set_identity(Vt, n)
        sched_np = sameh(n) if cfg.ordering == "sameh" else round_robin_padded(n)
        sched = torch.from_numpy(sched_np).to(device)
        tol = self.tolerance(cfg.precision_dtype(A), m)
        tol_mode = 1 if cfg.tol_mode == "absolute" else 0
        with Timer(device) as tm:
            sweeps, hist = K.scalar_solve(At, Vt, m_pad, sched, tol, tol_mode, cfg.max_sweeps)
            S = K.finalize(At, m_pad, scale_u=jobu != SVDOptions.NoVec)
        U = At[:, :m].t() if jobu != SVDOptions.NoVec else None
        V = Vt[:, :n].t() if want_v else None
        if cfg.bf16_mode(A):
            U = U.to(torch.bfloat16) if U is not None else None
            V = V.to(torch.bfloat16) if V is not None else None
        conv = sweeps < cfg.max_sweeps or (hist and hist[-1] <= tol)
        return SVDResult(U, S, V, sweeps, hist, tm.seconds, self.name,
                         {"tol": tol, "converged": bool(conv), "dtype": str(dtype),
                          "device": str(device), "ordering": cfg.ordering})
