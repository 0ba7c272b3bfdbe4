"""CPU oracle solver: native C++/OpenMP scalar one-sided Jacobi.

BASELINE config 1 ("512x512 fp64 random dense matrix, single-process CPU
reference sweep").  Wraps ``svdj_cpu_jacobi_f64/_f32`` (csrc/cpu/oracle.cpp),
which keeps the reference algorithm (reference main.cu:440-1423: Sameh
ordering, dot triple, symmetric Schur rotation, Givens update) with the
fixes listed there.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from ..config import SVDOptions
from ..ops._native import cpu_lib
from .base import SVDResult, Solver, Timer


class OracleJacobi(Solver):
    name = "oracle"

    def solve(self, A, jobu=SVDOptions.AllVec, jobv=SVDOptions.AllVec) -> SVDResult:
        cfg = self.config
        jobu, jobv = SVDOptions.parse(jobu), SVDOptions.parse(jobv)
        dtype = cfg.resolved_dtype(A)
        m, n = A.shape
        if m < n:
            raise ValueError("oracle expects m >= n (api.svd transposes wide inputs)")
        np_dt = np.float64 if dtype == torch.float64 else np.float32
        ctype = C.c_double if dtype == torch.float64 else C.c_float
        a = np.array(A.detach().cpu().to(dtype).t().numpy(), dtype=np_dt, order="C", copy=True)  # (n, m)
        s = np.zeros(n, dtype=np_dt)
        v = np.zeros((n, n), dtype=np_dt)
        hist = np.zeros(max(cfg.max_sweeps, 1), dtype=np.float64)
        fn = cpu_lib().svdj_cpu_jacobi_f64 if dtype == torch.float64 else cpu_lib().svdj_cpu_jacobi_f32
        tol = self.tolerance(dtype, m)
        P = C.POINTER(ctype)
        with Timer("cpu") as tm:
            sweeps = fn(int(jobu), int(jobv), m, n, a.ctypes.data_as(P), m, s.ctypes.data_as(P),
                        v.ctypes.data_as(P), n,
                        (0 if cfg.ordering == "sameh" else 1)
                        | ((1 if cfg.rotation == "ordered" else 0) << 4),
                        cfg.max_sweeps, tol, 1 if cfg.tol_mode == "absolute" else 0,
                        hist.ctypes.data_as(C.POINTER(C.c_double)), cfg.num_threads)
        if sweeps < 0:
            raise RuntimeError(f"oracle failed rc={sweeps}")
        h = hist[:sweeps].tolist()
        U = torch.from_numpy(a).t() if jobu != SVDOptions.NoVec else None
        V = torch.from_numpy(v).t() if jobv != SVDOptions.NoVec else None
        conv = sweeps < cfg.max_sweeps or (len(h) > 0 and h[-1] <= tol)
        return SVDResult(U, torch.from_numpy(s), V, sweeps, h, tm.seconds, self.name,
                         {"tol": tol, "converged": bool(conv), "dtype": str(dtype)})
