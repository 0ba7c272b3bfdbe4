"""Common result type and solver base class."""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import torch

from ..config import SolverConfig, SVDOptions
from ..utils.metrics import default_tol


@dataclass
class SVDResult:
    """U (m x k, column-major view), S (k,), V (n x k) -- V, not V^T
    (reference returns V, lib/JacobiMethods.cu:31 notwithstanding)."""

    U: torch.Tensor | None
    S: torch.Tensor
    V: torch.Tensor | None
    sweeps: int
    history: list = field(default_factory=list)   # per-sweep max off value
    seconds: float = 0.0
    method: str = ""
    info: dict = field(default_factory=dict)

    @property
    def converged(self) -> bool:
        return bool(self.info.get("converged", False))

    def __iter__(self):  # U, S, V = svd(A)
        return iter((self.U, self.S, self.V))


class Solver:
    """Base class of the solver families (models)."""

    name = "base"

    def __init__(self, config: SolverConfig | None = None):
        self.config = config or SolverConfig()

    def tolerance(self, dtype: torch.dtype, m: int) -> float:
        if self.config.tol is not None:
            return float(self.config.tol)
        if self.config.tol_mode == "absolute":
            return 1e-16  # reference TOLERANCE (lib/global.cuh:9)
        return default_tol(dtype, m)

    def solve(self, A: torch.Tensor, jobu=SVDOptions.AllVec, jobv=SVDOptions.AllVec) -> SVDResult:
        raise NotImplementedError


def sort_result(res: SVDResult) -> SVDResult:
    """Descending sigma with U/V columns permuted accordingly."""
    order = torch.argsort(res.S, descending=True)
    res.S = res.S[order]
    if res.U is not None:
        res.U = res.U[:, order]
    if res.V is not None:
        res.V = res.V[:, order]
    return res


class Timer:
    """Device-accurate wall timer (HIP events when on GPU)."""

    def __init__(self, device):
        self.cuda = torch.device(device).type == "cuda"

    def __enter__(self):
        if self.cuda:
            torch.cuda.synchronize()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.cuda:
            torch.cuda.synchronize()
        self.seconds = time.perf_counter() - self.t0
        return False
