"""Synthetic input matrices.

* :func:`reference_triu` -- bit-exact reference input: upper-triangular
  U(0,1) from std::default_random_engine(1000000) (reference
  main.cu:1445, 1558-1567), produced by the native C++ generator.
* :func:`reference_dense` -- the dense U(0,1) variant the reference's
  ``#ifdef TESTS`` block intended (main.cu:1569-1579).
* :func:`random_dense` -- fast seeded dense matrices generated on the target
  device (benchmarks: "synthetic random dense").
* :func:`with_spectrum` -- A = Q1 diag(s) Q2^T with prescribed singular values
  (accuracy tests with a known answer).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from ..ops._native import cpu_lib

REFERENCE_SEED = 1000000


def reference_triu(n: int, m: int | None = None, seed: int = REFERENCE_SEED) -> torch.Tensor:
    m = n if m is None else m
    a = np.zeros((n, m), dtype=np.float64)  # column-major storage: row c = column c
    cpu_lib().svdj_ref_triu_input(m, n, a.ctypes.data_as(C.POINTER(C.c_double)), m, seed)
    return torch.from_numpy(a).t()


def reference_dense(n: int, m: int | None = None, seed: int = REFERENCE_SEED) -> torch.Tensor:
    m = n if m is None else m
    a = np.zeros((n, m), dtype=np.float64)
    cpu_lib().svdj_ref_dense_input(m, n, a.ctypes.data_as(C.POINTER(C.c_double)), m, seed)
    return torch.from_numpy(a).t()


def reference_uniform_stream(count: int, seed: int = REFERENCE_SEED) -> np.ndarray:
    out = np.zeros(count, dtype=np.float64)
    cpu_lib().svdj_ref_uniform_stream(seed, count, out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def random_dense(m: int, n: int, dtype=torch.float64, device="cpu", seed: int = 0,
                 dist: str = "uniform") -> torch.Tensor:
    g = torch.Generator(device=device).manual_seed(seed)
    if dist == "uniform":
        return torch.rand(m, n, generator=g, dtype=dtype, device=device)
    if dist == "normal":
        return torch.randn(m, n, generator=g, dtype=dtype, device=device)
    raise ValueError(dist)


def with_spectrum(m: int, n: int, sigma, dtype=torch.float64, seed: int = 0) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    k = min(m, n)
    s = torch.as_tensor(sigma, dtype=torch.float64)
    assert s.numel() == k
    q1, _ = torch.linalg.qr(torch.randn(m, k, generator=g, dtype=torch.float64))
    q2, _ = torch.linalg.qr(torch.randn(n, k, generator=g, dtype=torch.float64))
    return ((q1 * s) @ q2.t()).to(dtype)


def geometric_spectrum(k: int, cond: float) -> torch.Tensor:
    return torch.logspace(0, -np.log10(cond), k, dtype=torch.float64)
