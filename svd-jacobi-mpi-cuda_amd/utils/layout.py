"""Matrix layout helpers.

The framework works on column-major storage like the reference
(iteratorC(i,j,ld) = j*ld + i, reference lib/global.cuh:13-14).  In PyTorch a
column-major (m x n) matrix with leading dimension ld is the row-major tensor
``At`` of shape (n, ld); row c of ``At`` is column c.  Rows are padded with
zeros to a multiple of ``ROW_ALIGN`` (so kernels never bounds-check rows) and
columns to a multiple of 2W for the block path (zero columns never rotate).
"""
from __future__ import annotations

import torch

ROW_ALIGN = 128


def round_up(a: int, b: int) -> int:
    return (a + b - 1) // b * b


def pad_rows(m: int) -> int:
    return max(ROW_ALIGN, round_up(m, ROW_ALIGN))


def pack_columns(A: torch.Tensor, dtype: torch.dtype, device, ncols_pad: int | None = None,
                 m_pad: int | None = None) -> torch.Tensor:
    """(m, n) matrix (any strides) -> zero-padded column-major At (ncols_pad, m_pad)."""
    m, n = A.shape
    m_pad = m_pad or pad_rows(m)
    ncols_pad = ncols_pad or n
    At = torch.zeros(ncols_pad, m_pad, dtype=dtype, device=device)
    At[:n, :m].copy_(A.t())
    return At


def unpack_columns(At: torch.Tensor, m: int, n: int) -> torch.Tensor:
    """Column-major At -> (m, n) tensor view with column-major strides."""
    return At[:n, :m].t()


def is_column_major(A: torch.Tensor) -> bool:
    return A.dim() == 2 and A.stride(0) == 1 and A.stride(1) >= A.shape[0]
