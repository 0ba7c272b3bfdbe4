"""MI355X-native distributed one-sided Jacobi SVD.

A brand-new gfx950 (CDNA4) framework with the capabilities of
acastellanos95/SVD-Jacobi-MPI-CUDA: the reference's
column-pair Jacobi sweep is rebuilt as hand-written HIP kernels (fused
scalar pair steps; MFMA block Gram / LDS EVD / MFMA apply), one process per
GPU with torch.distributed over RCCL/xGMI for the block tournament, and a
native C++ host runtime (schedules, oracle, reference input generator).

The directory name is not a Python identifier; import it as ``svdj``
(top-level alias module) or ``importlib.import_module("svd-jacobi-mpi-cuda_amd")``.
"""
from __future__ import annotations

__version__ = "0.1.0"

from . import cli, config, ops, models, parallel, utils  # noqa: F401
from .api import gesvd, svd, svd_on_the_fly  # noqa: F401
from .config import SolverConfig, SVDOptions  # noqa: F401
from .models.base import SVDResult  # noqa: F401

AllVec = SVDOptions.AllVec
SomeVec = SVDOptions.SomeVec
NoVec = SVDOptions.NoVec
