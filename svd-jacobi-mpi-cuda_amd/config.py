"""Solver configuration.

The reference's knobs are compile-time macros and hard-coded constants
(TOLERANCE 1e-16 lib/global.cuh:9, maxIterations = 1 main.cu:482, 16-thread
blocks main.cu:449, 36 OpenMP threads main.cu:1431, seed 1000000
main.cu:1445).  Here they are one dataclass, settable from the CLI
(:func:`add_cli_args`) or environment-free Python.
"""
from __future__ import annotations

import argparse
import enum
from dataclasses import dataclass, field, asdict

import torch


class SVDOptions(enum.IntEnum):
    """LAPACK-style job options (reference enum SVD_OPTIONS, main.cu:157-161)."""

    AllVec = 0
    SomeVec = 1
    NoVec = 2

    @classmethod
    def parse(cls, v) -> "SVDOptions":
        if isinstance(v, SVDOptions):
            return v
        if isinstance(v, int):
            return SVDOptions(v)
        s = str(v).strip().lower()
        table = {"a": cls.AllVec, "all": cls.AllVec, "allvec": cls.AllVec,
                 "s": cls.SomeVec, "some": cls.SomeVec, "somevec": cls.SomeVec,
                 "n": cls.NoVec, "none": cls.NoVec, "novec": cls.NoVec, "o": cls.AllVec}
        if s not in table:
            raise ValueError(f"bad SVD option {v!r}")
        return table[s]


def debug_knob(key: str, default=None):
    """Value of ``key`` in the A/B switch SVDJ_DEBUG="key=value,..." (int),
    or ``default`` -- the Python twin of csrc/include/svdj_debug.h, which
    lists the keys.  Production runs never set it."""
    import os

    for item in os.environ.get("SVDJ_DEBUG", "").split(","):
        k, sep, v = item.partition("=")
        if sep and k.strip() == key:
            return int(v)
    return default


_DTYPES = {"fp32": torch.float32, "float32": torch.float32, "fp64": torch.float64,
           "float64": torch.float64, "bf16": torch.bfloat16, "bfloat16": torch.bfloat16}


@dataclass
class SolverConfig:
    method: str = "auto"            # auto | block | scalar | oracle
    dtype: torch.dtype | None = None  # fp32 | fp64 | bf16 (None: the input's dtype)
    block: int | None = None        # block width W (block path); None: auto
    tol: float | None = None        # rotation threshold; None: sqrt(m) eps (utils.metrics.default_tol)
    tol_mode: str = "relative"      # relative | absolute (reference parity)
    max_sweeps: int = 60            # reference: 1 (main.cu:482)
    max_inner_sweeps: int = 1       # block path: Jacobi sweeps per pair EVD (1 = one pass)
    inner_order: str = "auto"       # block path, cross steps: cyclic (2W-1 EVD steps, all
                                    # pairs) | bipartite (W steps, cross pairs only) |
                                    # cross (bipartite steps, only the cross couplings
                                    # tracked) | auto (models.block.choose_inner_order)
    ordering: str = "sameh"         # scalar path: sameh (reference) | round_robin
    rotation: str = "schur"         # oracle: schur (reference inline) | ordered (lib/Utils.cu)
    sort: bool = False              # reference returns unsorted sigma
    mma: str = "auto"               # block apply matrix cores: auto | native | bf16x6 | bf16x3
    precondition: str = "auto"      # auto | qr | none  (QR first when m >= qr_ratio * n)
    # Measured on MI355X, 32768 x 8192 fp32: Jacobi on A directly 2.27-2.6 s; CholeskyQR2
    # + Jacobi on R + U = Q U_R 1.99 s (Householder QR via rocSOLVER geqrf: 5.4 s).
    qr_ratio: float = 2.0
    chains: int = 2                 # block path: independent step chains on separate streams
    num_threads: int = 0            # CPU oracle OpenMP threads (0: default)
    progress: bool = False          # rank 0 prints one line per sweep to stderr
    comm_timing: bool = False       # distributed: HIP-event timing of every exchange
    # distributed, pipelined: how a half super-block travels between GPUs.
    # direct: one grouped send/recv (one xGMI link); spread: cut into P-1
    # chunks, relayed over all links in two phases (parallel/spread.py);
    # auto: spread from 4 GPUs up
    exchange: str = "auto"
    # distributed, pipelined: fuse cross steps two at a time over quads of
    # blocks (csrc/hip/block.hip "quad step": Gram-space second-step
    # couplings, one K = 256 apply per two steps).  auto: models.block.choose_quad
    quad: str = "auto"
    # block path: when a sweep ends the iteration.  second_order: also after
    # a sweep whose applied rotations were all noise-level (largest coupling
    # x largest sine, csrc/include/svdj_stop.h); no_rotation: only after a
    # sweep that rotated nothing (the confirmation sweep)
    stop_rule: str = "second_order"
    checkpoint_dir: str | None = None
    checkpoint_every: int = 0       # sweeps between checkpoints (0: off)
    extra: dict = field(default_factory=dict)

    def __post_init__(self):
        if self.chains not in (1, 2):
            raise ValueError(f"chains must be 1 (blocking exchange) or 2 (pipelined), "
                             f"got {self.chains}")
        if self.max_inner_sweeps < 0 or self.max_sweeps < 0:
            raise ValueError("max_sweeps / max_inner_sweeps must be >= 0")
        if self.exchange not in ("auto", "direct", "spread"):
            raise ValueError(f"exchange must be auto, direct or spread, got {self.exchange!r}")
        if self.quad not in ("auto", "on", "off"):
            raise ValueError(f"quad must be auto, on or off, got {self.quad!r}")
        if self.stop_rule not in ("second_order", "no_rotation"):
            raise ValueError(f"stop_rule must be second_order or no_rotation, "
                             f"got {self.stop_rule!r}")

    def bf16_mode(self, A: torch.Tensor | None = None) -> bool:
        """bf16 problem: bf16 in/out, fp32 master copies of A and V, block
        apply on bf16 matrix cores (2-way split) and a bf16-level stop test."""
        if self.dtype is not None:
            return self.dtype == torch.bfloat16
        return A is not None and A.dtype == torch.bfloat16

    def resolved_dtype(self, A: torch.Tensor | None) -> torch.dtype:
        """Storage/compute dtype of the working copies (fp32 or fp64)."""
        if self.dtype is not None:
            return torch.float32 if self.dtype == torch.bfloat16 else self.dtype
        if A is not None and A.dtype == torch.float64:
            return torch.float64
        return torch.float32

    def precision_dtype(self, A: torch.Tensor | None) -> torch.dtype:
        """The dtype whose accuracy the stop test targets."""
        return torch.bfloat16 if self.bf16_mode(A) else self.resolved_dtype(A)

    def resolved_mma(self, A: torch.Tensor | None, W: int | None = None) -> str:
        """Matrix-core mode of the block apply: "auto" is bf16x3 in the bf16
        problem mode, else models.block.choose_mma(dtype, W)."""
        if self.mma != "auto":
            return self.mma
        if self.bf16_mode(A):
            return "bf16x3"
        from .models.block import choose_mma
        return choose_mma(self.resolved_dtype(A), W or 0)

    def to_dict(self) -> dict:
        d = asdict(self)
        d["dtype"] = str(self.dtype) if self.dtype is not None else None
        return d


def add_cli_args(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    p.add_argument("--method", default="auto", choices=["auto", "block", "scalar", "oracle"])
    p.add_argument("--dtype", default=None, choices=sorted(_DTYPES))
    p.add_argument("--block", type=int, default=None)
    p.add_argument("--tol", type=float, default=None)
    p.add_argument("--tol-mode", default="relative", choices=["relative", "absolute"])
    p.add_argument("--max-sweeps", type=int, default=60)
    p.add_argument("--max-inner-sweeps", type=int, default=1)
    p.add_argument("--inner-order", default=None,
                   choices=["auto", "cyclic", "bipartite", "cross"],
                   help="EVD ordering of the block cross steps (default: the config's)")
    p.add_argument("--ordering", default="sameh", choices=["sameh", "round_robin"])
    p.add_argument("--sort", action="store_true")
    p.add_argument("--mma", default="auto", choices=["auto", "native", "bf16x6", "bf16x3"])
    p.add_argument("--precondition", default="auto", choices=["auto", "qr", "none"])
    p.add_argument("--checkpoint-dir", default=None)
    p.add_argument("--checkpoint-every", type=int, default=0)
    p.add_argument("--progress", action="store_true", help="print one line per sweep (rank 0)")
    p.add_argument("--quad", default="auto", choices=["auto", "on", "off"],
                   help="fused two-step quad block steps (fp32, W=64, split-bf16 apply)")
    p.add_argument("--stop-rule", default="second_order", choices=["second_order", "no_rotation"],
                   help="block path: also stop after a sweep of noise-level rotations "
                        "(second_order) or only after a sweep without rotations")
    return p


def config_from_args(a) -> SolverConfig:
    return SolverConfig(method=a.method, dtype=_DTYPES[a.dtype] if a.dtype else None,
                        block=a.block, tol=a.tol, tol_mode=a.tol_mode, max_sweeps=a.max_sweeps,
                        max_inner_sweeps=a.max_inner_sweeps, ordering=a.ordering, sort=a.sort,
                        mma=a.mma, precondition=a.precondition, checkpoint_dir=a.checkpoint_dir,
                        checkpoint_every=a.checkpoint_every,
                        progress=bool(getattr(a, "progress", False)),
                        quad=getattr(a, "quad", "auto"),
                        stop_rule=getattr(a, "stop_rule", "second_order"),
                        **({"inner_order": a.inner_order}
                           if getattr(a, "inner_order", None) else {}))
