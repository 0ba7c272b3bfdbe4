"""Tensor-level entry points of the native ops.

Device (HIP) tensors go to the gfx950 kernels in ``libsvdj_hip.so`` via
ctypes on torch's current stream; CPU tensors go to ``ops.reference``.  A
device tensor never falls back to PyTorch math: a missing/failed native
library raises :class:`NativeError`.

All matrices use the transposed column-major layout of the kernels: ``At``
has shape (ncols, ld) and row c is column c of the matrix; rows are padded to
``ROW_ALIGN`` with zeros (``m_pad``).
"""
from __future__ import annotations

import ctypes as C
import struct

import numpy as np
import torch

from . import reference as ref
from ._native import NativeError, cpu_lib, hip_check, hip_lib

ROW_ALIGN = 128
SUPPORTED_BLOCK = {torch.float32: (32, 64), torch.float64: (32, 64)}
# Matrix-core modes of the block apply (csrc/hip/block.hip): native f32/f64
# MFMA (default, fp32-exact products and sums), or fp32 data on bf16 MFMA
# with a 3-way / 2-way operand split -- faster (memory-bound instead of
# MFMA-bound at W=64) but NOT fp32-accurate on every input: the bf16 MFMA's
# internal accumulation is biased when magnitudes mix (see block.hip).
MMA_CODES = {"native": 0, "bf16x6": 1, "bf16x3": 2}


def mma_code(mma: str | int, dtype: torch.dtype) -> int:
    if isinstance(mma, int):
        return mma
    if mma == "auto":
        mma = "native"
    if mma not in MMA_CODES:
        raise ValueError(f"bad mma mode {mma!r}; one of {sorted(MMA_CODES)} or 'auto'")
    if mma != "native" and dtype != torch.float32:
        raise ValueError(f"mma={mma} needs fp32 data")
    return MMA_CODES[mma]


def tol_mode_code(tol_mode) -> int:
    """0 = relative |g_pq| > tol sqrt(g_pp g_qq) (default), 1 = absolute
    |g_pq| > tol (the reference's TOLERANCE test, lib/global.cuh:9)."""
    if tol_mode in (0, 1):
        return int(tol_mode)
    table = {"relative": 0, "absolute": 1}
    if tol_mode not in table:
        raise ValueError(f"bad tol_mode {tol_mode!r}; 'relative' or 'absolute'")
    return table[tol_mode]


def dtype_code(dtype: torch.dtype) -> int:
    if dtype == torch.float32:
        return 0
    if dtype == torch.float64:
        return 1
    raise TypeError(f"unsupported dtype {dtype} (fp32/fp64)")


def _stream(t: torch.Tensor):
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def _check_layout(At: torch.Tensor, m_pad: int):
    if At.dim() != 2 or At.stride(1) != 1:
        raise ValueError("At must be a 2-D tensor with contiguous rows (ncols, ld)")
    if m_pad % ROW_ALIGN or At.stride(0) < m_pad or At.shape[1] < m_pad:
        raise ValueError(f"m_pad={m_pad} must be a multiple of {ROW_ALIGN} and <= ld")


# ------------------------------------------------------------------ metric
METRIC_WORDS = 8  # csrc/include/svdj_stop.h SVDJ_METRIC_WORDS


def new_metric(device) -> torch.Tensor:
    """Per-sweep stop-test state: [0] max convergence value, [1] rotated
    pairs, the negligible-column floor of the solve (block path), and for the
    block path's second-order stop test the largest effective sine of an
    applied rotation and the number of column rotations applied.  Device:
    int32[8] (csrc/include/svdj_stop.h: floor a double in [2..3], sine float
    bits in [4], count [5]); CPU: float64[5] (floor [2], sine [3], count [4])."""
    if torch.device(device).type == "cpu":
        return torch.zeros(5, dtype=torch.float64)
    return torch.zeros(METRIC_WORDS, dtype=torch.int32, device=device)


def reset_metric(metric: torch.Tensor):
    """Zero the per-sweep words; the floor (set once per solve) stays."""
    metric[:2].zero_()
    if metric.device.type == "cpu":
        metric[3:].zero_()
    else:
        metric[4:].zero_()


def norm_floor(dtype: torch.dtype, m: int, dmax: float = 1.0) -> float:
    """Negligible-column floor: the block EVDs (block.hip needs_rotation) do
    not rotate pairs with a squared column norm at or below
    max(m realmin, m realmin / eps * dmax), dmax the largest squared column
    norm of the matrix.  The second term is the round-3 floor m realmin / eps
    taken relative to the matrix's scale, so c A is solved like A (LAPACK
    xGESVJ prescales A for the same reason); the first keeps columns whose
    products would be subnormal out whatever the scale."""
    fi = torch.finfo(torch.float64 if dtype == torch.float64 else torch.float32)
    return max(m * fi.tiny, m * fi.tiny / fi.eps * float(dmax))


def set_norm_floor(metric: torch.Tensor, dtype: torch.dtype, m: int, dmax: float = 1.0):
    """Store :func:`norm_floor` in the metric (once per solve)."""
    v = norm_floor(dtype, m, dmax)
    if metric.device.type == "cpu":
        metric[2] = v
    else:
        metric[2:4].view(torch.float64).fill_(v)


def read_metric(metric: torch.Tensor):
    """(max convergence value, rotations) -- synchronises for device metrics."""
    if metric.device.type == "cpu":
        return float(metric[0]), int(metric[1])
    h = metric.cpu().numpy().astype(np.int32)
    mx = struct.unpack("<f", struct.pack("<i", int(h[0])))[0]
    return mx, int(np.uint32(h[1]))


def metric_as_float_pair(metric: torch.Tensor) -> torch.Tensor:
    """Device-side (maxconv, rotations) as float64 without host sync."""
    if metric.device.type == "cpu":
        return metric[:2].clone()
    return torch.stack([metric[0:1].view(torch.float32).double()[0], metric[1].double()])


def metric_stop_values(metric: torch.Tensor) -> torch.Tensor:
    """(maxconv, max effective sine, rotated pairs, column rotations) as
    float64, device-side for device metrics (no host sync)."""
    if metric.device.type == "cpu":
        return torch.stack([metric[0], metric[3], metric[1], metric[4]]).clone()
    f = metric.view(torch.float32)
    u = metric[5:6].view(torch.int32)[0].double()
    u = torch.where(u < 0, u + 2.0 ** 32, u)  # uint32 count
    return torch.stack([f[0].double(), f[4].double(), metric[1].double(), u])


def metric_work(metric: torch.Tensor) -> torch.Tensor:
    """The quad apply's work counters of the sweep (svdj_stop.h words 6, 7),
    float64 on the metric's device without a host sync: [MFMAs issued / 24,
    32-row x 256-column tiles moved].  Zeros for CPU metrics (the CPU
    emulation has no counters)."""
    if metric.device.type == "cpu":
        return torch.zeros(2, dtype=torch.float64)
    w = metric[6:8].double()
    return torch.where(w < 0, w + 2.0 ** 32, w)


def read_stop(metric: torch.Tensor):
    """(max convergence value, max effective sine, rotated pairs, column
    rotations) -- synchronises."""
    v = metric_stop_values(metric).cpu()
    return float(v[0]), float(v[1]), int(v[2]), int(v[3])


STOP_RULES = {"no_rotation": 0, "second_order": 1}


def sweep_converged(mx: float, ms: float, nrot_pairs: float, nrot_cols: float, tol: float,
                    tol_mode="relative", stop_rule="second_order") -> int:
    """The block path's sweep stop test (csrc/include/svdj_stop.h, the same
    native code every engine runs): 0 continue, 1 the sweep rotated nothing,
    2 its rotations were all noise-level (second-order rule:
    nrot_cols * mx * ms <= tol / 2)."""
    rule = STOP_RULES[stop_rule] if isinstance(stop_rule, str) else int(stop_rule)
    return int(cpu_lib().svdj_sweep_converged(float(mx), float(ms), float(nrot_pairs),
                                              float(nrot_cols), float(tol),
                                              tol_mode_code(tol_mode), rule))


# --------------------------------------------------------------- utilities
def set_identity(Vt: torch.Tensor, ncols: int, col_offset: int = 0):
    if Vt.is_cuda:
        hip_check(hip_lib().svdj_set_identity(dtype_code(Vt.dtype), _ptr(Vt), Vt.shape[1],
                                              Vt.stride(0), ncols, col_offset, _stream(Vt)),
                  "set_identity")
    else:
        Vt[:ncols].zero_()
        idx = torch.arange(ncols)
        ok = idx + col_offset < Vt.shape[1]
        Vt[idx[ok], idx[ok] + col_offset] = 1


def col_norms2(At: torch.Tensor, m_pad: int, out: torch.Tensor | None = None) -> torch.Tensor:
    _check_layout(At, m_pad)
    ncols = At.shape[0]
    if out is None:
        out = torch.empty(ncols, dtype=At.dtype, device=At.device)
    if At.is_cuda:
        hip_check(hip_lib().svdj_col_norms2(dtype_code(At.dtype), _ptr(At), m_pad, At.stride(0),
                                            ncols, _ptr(out), _stream(At)), "col_norms2")
    else:
        out.copy_(ref.col_norms2(At[:, :m_pad]))
    return out


def finalize(At: torch.Tensor, m_pad: int, scale_u: bool = True) -> torch.Tensor:
    """sigma_c = ||a_c||; optionally a_c /= sigma_c (sigma 0 untouched)."""
    _check_layout(At, m_pad)
    ncols = At.shape[0]
    sigma = torch.empty(ncols, dtype=At.dtype, device=At.device)
    if At.is_cuda:
        hip_check(hip_lib().svdj_finalize(dtype_code(At.dtype), _ptr(At), m_pad, At.stride(0),
                                          ncols, _ptr(sigma), int(scale_u), _stream(At)),
                  "finalize")
    else:
        sigma.copy_(ref.finalize(At[:, :m_pad], scale_u))
    return sigma


def spin_ns(device, ns: float):
    """Enqueue a device-side wait of ``ns`` nanoseconds on the current stream
    of ``device`` (link-time model of the simulated exchange)."""
    st = C.c_void_p(torch.cuda.current_stream(torch.device(device)).cuda_stream)
    hip_check(hip_lib().svdj_spin_ns(float(ns), st), "spin_ns")


# ---------------------------------------------------------------- scalar path
def scalar_step(At, Vt, m_pad, pairs, tol, tol_mode, metric):
    """One parallel step; pairs: int32 tensor (k, 2) on At's device."""
    _check_layout(At, m_pad)
    if At.is_cuda:
        n_v = Vt.shape[1] if Vt is not None else 0
        ldv = Vt.stride(0) if Vt is not None else 0
        hip_check(hip_lib().svdj_scalar_step(
            dtype_code(At.dtype), m_pad, _ptr(At), At.stride(0), _ptr(Vt), n_v, ldv,
            _ptr(pairs), pairs.shape[0], float(tol), int(tol_mode), _ptr(metric), _stream(At)),
            "scalar_step")
    else:
        mx, nrot = ref.scalar_step(At, Vt, pairs, tol, tol_mode)
        metric[0] = max(float(metric[0]), mx)
        metric[1] += nrot


def scalar_solve(At, Vt, m_pad, sched, tol, tol_mode, max_sweeps):
    """Repeated sweeps over ``sched`` (int32 (steps, per_step, 2)) until no
    rotation.  Returns (sweeps, per-sweep max convergence value list)."""
    _check_layout(At, m_pad)
    steps, per_step = int(sched.shape[0]), int(sched.shape[1])
    if At.is_cuda:
        metric = new_metric(At.device)
        hist = (C.c_double * max(max_sweeps, 1))()
        n_v = Vt.shape[1] if Vt is not None else 0
        ldv = Vt.stride(0) if Vt is not None else 0
        sweeps = hip_check(hip_lib().svdj_scalar_solve(
            dtype_code(At.dtype), m_pad, _ptr(At), At.stride(0), _ptr(Vt), n_v, ldv,
            _ptr(sched), steps, per_step, float(tol), int(tol_mode), int(max_sweeps),
            _ptr(metric), hist, _stream(At)), "scalar_solve")
        return sweeps, [hist[i] for i in range(sweeps)]
    hist = []
    for _ in range(max_sweeps):
        metric = new_metric("cpu")
        for s in range(steps):
            scalar_step(At, Vt, m_pad, sched[s], tol, tol_mode, metric)
        mx, nrot = read_metric(metric)
        hist.append(mx)
        if nrot == 0:
            break
    return len(hist), hist


# ----------------------------------------------------------------- block path
_WS_CACHE: dict = {}


def block_workspace(dtype, W, P, m_pad, device, slot: int = 0, pool: dict | None = None,
                    quad: bool = False) -> torch.Tensor:
    """Per (device, shape, slot, quad) workspace; concurrent chains use
    distinct slots.  ``pool`` is the caller's own cache (a solver instance owns
    one, so solvers running concurrently -- e.g. several ranks in one process
    -- never share scratch); None uses the module-wide cache.  ``quad``: the
    step list holds quad steps (their scratch is sized only then)."""
    nbytes = int(hip_lib().svdj_block_workspace_bytes(dtype_code(dtype), W, P, m_pad, int(quad)))
    cache = _WS_CACHE if pool is None else pool
    key = (torch.device(device), dtype, W, P, m_pad, slot, bool(quad))
    ws = cache.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
        cache[key] = ws
    return ws


INNER_ORDERS = ("cyclic", "bipartite", "cross")


def step_modes(modes, inner_order="cyclic"):
    """Plan modes (0 cross, 1 full) -> kernel modes: with the bipartite inner
    ordering cross steps become mode 2 (block.hip EVD_BIP, W EVD steps instead
    of 2W-1), with the cross-only ordering mode 3 (evd_cross_kernel: the
    bipartite steps tracking only the cross couplings); full steps always use
    the cyclic EVD."""
    if inner_order not in INNER_ORDERS:
        raise ValueError(f"inner_order must be one of {INNER_ORDERS}, got {inner_order!r}")
    cm = {"cyclic": 0, "bipartite": 2, "cross": 3}[inner_order]  # "auto": resolve first
    return [cm if int(x) == 0 else int(x) for x in modes]


def check_block(dtype, W):
    if W not in SUPPORTED_BLOCK.get(dtype, ()):
        raise ValueError(f"block width {W} unsupported for {dtype}; supported "
                         f"{SUPPORTED_BLOCK.get(dtype, ())}")


def block_steps(At, Vt, D, m_pad, pairs, W, modes, tol, max_inner, metric, ws_slot: int = 0,
                mma="native", pool: dict | None = None, tol_mode="relative",
                inner_order="cyclic", gram_parts: int = 3, shared_gpu: bool = False):
    """Run ``len(modes)`` block steps on the current stream.  pairs: int32
    (steps, P, 2) on At's device (block indices local to At); modes: list of
    0 (cross) / 1 (full) (see step_modes for ``inner_order``).  Chains running
    concurrently on different streams must use different ``ws_slot`` values.
    ``gram_parts`` 2: the quad Gram on 2 bf16 parts (svdj_block_steps' mma bit
    8; GPU only, the CPU emulation keeps the exact Gram).  ``shared_gpu``:
    another chain runs concurrently on this GPU (bit 9: the quad apply leaves
    it a quarter of the CUs)."""
    modes = step_modes(modes, inner_order)
    _check_layout(At, m_pad)
    check_block(At.dtype, W)
    steps, P = int(pairs.shape[0]), int(pairs.shape[1])
    if steps == 0 or P == 0:
        return
    if At.is_cuda:
        ws = block_workspace(At.dtype, W, P, m_pad, At.device, ws_slot, pool,
                             quad=any(int(x) == 4 for x in modes))
        md = (C.c_int32 * steps)(*[int(x) for x in modes])
        n_v = Vt.shape[1] if Vt is not None else 0
        ldv = Vt.stride(0) if Vt is not None else 0
        hip_check(hip_lib().svdj_block_steps(
            dtype_code(At.dtype), W, m_pad, _ptr(At), At.stride(0), _ptr(Vt), n_v, ldv,
            _ptr(D), _ptr(pairs), P, steps, md, float(tol), tol_mode_code(tol_mode),
            int(max_inner), _ptr(ws), ws.numel(), _ptr(metric),
            mma_code(mma, At.dtype) | (256 if gram_parts == 2 else 0) | (512 if shared_gpu else 0),
            _stream(At)), "block_steps")
    else:
        for s in range(steps):
            if modes[s] == 5:  # second step of a quad: done with its first
                continue
            stats = {"smax": 0.0}
            if modes[s] == 4:
                mx, nrot = ref.quad_step(At[:, :m_pad], Vt, D, pairs[s], pairs[s + 1], W, tol,
                                         max_inner, tol_mode=tol_mode_code(tol_mode),
                                         floor=float(metric[2]) if metric.numel() > 2 else 0.0,
                                         stats=stats)
            else:
                mx, nrot = ref.block_step(At[:, :m_pad], Vt, D, pairs[s], W, modes[s] == 1, tol,
                                          max_inner, tol_mode=tol_mode_code(tol_mode),
                                          floor=float(metric[2]) if metric.numel() > 2 else 0.0,
                                          order={2: "bipartite", 3: "cross"}.get(modes[s],
                                                                                 "cyclic"),
                                          stats=stats)
            metric[0] = max(float(metric[0]), mx)
            metric[1] += nrot
            if metric.numel() > 4:
                metric[3] = max(float(metric[3]), stats["smax"])
                metric[4] += stats.get("ncols", 0)


def gram_cross(At: torch.Tensor, m_pad: int, pairs: torch.Tensor, W: int,
               rows_per_chunk: int) -> torch.Tensor:
    """Cross Gram A_bi^T A_bj of every (bi, bj) in ``pairs`` (P, 2) on the
    device, split over row chunks as in a block step; returns the chunk slabs
    (P, nchunk, W, W)."""
    _check_layout(At, m_pad)
    pairs = pairs.to(torch.int32).contiguous().to(At.device)
    P = pairs.shape[0]
    nchunk = -(-m_pad // rows_per_chunk)
    slabs = torch.empty(P, nchunk, W, W, dtype=At.dtype, device=At.device)
    hip_check(hip_lib().svdj_gram_cross(dtype_code(At.dtype), W, _ptr(At), At.stride(0), m_pad,
                                        _ptr(pairs), P, rows_per_chunk, _ptr(slabs), _stream(At)),
              "gram_cross")
    return slabs


def gram_quad(At: torch.Tensor, m_pad: int, pairs: torch.Tensor, W: int,
              rows_per_chunk: int, parts: int = 3) -> torch.Tensor:
    """The six cross Grams of a quad step (fp32, W = 64): ``pairs`` (P, 2) on
    the device in quad order ((a, c), (b, d) per quad).  Returns the slabs
    (3P, nchunk, W, W): the P pairs' Grams, then C_ad, C_bc, C_ab, C_cd of
    every quad (csrc/hip/block.hip gram_quad_kernel; ``parts`` 2: the
    early-sweep form on 2 bf16 parts)."""
    _check_layout(At, m_pad)
    if At.dtype != torch.float32 or W != 64:
        raise ValueError("gram_quad: fp32 data, W = 64")
    pairs = pairs.to(torch.int32).contiguous().to(At.device)
    P = pairs.shape[0]
    nchunk = -(-m_pad // rows_per_chunk)
    slabs = torch.empty(3 * P, nchunk, W, W, dtype=At.dtype, device=At.device)
    hip_check(hip_lib().svdj_gram_quad(_ptr(At), At.stride(0), m_pad, _ptr(pairs), P,
                                       rows_per_chunk, _ptr(slabs), int(parts), _stream(At)),
              "gram_quad")
    return slabs


def apply_q(Xt: torch.Tensor, Q: torch.Tensor, W: int, mma="native"):
    """Xt (2W, ld) rows = columns of X, in place X <- X Q (device tensors)."""
    _check_layout(Xt, Xt.shape[1] // ROW_ALIGN * ROW_ALIGN)
    if Xt.shape[0] != 2 * W or tuple(Q.shape) != (2 * W, 2 * W) or not Q.is_contiguous():
        raise ValueError("Xt must be (2W, ld) and Q contiguous (2W, 2W)")
    rows = Xt.shape[1] // ROW_ALIGN * ROW_ALIGN
    hip_check(hip_lib().svdj_apply_q(dtype_code(Xt.dtype), W, mma_code(mma, Xt.dtype), _ptr(Xt),
                                     rows, Xt.stride(0), _ptr(Q), _stream(Xt)), "apply_q")


def block_solve(At, Vt, D, m_pad, W, tol, max_inner, max_sweeps, mma="native",
                tol_mode="relative", inner_order="cyclic", stop_rule="second_order"):
    """Single-device block Jacobi (round-robin over ncols/W blocks, first
    step of each sweep full; cross steps with ``inner_order``; stop test
    :func:`sweep_converged`).  Returns (sweeps, hist)."""
    step_modes([], inner_order)  # validates
    _check_layout(At, m_pad)
    check_block(At.dtype, W)
    ncols = At.shape[0]
    if At.is_cuda:
        nb = ncols // W
        ws = block_workspace(At.dtype, W, nb // 2, m_pad, At.device)
        metric = new_metric(At.device)
        hist = (C.c_double * max(max_sweeps, 1))()
        n_v = Vt.shape[1] if Vt is not None else 0
        ldv = Vt.stride(0) if Vt is not None else 0
        sweeps = hip_check(hip_lib().svdj_block_solve(
            dtype_code(At.dtype), W, m_pad, _ptr(At), At.stride(0), _ptr(Vt), n_v, ldv, _ptr(D),
            ncols, float(tol), tol_mode_code(tol_mode), int(max_inner), int(max_sweeps),
            INNER_ORDERS.index(inner_order), _ptr(ws), ws.numel(), _ptr(metric), hist,
            mma_code(mma, At.dtype), STOP_RULES[stop_rule], _stream(At)),
            "block_solve")
        return sweeps, [hist[i] for i in range(sweeps)]
    from ..parallel.schedule import round_robin

    nb = ncols // W
    pairs = torch.from_numpy(round_robin(nb))
    modes = [1] + [0] * (nb - 2)
    hist = []
    metric = new_metric("cpu")
    set_norm_floor(metric, At.dtype, m_pad, float(D.max()) if D.numel() else 1.0)
    for _ in range(max_sweeps):
        reset_metric(metric)
        block_steps(At, Vt, D, m_pad, pairs, W, modes, tol, max_inner, metric,
                    tol_mode=tol_mode, inner_order=inner_order)
        mx, ms, nrot, ncr = read_stop(metric)
        hist.append(mx)
        if sweep_converged(mx, ms, nrot, ncr, tol, tol_mode, stop_rule):
            break
    return len(hist), hist


__all__ = [
    "NativeError", "ROW_ALIGN", "SUPPORTED_BLOCK", "INNER_ORDERS", "step_modes", "dtype_code", "new_metric", "reset_metric", "set_norm_floor",
    "METRIC_WORDS", "read_stop", "metric_stop_values", "metric_work", "sweep_converged", "STOP_RULES",
    "read_metric", "set_identity", "col_norms2", "finalize", "scalar_step", "scalar_solve",
    "block_workspace", "block_steps", "block_solve", "check_block", "MMA_CODES", "mma_code",
    "apply_q",
    "gram_cross", "gram_quad",
]
