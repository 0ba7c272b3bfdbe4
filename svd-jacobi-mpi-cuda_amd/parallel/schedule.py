"""Pair / block-pair schedules (thin numpy wrappers of the native C++).

* :func:`sameh`        -- the reference's Sameh 1971 ordering
                          (reference main.cu:500-538, 945-983).
* :func:`round_robin`  -- circle-method tournament for block pairs on one GPU.
* :func:`bipartite`    -- cross pairs between the two resident super-blocks.
* :func:`tournament`   -- multi-GPU super-block tournament, one block
                          exchanged per GPU per round.
* :func:`distributed_sweep_plan` -- the per-GPU step list of one sweep.

Pure-Python twins (``*_py``) exist for cross-checking the native code.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..ops._native import cpu_lib


def _i32(shape):
    return np.zeros(shape, dtype=np.int32)


def _ptr(a):
    import ctypes as C

    return a.ctypes.data_as(C.POINTER(C.c_int32))


def sameh(n: int) -> np.ndarray:
    """(steps, n//2, 2) 0-based (p, q) pairs of the reference ordering."""
    lib = cpu_lib()
    steps = lib.svdj_sameh_num_steps(n)
    out = _i32((max(steps, 0), n // 2, 2))
    if steps > 0:
        lib.svdj_sameh_schedule(n, _ptr(out))
    return out


def round_robin(nb: int) -> np.ndarray:
    """(nb-1, nb//2, 2) pairs, nb even."""
    if nb < 2 or nb % 2:
        raise ValueError(f"round_robin needs an even count >= 2, got {nb}")
    out = _i32((nb - 1, nb // 2, 2))
    cpu_lib().svdj_round_robin(nb, _ptr(out))
    return out


def round_robin_padded(n: int) -> np.ndarray:
    """Round robin over n indices; for odd n a dummy index is paired and
    reported as -1."""
    nb = n + (n & 1)
    out = round_robin(nb)
    out[out >= n] = -1
    return out


def bipartite(k: int) -> np.ndarray:
    """(k, k, 2): step t pairs (a, k + (a+t) mod k)."""
    out = _i32((k, k, 2))
    cpu_lib().svdj_bipartite(k, _ptr(out))
    return out


@dataclass
class Tournament:
    P: int
    held: np.ndarray        # (rounds, P, 2) super-block ids per GPU slot
    xslot: np.ndarray       # (rounds, P) slot replaced before round r (r>=1)
    send_to: np.ndarray     # (rounds, P)
    recv_from: np.ndarray   # (rounds, P)

    @property
    def rounds(self) -> int:
        return self.held.shape[0]


def tournament(P: int) -> Tournament:
    R = 2 * P - 1
    held, xs, st, rf = _i32((R, P, 2)), _i32((R, P)), _i32((R, P)), _i32((R, P))
    cpu_lib().svdj_tournament(P, _ptr(held), _ptr(xs), _ptr(st), _ptr(rf))
    return Tournament(P, held, xs, st, rf)


# ------------------------------------------------------- quad-step orders
# A quad step (csrc/hip/block.hip "quad step") fuses two cross steps over
# the four blocks (a, b, c, d): step s pairs (a, c), (b, d), step s+1 pairs
# (a, d), (b, c), i.e. all cross pairs of the super-block pair {a, b} x
# {c, d}.  Pair 2q / 2q+1 of both steps belong to quad q, in that
# orientation (the kernels read the quad from the pair lists).  Mode codes:
# 4 = first step of a quad (does both), 5 = its second step.
QUAD_HEAD, QUAD_TAIL = 4, 5


def quad_round_robin(nb: int) -> np.ndarray:
    """(nb-1, nb//2, 2) block pairs covering every pair of nb blocks once,
    nb % 4 == 0: step 0 pairs the two blocks of every super-block (2i, 2i+1)
    (the full-Gram step of a sweep), then a round robin over the nb/2
    super-blocks, each super-step as the two steps of a quad (native:
    svdj_quad_round_robin)."""
    if nb < 4 or nb % 4:
        raise ValueError(f"quad_round_robin needs a multiple of 4 blocks, got {nb}")
    out = _i32((nb - 1, nb // 2, 2))
    cpu_lib().svdj_quad_round_robin(nb, _ptr(out))
    return out


def quad_round_robin_py(nb: int) -> np.ndarray:
    """Pure-Python twin of :func:`quad_round_robin`."""
    if nb < 4 or nb % 4:
        raise ValueError(f"quad_round_robin needs a multiple of 4 blocks, got {nb}")
    K = nb // 2
    out = _i32((nb - 1, K, 2))
    out[0, :, 0] = np.arange(0, nb, 2)
    out[0, :, 1] = np.arange(1, nb, 2)
    srr = round_robin(K)
    for t in range(K - 1):
        for q, (I, J) in enumerate(srr[t]):
            a, b, c, d = 2 * I, 2 * I + 1, 2 * J, 2 * J + 1
            out[1 + 2 * t, 2 * q] = (a, c)
            out[1 + 2 * t, 2 * q + 1] = (b, d)
            out[2 + 2 * t, 2 * q] = (a, d)
            out[2 + 2 * t, 2 * q + 1] = (b, c)
    return out


def quad_round_robin_modes(nb: int) -> list:
    return [1] + [QUAD_HEAD, QUAD_TAIL] * (nb // 2 - 1)


def quad_bipartite(xs, ys) -> np.ndarray:
    """(h, h, 2) cross pairs between block lists xs and ys (h = len, even)
    in quad order: super-step t pairs super-block (xs[2i], xs[2i+1]) with
    (ys[2j], ys[2j+1]), j = (i + t) mod h/2."""
    h = len(xs)
    if h < 2 or h % 2 or len(ys) != h:
        raise ValueError(f"quad_bipartite needs two even lists of equal length, got {h}, {len(ys)}")
    out = _i32((h, h, 2))
    x = np.ascontiguousarray(np.asarray(xs, dtype=np.int32))
    y = np.ascontiguousarray(np.asarray(ys, dtype=np.int32))
    cpu_lib().svdj_quad_bipartite(h, _ptr(x), _ptr(y), _ptr(out))
    return out


def quad_bipartite_py(xs, ys) -> np.ndarray:
    """Pure-Python twin of :func:`quad_bipartite`."""
    h = len(xs)
    if h < 2 or h % 2 or len(ys) != h:
        raise ValueError(f"quad_bipartite needs two even lists of equal length, got {h}, {len(ys)}")
    H = h // 2
    out = _i32((h, h, 2))
    for t in range(H):
        for i in range(H):
            j = (i + t) % H
            a, b, c, d = xs[2 * i], xs[2 * i + 1], ys[2 * j], ys[2 * j + 1]
            out[2 * t, 2 * i] = (a, c)
            out[2 * t, 2 * i + 1] = (b, d)
            out[2 * t + 1, 2 * i] = (a, d)
            out[2 * t + 1, 2 * i + 1] = (b, c)
    return out


def quad_bipartite_modes(h: int) -> list:
    return [QUAD_HEAD, QUAD_TAIL] * (h // 2)


def check_quad_steps(pairs: np.ndarray, modes) -> None:
    """Raise ValueError unless every mode-4 step and the following mode-5
    step hold quads in the orientation the kernels read."""
    modes = [int(x) for x in modes]
    for s, md in enumerate(modes):
        if md == QUAD_TAIL and (s == 0 or modes[s - 1] != QUAD_HEAD):
            raise ValueError(f"step {s}: quad tail without head")
        if md != QUAD_HEAD:
            continue
        if s + 1 >= len(modes) or modes[s + 1] != QUAD_TAIL:
            raise ValueError(f"step {s}: quad head without tail")
        p0, p1 = pairs[s], pairs[s + 1]
        if p0.shape[0] % 2:
            raise ValueError(f"step {s}: odd pair count {p0.shape[0]}")
        for q in range(p0.shape[0] // 2):
            (a, c), (b, d) = p0[2 * q], p0[2 * q + 1]
            if tuple(p1[2 * q]) != (a, d) or tuple(p1[2 * q + 1]) != (b, c):
                raise ValueError(f"steps {s},{s + 1} quad {q}: not (a,c),(b,d) / (a,d),(b,c)")


# ------------------------------------------------------------ python twins
def sameh_py(n: int) -> np.ndarray:
    M = (n + 1) // 2
    steps = n - 1 if n % 2 == 0 else n
    out = -np.ones((steps, n // 2, 2), dtype=np.int32)
    s = 0
    for k in range(1, M):
        for slot, q in enumerate(range(M - k + 1, n - k + 1)):
            if q <= 2 * M - 2 * k:
                p = 2 * M - 2 * k + 1 - q
            elif q <= 2 * M - k - 1:
                p = 4 * M - 2 * k - q
            else:
                p = n
            out[s, slot] = (p - 1, q - 1)
        s += 1
    for k in range(M, 2 * M):
        for slot, q in enumerate(range(4 * M - n - k, 3 * M - k)):
            if q < 2 * M - k + 1:
                p = n
            elif q <= 4 * M - 2 * k - 1:
                p = 4 * M - 2 * k - q
            else:
                p = 6 * M - 2 * k - 1 - q
            out[s, slot] = (p - 1, q - 1)
        s += 1
    return out


def round_robin_py(nb: int) -> np.ndarray:
    out = np.zeros((nb - 1, nb // 2, 2), dtype=np.int32)
    for r in range(nb - 1):
        out[r, 0] = (r, nb - 1)
        for k in range(1, nb // 2):
            a, b = (r + k) % (nb - 1), (r - k + nb - 1) % (nb - 1)
            out[r, k] = (min(a, b), max(a, b))
    return out


# ---------------------------------------------------------- sweep planning
@dataclass
class RoundPlan:
    """Local work of one tournament round on one GPU.

    ``pairs`` are LOCAL block indices into the GPU's resident buffer, which
    holds slot 0 in blocks [0, k) and slot 1 in blocks [k, 2k)."""
    pairs: np.ndarray   # (steps, k, 2)
    modes: list         # per step 0 cross / 1 full


def distributed_sweep_plan(P: int, k: int) -> list:
    """Per-round local plans for a sweep with P GPUs, k blocks per super-block.

    Round 0: full round robin over the 2k resident blocks (covers the
    within-super-block pairs of all 2P super-blocks once); its first step
    uses the full Gram (refresh).  Rounds 1..2P-2: bipartite cross pairs
    between the two resident super-blocks.  Every block pair of the whole
    matrix is visited exactly once per sweep.
    """
    plans = [RoundPlan(round_robin(2 * k), [1] + [0] * (2 * k - 2))]
    bp = bipartite(k)
    for _ in range(1, 2 * P - 1):
        plans.append(RoundPlan(bp, [0] * k))
    return plans
