"""Two-level block Jacobi: the block pairs of a super-block pair are solved in
Gram space, and A and V are rotated once per super-block pair with one
large-K matrix-core GEMM.

The one-level block path (models/block.py, parallel/pipeline.py) rotates a
pair of W-column blocks per step: Gram (m x W x W), EVD, then
[A_i A_j] <- [A_i A_j] Q with K = 2W.  At W = 64 that apply moves 1 KB of A
and V per 32 KFLOP, so it sits at the HBM / fp32-MFMA balance point, and the
Gram of the next step re-reads what the apply just wrote.  Here the columns
are cut into S super-blocks of Wb >= 4W columns and a sweep is a round robin
over super-blocks.  For every super-block pair X = [A_I A_J] of a round:

1. G = X^T X.  Only the cross block A_I^T A_J is a fresh GEMM over the m
   rows; the diagonal blocks A_I^T A_I are carried from the previous round
   (they are Gram blocks of the small factor below) and recomputed from A in
   round 0 of every sweep;
2. Y = chol(G)^T (2Wb x 2Wb, fp64 factorisation): Y^T Y = X^T X, so the
   rotations that orthogonalise the columns of Y are the ones that
   orthogonalise X;
3. the W-block pairs of X (round 0: all of them, by round robin; later
   rounds: the I x J cross pairs, bipartite) run through the existing
   Gram -> EVD -> apply kernels (csrc/hip/block.hip) on Y, whose columns
   have 2Wb rows instead of m, accumulating Q_X (2Wb x 2Wb) in place of V;
4. X <- X Q_X and V_X <- V_X Q_X: one GEMM with K = 2Wb per output half,
   written out of place into the next round's placement (ping-pong
   buffers), so every super-block pair of the next round is contiguous.

The work on A and V is the same 8 n^3 + n^2 m FLOP per sweep as the
one-level path, but as GEMMs with K = 2Wb, which run at the matrix-core
rate instead of the HBM rate.  The Gram-space problems are 2Wb / m of the
size and stay in the caches.

Accuracy: Q_X is orthogonal to fp32 rounding whatever Y is, so A V = A_0
holds as in the one-level path; Y only steers the rotations.  The stop test
is the same relative test on the block Grams, evaluated on Y's columns,
whose Grams equal X's up to the fp32 Gram rounding.  A super-block pair
whose Gram does not factor (numerically dependent columns) is left
unrotated in that round and the sweep is not counted as converged.

Reference: the per-pair host loop this replaces is reference main.cu:685-852
(dot triple 698-707, rotation 734).
"""
from __future__ import annotations

import numpy as np
import torch

from svdj.ops import kernels as K
from svdj.parallel.schedule import bipartite, round_robin


def usable(ncols: int, W: int, Wb: int) -> bool:
    """Geometry check: Wb a multiple of 2W (whole W-blocks, even block count
    per super-block) and at least 4 super-blocks."""
    return Wb % (2 * W) == 0 and ncols % (2 * Wb) == 0 and ncols // Wb >= 4


class TwoLevel:
    """Two-level solver state for one (ncols, m_pad, n_v, W, Wb) geometry on
    one device.  Buffers are allocated once and reused across solves."""

    def __init__(self, ncols: int, m_pad: int, n_v: int, W: int, Wb: int, dtype, device,
                 want_v: bool = True):
        if not usable(ncols, W, Wb):
            raise ValueError(f"two-level geometry: ncols={ncols} W={W} Wb={Wb}")
        if dtype != torch.float32:
            raise ValueError("two-level path: fp32")
        self.ncols, self.m_pad, self.n_v, self.W, self.Wb = ncols, m_pad, n_v, W, Wb
        self.dtype, self.device, self.want_v = dtype, torch.device(device), want_v
        S = self.S = ncols // Wb
        self.H = S // 2                     # super-block pairs per round
        k = self.k = Wb // W                # W-blocks per super-block
        N2 = self.N2 = 2 * Wb               # columns of one super-block pair
        dev = self.device
        self.sched = round_robin(S)         # (S-1, H, 2) super-block labels
        # placement: the super-block labelled L sits at position pos[L]; a
        # round's pair s occupies positions (2s, 2s+1).  Labels are chosen so
        # that round 0's pairs are adjacent in the canonical column order.
        self.label0 = np.empty(S, dtype=np.int64)   # canonical position -> label
        for s, (a, b) in enumerate(self.sched[0]):
            self.label0[2 * s], self.label0[2 * s + 1] = a, b
        # Gram-space buffers (all super-block pairs of a round at once)
        self.Y = torch.empty(self.H * N2, N2, dtype=dtype, device=dev)
        self.Q = torch.empty(self.H * N2, N2, dtype=dtype, device=dev)
        self.Dy = torch.empty(self.H * N2, dtype=dtype, device=dev)
        self.G = torch.empty(self.H, N2, N2, dtype=torch.float64, device=dev)
        self.Gint = torch.empty(S, Wb, Wb, dtype=dtype, device=dev)  # by label
        self.eye = torch.eye(N2, dtype=dtype, device=dev)
        # ping-pong storage
        self.At2 = None
        self.Vt2 = None
        # inner pair lists on Gram-space block ids (pair s owns blocks
        # [s 2k, (s+1) 2k)): round 0 all pairs (round robin, first step full),
        # later rounds the I x J cross pairs
        off = (np.arange(self.H, dtype=np.int32) * 2 * k)[None, :, None, None]
        rr = round_robin(2 * k)[:, None, :, :] + off          # (2k-1, H, k, 2)
        bp = bipartite(k)[:, None, :, :] + off                # (k, H, k, 2)
        self.pairs0 = torch.from_numpy(np.ascontiguousarray(
            rr.reshape(2 * k - 1, self.H * k, 2))).to(dev)
        self.modes0 = [1] + [0] * (2 * k - 2)
        self.pairsX = torch.from_numpy(np.ascontiguousarray(bp.reshape(k, self.H * k, 2))).to(dev)
        self.modesX = [0] * k
        self.ws = {}

    # ------------------------------------------------------------------
    def _alt(self, At, Vt):
        if self.At2 is None or self.At2.shape != At.shape:
            self.At2 = torch.empty_like(At)
        if Vt is not None and (self.Vt2 is None or self.Vt2.shape != Vt.shape):
            self.Vt2 = torch.empty_like(Vt)
        return self.At2, (self.Vt2 if Vt is not None else None)

    def _rows(self, pos: int):
        return slice(pos * self.Wb, (pos + 1) * self.Wb)

    def solve(self, At, Vt, tol, max_sweeps, metric, max_inner=1, tol_mode="relative",
              inner_order="bipartite", reduce_metric=None, progress=None):
        """Sweeps on At (ncols, ld) / Vt (ncols, ldv) in canonical column
        order until a sweep rotates nothing.  Returns (sweeps, hist); the
        result is in At / Vt (canonical order) on return."""
        S, H, Wb, N2, m_pad = self.S, self.H, self.Wb, self.N2, self.m_pad
        A_alt, V_alt = self._alt(At, Vt)
        cur = [At, Vt]
        nxt = [A_alt, V_alt]
        pos = np.empty(S, dtype=np.int64)
        pos[self.label0] = np.arange(S)
        floor = K.norm_floor(self.dtype, m_pad)
        fail = torch.zeros((), dtype=torch.int32, device=self.device)
        hist = []
        sweeps = 0
        R = S - 1
        for sw in range(max_sweeps):
            K.reset_metric(metric)
            fail.zero_()
            for r in range(R):
                prs = self.sched[r]
                Ac, Vc = cur
                An, Vn = nxt
                # ---- 1. Gram of every super-block pair (contiguous at 2s, 2s+1)
                for s in range(H):
                    a, b = int(prs[s, 0]), int(prs[s, 1])
                    pa, pb = int(pos[a]), int(pos[b])
                    assert pb == pa + 1 and pa == 2 * s, (r, s, pa, pb)
                    X = Ac[pa * Wb:(pa + 2) * Wb, :m_pad]
                    Gs = self.G[s]
                    if r == 0:
                        torch.mm(X, X.t(), out=self.Y[s * N2:(s + 1) * N2])
                        Gs.copy_(self.Y[s * N2:(s + 1) * N2])
                    else:
                        C = torch.mm(X[:Wb], X[Wb:].t())
                        Gs[:Wb, Wb:].copy_(C)
                        Gs[Wb:, :Wb].copy_(C.t())
                        Gs[:Wb, :Wb].copy_(self.Gint[a])
                        Gs[Wb:, Wb:].copy_(self.Gint[b])
                # ---- 2. Y = chol(G)^T in the kernels' layout (row c = column c of Y
                # = row c of L): zero columns get a unit pivot (never rotated)
                d = torch.diagonal(self.G, dim1=1, dim2=2)
                dead = d <= floor
                self.Dy.copy_(d.reshape(-1))
                Gm = self.G.masked_fill(dead[:, :, None] | dead[:, None, :], 0.0)
                torch.diagonal(Gm, dim1=1, dim2=2).masked_fill_(dead, 1.0)
                L, info = torch.linalg.cholesky_ex(Gm)
                bad = info != 0
                fail += bad.sum().to(torch.int32)
                # unfactorable pair: Y = diag(sqrt(d)) -> no rotation this round
                Ldiag = torch.diag_embed(torch.sqrt(torch.diagonal(Gm, dim1=1, dim2=2)))
                L = torch.where(bad[:, None, None], Ldiag, L)
                self.Y.view(H, N2, N2).copy_(L)
                self.Q.view(H, N2, N2).copy_(self.eye)
                # ---- 3. block Jacobi on Y, Q accumulated
                if r == 0:
                    pairs, modes = self.pairs0, self.modes0
                else:
                    pairs, modes = self.pairsX, self.modesX
                K.block_steps(self.Y, self.Q, self.Dy, N2, pairs, self.W, modes, tol, max_inner,
                              metric, 0, pool=self.ws, tol_mode=tol_mode, inner_order=inner_order)
                # carried diagonal Gram blocks of the rotated super-blocks
                Yv = self.Y.view(H, N2, N2)
                Gi = torch.bmm(Yv[:, :Wb], Yv[:, :Wb].transpose(1, 2))
                Gj = torch.bmm(Yv[:, Wb:], Yv[:, Wb:].transpose(1, 2))
                la = torch.from_numpy(prs[:, 0].astype(np.int64)).to(self.device)
                lb = torch.from_numpy(prs[:, 1].astype(np.int64)).to(self.device)
                self.Gint.index_copy_(0, la, Gi)
                self.Gint.index_copy_(0, lb, Gj)
                # ---- 4. X <- X Q_X, V_X <- V_X Q_X into the next placement
                nprs = self.sched[(r + 1) % R]
                npos = np.empty(S, dtype=np.int64)
                for s2 in range(H):
                    npos[int(nprs[s2, 0])] = 2 * s2
                    npos[int(nprs[s2, 1])] = 2 * s2 + 1
                Qv = self.Q.view(H, N2, N2)
                for s in range(H):
                    a, b = int(prs[s, 0]), int(prs[s, 1])
                    pa = int(pos[a])
                    for lab, half in ((a, 0), (b, 1)):
                        q = Qv[s, half * Wb:(half + 1) * Wb]          # (Wb, 2Wb) rows of Q^T
                        dst = self._rows(int(npos[lab]))
                        torch.mm(q, Ac[pa * Wb:(pa + 2) * Wb, :m_pad], out=An[dst, :m_pad])
                        if Vc is not None:
                            torch.mm(q, Vc[pa * Wb:(pa + 2) * Wb], out=Vn[dst])
                pos = npos
                cur, nxt = nxt, cur
            mx, nrot = reduce_metric(metric) if reduce_metric else K.read_metric(metric)
            nfail = int(fail)
            hist.append(mx)
            sweeps = sw + 1
            if progress:
                progress(sweeps, mx, nrot, nfail)
            if nrot == 0 and nfail == 0:
                break
        # back to canonical column order: canonical position p holds label0[p]
        Ac, Vc = cur
        src = torch.from_numpy(pos[self.label0]).to(self.device)
        perm = (src[:, None] * Wb + torch.arange(Wb, device=self.device)[None, :]).reshape(-1)
        if Ac is At:  # gather into the spare buffer, then copy back
            torch.index_select(Ac, 0, perm, out=self.At2)
            At.copy_(self.At2)
            if Vt is not None:
                torch.index_select(Vc, 0, perm, out=self.Vt2)
                Vt.copy_(self.Vt2)
        else:
            torch.index_select(Ac, 0, perm, out=At)
            if Vt is not None:
                torch.index_select(Vc, 0, perm, out=Vt)
        return sweeps, hist
