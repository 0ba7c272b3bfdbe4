"""Plain-PyTorch reference implementations of every device op.

These run on CPU tensors.  They are the numerics oracle for the HIP kernels
(tests compare kernel output against them, in fp64) and the compute path of
the CPU-only multi-process tests (gloo), so the distributed orchestration is
exercised end to end without a GPU.  They are never used for GPU tensors.

Layout: a column-major matrix is held as its transpose ``At`` (ncols, ld):
row c of ``At`` is column c of the matrix (contiguous, like the kernels).
"""
from __future__ import annotations

import math

import torch


def _rotation(alpha, beta, gamma):
    """Reference symmetric-Schur rotation (reference main.cu:715-725), batched."""
    safe = torch.where(alpha == 0, torch.ones_like(alpha), alpha)
    tau = (gamma - beta) / (2 * safe)
    big = 1e150 if alpha.dtype == torch.float64 else 1e18
    at = tau.abs()
    t = torch.where(at > big, 1.0 / (2 * tau), 1.0 / (at + torch.sqrt(1 + torch.clamp(tau * tau, max=1e300 if alpha.dtype == torch.float64 else 3e38))))
    t = torch.where((at <= big) & (tau < 0), -t, t)
    c = 1.0 / torch.sqrt(1 + t * t)
    s = t * c
    return c, s, t


def scalar_step(At, Vt, pairs, tol, tol_mode=0):
    """One parallel step of the scalar method on disjoint column pairs.

    pairs: int tensor (k, 2) (negative entries skipped).  Returns (maxconv, rotations).
    """
    pairs = pairs[(pairs[:, 0] >= 0) & (pairs[:, 1] >= 0)]
    if pairs.numel() == 0:
        return 0.0, 0
    p, q = pairs[:, 0].long(), pairs[:, 1].long()
    x, y = At[p], At[q]
    alpha = (x * y).sum(1)
    beta = (x * x).sum(1)
    gamma = (y * y).sum(1)
    nrm = beta.sqrt() * gamma.sqrt()
    conv = torch.where(nrm > 0, alpha.abs() / torch.where(nrm > 0, nrm, torch.ones_like(nrm)), torch.zeros_like(nrm))
    if tol_mode == 1:
        rot = alpha.abs() > tol
    else:
        rot = (nrm > 0) & (alpha.abs() > tol * nrm)
    rot &= alpha != 0
    maxconv = float(conv.max()) if conv.numel() else 0.0
    if not bool(rot.any()):
        return maxconv, 0
    c, s, _ = _rotation(alpha, beta, gamma)
    c = torch.where(rot, c, torch.ones_like(c))[:, None]
    s = torch.where(rot, s, torch.zeros_like(s))[:, None]
    At[p] = c * x - s * y
    At[q] = s * x + c * y
    if Vt is not None:
        vx, vy = Vt[p], Vt[q]
        Vt[p] = c * vx - s * vy
        Vt[q] = s * vx + c * vy
    return maxconv, int(rot.sum())


def round_robin_pairs(N):
    out = []
    for r in range(N - 1):
        prs = [(r, N - 1)]
        for k in range(1, N // 2):
            a, b = (r + k) % (N - 1), (r - k + N - 1) % (N - 1)
            prs.append((min(a, b), max(a, b)))
        out.append(prs)
    return out


_RR_CACHE = {}


def bipartite_pairs(W):
    """Cross-pair ordering of the bipartite EVD (block.hip Ord<W, EVD_BIP>):
    step t pairs local column a of block i with column (a + t) mod W of
    block j (player W + ...), W steps per sweep."""
    return [[(a, W + (a + t) % W) for a in range(W)] for t in range(W)]


def jacobi_evd(G, tol, max_sweeps, tol_mode: int = 0, order: str = "cyclic", floor: float = 0.0,
               stats: dict | None = None):
    """Cyclic parallel Jacobi EVD of a batch of SPD matrices G (P, N, N).

    Same orderings (``cyclic``: circle-method round robin over all pairs;
    ``bipartite``: the cross pairs only; ``cross``: the bipartite steps with
    the within-block couplings held at zero, i.e. only the cross couplings
    and the diagonal tracked -- block.hip evd_cross_kernel), threshold and
    update formulas as the kernels.  Returns (G_diag_final, Q, rotated);
    with ``stats`` (a dict) the second-order stop test's inputs
    (csrc/include/svdj_stop.h) accumulate: ``smax`` the largest effective
    sine (|s| times the larger norm ratio after the rotation) and ``ncols``
    the number of column rotations applied.
    """
    G = G.clone()
    P, N, _ = G.shape
    Q = torch.eye(N, dtype=G.dtype).expand(P, N, N).clone()
    key = (N, "cyclic" if order == "cyclic" else "bipartite")
    sched = _RR_CACHE.get(key)
    if sched is None:
        prs_all = round_robin_pairs(N) if order == "cyclic" else bipartite_pairs(N // 2)
        sched = [(torch.tensor([a for a, b in prs]), torch.tensor([b for a, b in prs]))
                 for prs in prs_all]
        _RR_CACHE[key] = sched
    within = None
    if order == "cross":  # within-block couplings are never tracked
        W = N // 2
        within = torch.ones(N, N, dtype=torch.bool)
        within[:W, W:] = False
        within[W:, :W] = False
        within.fill_diagonal_(False)
        G[:, within] = 0
    rotated = torch.zeros(P, dtype=torch.bool)
    for _ in range(max_sweeps):
        sweep_rot = torch.zeros(P, dtype=torch.bool)
        for p, q in sched:
            gpp, gqq, gpq = G[:, p, p], G[:, q, q], G[:, p, q]
            nrm = gpp.clamp(min=0).sqrt() * gqq.clamp(min=0).sqrt()
            rot = (gpq.abs() > tol) if tol_mode == 1 else (
                (nrm > 0) & (gpq.abs() > tol * nrm) & (torch.minimum(gpp, gqq) > floor))
            if not bool(rot.any()):
                continue
            sweep_rot |= rot.any(1)
            c, s, t = _rotation(gpq, gpp, gqq)
            c = torch.where(rot, c, torch.ones_like(c))
            s = torch.where(rot, s, torch.zeros_like(s))
            t = torch.where(rot, t, torch.zeros_like(t))
            if stats is not None:  # second-order stop test (csrc/include/svdj_stop.h)
                dp, dq = (gpp - t * gpq).abs(), (gqq + t * gpq).abs()
                lo, hi = torch.minimum(dp, dq), torch.maximum(dp, dq)
                eff = torch.where(lo > 0, s.abs() * (hi / torch.where(lo > 0, lo, torch.ones_like(lo))).sqrt(),
                                  torch.ones_like(lo))
                eff = torch.where(rot, eff, torch.zeros_like(eff))
                stats["smax"] = max(stats.get("smax", 0.0), float(eff.max()))
                stats["ncols"] = stats.get("ncols", 0) + int(rot.sum())
            Gp, Gq = G[:, p, :].clone(), G[:, q, :].clone()
            G[:, p, :] = c[:, :, None] * Gp - s[:, :, None] * Gq
            G[:, q, :] = s[:, :, None] * Gp + c[:, :, None] * Gq
            Gp, Gq = G[:, :, p].clone(), G[:, :, q].clone()
            G[:, :, p] = c[:, None, :] * Gp - s[:, None, :] * Gq
            G[:, :, q] = s[:, None, :] * Gp + c[:, None, :] * Gq
            # exact diagonal-block update (matches the kernel)
            G[:, p, p] = gpp - t * gpq
            G[:, q, q] = gqq + t * gpq
            G[:, p, q] = torch.where(rot, torch.zeros_like(gpq), G[:, p, q])
            G[:, q, p] = G[:, p, q]
            if within is not None:
                G[:, within] = 0
            Qp, Qq = Q[:, :, p].clone(), Q[:, :, q].clone()
            Q[:, :, p] = c[:, None, :] * Qp - s[:, None, :] * Qq
            Q[:, :, q] = s[:, None, :] * Qp + c[:, None, :] * Qq
        rotated |= sweep_rot
        if not bool(sweep_rot.any()):
            break
    return torch.diagonal(G, dim1=1, dim2=2).clone(), Q, rotated


def block_step(At, Vt, D, pairs, W, full, tol, max_inner, tol_mode: int = 0,
               order: str = "cyclic", floor: float = 0.0, stats: dict | None = None):
    """One block step on P disjoint block pairs (pairs: (P, 2) block ids).

    Mirrors csrc/hip/block.hip (gram -> evd -> apply).  Updates At, Vt, D in
    place.  ``order`` is the EVD ordering of a cross step (a full step is
    always cyclic).  Returns (maxconv, pairs_rotated).
    """
    P = pairs.shape[0]
    if P == 0:
        return 0.0, 0
    ar = torch.arange(W)
    ci = pairs[:, 0].long()[:, None] * W + ar
    cj = pairs[:, 1].long()[:, None] * W + ar
    cols = torch.cat([ci, cj], 1)  # (P, 2W)
    X = At[cols]  # (P, 2W, ld)
    N = 2 * W
    idx = torch.arange(N)
    if full:
        G = X @ X.transpose(1, 2)
        mask = torch.triu(torch.ones(N, N, dtype=torch.bool), 1)
    else:
        C = X[:, :W] @ X[:, W:].transpose(1, 2)
        G = torch.zeros(P, N, N, dtype=At.dtype)
        G[:, idx, idx] = D[cols]
        G[:, :W, W:] = C
        G[:, W:, :W] = C.transpose(1, 2)
        mask = torch.zeros(N, N, dtype=torch.bool)
        mask[:W, W:] = True
    dg = torch.diagonal(G, dim1=1, dim2=2).clamp(min=0).sqrt()
    den = dg[:, :, None] * dg[:, None, :]
    R = torch.where(den > 0, G.abs() / torch.where(den > 0, den, torch.ones_like(den)), torch.zeros_like(den))
    if tol_mode != 1 and floor > 0:  # couplings of negligible columns do not count
        big = torch.diagonal(G, dim1=1, dim2=2) > floor
        R = torch.where(big[:, :, None] & big[:, None, :], R, torch.zeros_like(R))
    maxconv = float(R[:, mask].max()) if mask.any() else 0.0
    lam, Q, rotated = jacobi_evd(G, tol, max_inner, tol_mode,
                                 order="cyclic" if full else order, floor=floor, stats=stats)
    if bool(rotated.any()):
        sel = rotated
        Qs = Q[sel]
        csel = cols[sel]
        At[csel] = Qs.transpose(1, 2) @ X[sel]
        if Vt is not None:
            Vt[csel] = Qs.transpose(1, 2) @ Vt[csel]
    upd = rotated if not full else torch.ones_like(rotated)
    if bool(upd.any()):
        D[cols[upd]] = lam[upd]
    return maxconv, int(rotated.sum())


def quad_step(At, Vt, D, pairs0, pairs1, W, tol, max_inner, tol_mode: int = 0,
              floor: float = 0.0, stats: dict | None = None):
    """Two cross steps fused as one quad step (csrc/hip/block.hip "quad
    step"), on the quads of ``pairs0`` ((a,c), (b,d) per quad) and
    ``pairs1`` ((a,d), (b,c)).  The couplings of the second step come from
    the Gram blocks of the first and its rotations (Gram space), the two
    EVDs are cross-only, and the data is updated once by T = T1 T2.
    Returns (maxconv, pairs_rotated) over both steps."""
    Q = pairs0.shape[0] // 2
    if Q == 0:
        return 0.0, 0
    p0, p1 = pairs0.long().view(Q, 2, 2), pairs1.long().view(Q, 2, 2)
    a, c, b, d = p0[:, 0, 0], p0[:, 0, 1], p0[:, 1, 0], p0[:, 1, 1]
    if not (bool((p1[:, 0, 0] == a).all()) and bool((p1[:, 0, 1] == d).all())
            and bool((p1[:, 1, 0] == b).all()) and bool((p1[:, 1, 1] == c).all())):
        raise ValueError("quad steps need pairs (a,c),(b,d) then (a,d),(b,c)")
    ar = torch.arange(W)
    blk = torch.stack([a, b, c, d], 1)                       # (Q, 4) in [a b c d] order
    cols = (blk[:, :, None] * W + ar).reshape(Q, 4 * W)      # quad columns
    X = At[cols]                                             # (Q, 4W, ld)
    G = X @ X.transpose(1, 2)                                # only off-diagonal blocks used
    Dq = D[cols]
    N = 2 * W
    ia, ib, ic, id_ = (torch.arange(W) + k * W for k in range(4))

    def evd(x_idx, y_idx, C):
        Gp = torch.zeros(C.shape[0], N, N, dtype=At.dtype)
        n_idx = torch.arange(N)
        Gp[:, n_idx, n_idx] = torch.cat([Dq[:, x_idx], Dq[:, y_idx]], 1)
        Gp[:, :W, W:] = C
        Gp[:, W:, :W] = C.transpose(1, 2)
        dg = torch.cat([Dq[:, x_idx], Dq[:, y_idx]], 1).clamp(min=0).sqrt()
        den = dg[:, :W, None] * dg[:, None, W:]
        R = torch.where(den > 0, C.abs() / torch.where(den > 0, den, torch.ones_like(den)),
                        torch.zeros_like(den))
        if tol_mode != 1 and floor > 0:
            big = torch.cat([Dq[:, x_idx], Dq[:, y_idx]], 1) > floor
            R = torch.where(big[:, :W, None] & big[:, None, W:], R, torch.zeros_like(R))
        mx = float(R.max()) if R.numel() else 0.0
        lam, Qm, rot = jacobi_evd(Gp, tol, max_inner, tol_mode, order="cross", floor=floor,
                                  stats=stats)
        lam = torch.where(rot[:, None], lam, torch.cat([Dq[:, x_idx], Dq[:, y_idx]], 1))
        Dq[:, x_idx], Dq[:, y_idx] = lam[:, :W], lam[:, W:]
        eye = torch.eye(N, dtype=At.dtype).expand_as(Qm)
        return torch.where(rot[:, None, None], Qm, eye), mx, int(rot.sum())

    Qac, m1, r1 = evd(ia, ic, G[:, ia][:, :, ic])
    Qbd, m2, r2 = evd(ib, id_, G[:, ib][:, :, id_])
    T1 = torch.zeros(Q, 4 * W, 4 * W, dtype=At.dtype)
    ac, bd = torch.cat([ia, ic]), torch.cat([ib, id_])
    T1[:, ac[:, None], ac[None, :]] = Qac
    T1[:, bd[:, None], bd[None, :]] = Qbd
    G1 = T1.transpose(1, 2) @ G @ T1                         # Gram of [a' b' c' d']
    Qad, m3, r3 = evd(ia, id_, G1[:, ia][:, :, id_])
    Qbc, m4, r4 = evd(ib, ic, G1[:, ib][:, :, ic])
    T2 = torch.zeros_like(T1)
    ad, bc = torch.cat([ia, id_]), torch.cat([ib, ic])
    T2[:, ad[:, None], ad[None, :]] = Qad
    T2[:, bc[:, None], bc[None, :]] = Qbc
    T = T1 @ T2
    nrot = r1 + r2 + r3 + r4
    if nrot:
        At[cols] = T.transpose(1, 2) @ X
        if Vt is not None:
            Vt[cols] = T.transpose(1, 2) @ Vt[cols]
    D[cols] = Dq
    return max(m1, m2, m3, m4), nrot


def col_norms2(At):
    return (At.double() ** 2).sum(1).to(At.dtype)


def finalize(At, scale_u=True):
    sig = (At.double() ** 2).sum(1).sqrt()
    if scale_u:
        nz = sig > 0
        At[nz] = (At[nz].double() / sig[nz, None]).to(At.dtype)
    return sig.to(At.dtype)


def default_tol(dtype, m):
    from ..utils.metrics import default_tol as _dt
    return _dt(dtype, m)
