"""Schedules: reference Sameh ordering parity + tournament properties (CPU)."""
import itertools

import numpy as np
import pytest

from svdj.parallel import schedule as S


def _check_cover(steps, n, expect_all=True):
    seen = set()
    for st in steps:
        cols = [c for pq in st for c in pq if c >= 0]
        assert len(cols) == len(set(cols)), "column repeated within a step"
        for p, q in st:
            if p < 0 or q < 0:
                continue
            assert 0 <= p < n and 0 <= q < n and p != q
            key = (min(p, q), max(p, q))
            assert key not in seen, f"pair {key} twice in a sweep"
            seen.add(key)
    if expect_all:
        assert len(seen) == n * (n - 1) // 2


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 100, 101])
def test_sameh_native_matches_python_and_covers(n):
    a = S.sameh(n)
    b = S.sameh_py(n)
    assert np.array_equal(a, b)
    assert a.shape[0] == (n - 1 if n % 2 == 0 else n)
    _check_cover(a, n)


def test_sameh_worked_example_n8():
    # SURVEY.md section 2.7 (reference main.cu:526-538, 971-983)
    a = S.sameh(8)
    assert a[0].tolist() == [[2, 3], [1, 4], [0, 5], [7, 6]]
    assert a[3].tolist() == [[7, 3], [2, 4], [1, 5], [0, 6]]
    assert a[6].tolist() == [[7, 0], [6, 1], [5, 2], [4, 3]]


@pytest.mark.parametrize("nb", [2, 4, 6, 8, 16, 64])
def test_round_robin(nb):
    a = S.round_robin(nb)
    assert np.array_equal(a, S.round_robin_py(nb))
    _check_cover(a, nb)


@pytest.mark.parametrize("n", [5, 7, 9])
def test_round_robin_padded_odd(n):
    _check_cover(S.round_robin_padded(n), n)


@pytest.mark.parametrize("k", [1, 2, 3, 8])
def test_bipartite(k):
    a = S.bipartite(k)
    pairs = {(int(p), int(q)) for st in a for p, q in st}
    assert pairs == {(x, y) for x in range(k) for y in range(k, 2 * k)}
    for st in a:
        cols = st.reshape(-1).tolist()
        assert len(cols) == len(set(cols))


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 8])
def test_tournament_one_exchange_per_round(P):
    t = S.tournament(P)
    assert t.rounds == 2 * P - 1
    seen = set()
    for r in range(t.rounds):
        blocks = t.held[r].reshape(-1).tolist()
        assert sorted(blocks) == list(range(2 * P))
        for g in range(P):
            a, b = t.held[r, g]
            key = (min(a, b), max(a, b))
            assert key not in seen
            seen.add(key)
        if r == 0:
            continue
        for g in range(P):
            x = t.xslot[r, g]
            assert x in (0, 1)
            # the other slot is kept
            assert t.held[r, g, 1 - x] == t.held[r - 1, g, 1 - x]
            src = t.recv_from[r, g]
            assert t.send_to[r, src] == g
            # what arrives is what src sent
            assert t.held[r, g, x] == t.held[r - 1, src, t.xslot[r, src]]
    assert len(seen) == P * (2 * P - 1)


@pytest.mark.parametrize("P,k", [(1, 1), (1, 3), (2, 1), (2, 2), (3, 2), (4, 1), (4, 3)])
def test_distributed_sweep_covers_every_block_pair_once(P, k):
    """Simulate placement + local plans: every W-block pair exactly once per sweep,
    over two consecutive sweeps (the second starts from the permuted placement)."""
    t = S.tournament(P)
    plans = S.distributed_sweep_plan(P, k)
    phys = [[int(t.held[0, g, 0]), int(t.held[0, g, 1])] for g in range(P)]
    nblocks = 2 * P * k
    for _sweep in range(2):
        seen = set()
        for r in range(t.rounds):
            if r > 0:
                old = [list(x) for x in phys]
                for g in range(P):
                    src = int(t.recv_from[r, g])
                    phys[g][int(t.xslot[r, g])] = old[src][int(t.xslot[r, src])]
            for g in range(P):
                for st in plans[r].pairs:
                    for a, b in st:
                        ga = phys[g][a // k] * k + a % k
                        gb = phys[g][b // k] * k + b % k
                        key = (min(ga, gb), max(ga, gb))
                        assert key not in seen
                        seen.add(key)
        assert len(seen) == nblocks * (nblocks - 1) // 2
        assert plans[0].modes[0] == 1 and all(m == 0 for m in plans[0].modes[1:])


def test_evd_ring_matches_dpp_movement():
    """The EVD kernel computes slot players arithmetically (ring_slot in
    csrc/hip/block.hip) for the G updates, while the register Q follows the
    DPP shifts; both must describe the same circle-method movement and cover
    every pair once per N-1 steps."""
    def ring_player(W, pos, st):
        R = 2 * W - 1
        x = pos - st
        x += R if x < 0 else 0
        return 0 if x + 1 == R else x + 1

    for W in (4, 8, 32, 64):
        N = 2 * W
        pf = [N - 1 if a == 0 else a for a in range(W)]
        ps = [0 if a == 0 else N - 1 - a for a in range(W)]
        seen = set()
        for st in range(N - 1):
            for a in range(W):
                p = N - 1 if a == 0 else ring_player(W, a - 1, st)
                q = ring_player(W, 2 * W - 2 - a, st)
                assert (p, q) == (pf[a], ps[a])
                seen.add((min(p, q), max(p, q)))
            nf = [pf[a] if a == 0 else (ps[0] if a == 1 else pf[a - 1]) for a in range(W)]
            ns = [pf[a] if a == W - 1 else ps[a + 1] for a in range(W)]
            pf, ps = nf, ns
        assert len(seen) == N * (N - 1) // 2


def _ring_player(W, pos, st):
    R = 2 * W - 1
    x = (pos - st) % R
    return 0 if x + 1 == R else x + 1


def _ring_slot(W, a, st):
    p = 2 * W - 1 if a == 0 else _ring_player(W, a - 1, st)
    return p, _ring_player(W, 2 * W - 2 - a, st)


def _pos_next(W, P):
    R = 2 * W - 1
    return P if P == R else (P + 1) % R


def _next_meeting(W, P1, P2):
    """Python twin of block.hip next_meeting (position R = fixed player)."""
    R = 2 * W - 1

    def slot_of(pos):
        return pos + 1 if pos <= W - 2 else 2 * W - 2 - pos

    if P1 == R or P2 == R:
        o = P2 if P1 == R else P1
        return -1 if _pos_next(W, o) != R - 1 else (1 if P1 == R else 0)
    n1, n2 = _pos_next(W, P1), _pos_next(W, P2)
    if slot_of(n1) != slot_of(n2):
        return -1
    return 2 * slot_of(n1) + (1 if n1 <= W - 2 else 0)


@pytest.mark.parametrize("W", [2, 4, 8, 32, 64])
def test_evd_next_step_pairs_are_static(W):
    """The EVD kernel solves step st+1's rotations inside step st: the
    coupling of every next-step pair sits in exactly one off-diagonal
    slot-pair block, at a position that does not depend on st (each non-fixed
    player advances one ring position per step)."""
    R = 2 * W - 1
    for st in range(R):
        stn = (st + 1) % R
        nxt = {}
        for a in range(W):
            p, q = _ring_slot(W, a, stn)
            nxt[frozenset((p, q))] = (a, p)
        found = 0
        for a in range(W):
            for b in range(a + 1, W):
                per_block = 0
                pa = [R if a == 0 else a - 1, 2 * W - 2 - a]
                pb = [b - 1, 2 * W - 2 - b]
                P, Q = _ring_slot(W, a, st), _ring_slot(W, b, st)
                for e in range(4):
                    x, y = P[e >> 1], Q[e & 1]
                    mt = _next_meeting(W, pa[e >> 1], pb[e & 1])
                    if frozenset((x, y)) in nxt:
                        sl, first = nxt[frozenset((x, y))]
                        assert mt == 2 * sl + (1 if first == x else 0)
                        found += 1
                        per_block += 1
                    else:
                        assert mt == -1
                assert per_block <= 1 or W < 3  # the kernel (W >= 4) keeps ONE duty per block
        assert found == W  # every next-step pair sits in exactly one block


def _tri(N, i, j):
    a, b = min(i, j), max(i, j)
    return a * N - a * (a + 1) // 2 + (b - a - 1)


def _rot(gpp, gqq, gpq, tol):
    nrm = np.sqrt(gpp) * np.sqrt(gqq)
    if not (nrm > 0 and abs(gpq) > tol * nrm):
        return 1.0, 0.0, 0.0, False
    tau = (gqq - gpp) / (2 * gpq)
    t = np.sign(tau) / (abs(tau) + np.sqrt(1 + tau * tau)) if tau != 0 else 1.0
    c = 1 / np.sqrt(1 + t * t)
    return c, t * c, t, True


@pytest.mark.parametrize("W", [2, 3, 4, 8])
def test_evd_position_space_emulation(W):
    """Emulates the EVD kernel's position-space data flow (double-buffered G
    with static addresses, pending couplings moved twice, rotations solved one
    step ahead from the records) and checks it against a plain player-space
    cyclic Jacobi with the same circle ordering: same rotations, same final
    diagonal, exactly."""
    N, R = 2 * W, 2 * W - 1
    rng = np.random.default_rng(W)
    X = rng.random((3 * N, N))
    G0 = X.T @ X
    tol = 1e-14
    # ---- reference: player space
    G = G0.copy()
    ref_rots = []
    for st in range(R):
        rots = []
        for a in range(W):
            p, q = _ring_slot(W, a, st)
            c, s, t, _ = _rot(G[p, p], G[q, q], G[p, q], tol)
            rots.append((c, s))
            J = np.eye(N)
            J[p, p], J[p, q], J[q, p], J[q, q] = c, s, -s, c  # x' = c x - s y ; y' = s x + c y
            dpp, dqq, gpq = G[p, p], G[q, q], G[p, q]
            G = J.T @ G @ J
            if t != 0.0:
                G[p, p], G[q, q] = dpp - t * gpq, dqq + t * gpq
                G[p, q] = G[q, p] = 0.0
        ref_rots.append(rots)
    # ---- emulation of the kernel
    pos0 = [R - 1 if x == 0 else (R if x == N - 1 else x - 1) for x in range(N)]
    Gb = [np.zeros(N * (N - 1) // 2), np.zeros(N * (N - 1) // 2)]
    for r in range(N):
        for c in range(r + 1, N):
            Gb[0][_tri(N, pos0[r], pos0[c])] = G0[r, c]
    rec = [dict(), dict()]
    for a in range(W):  # prologue
        fa, sa = (R if a == 0 else a - 1), 2 * W - 2 - a
        p, q = _ring_slot(W, a, 0)
        g = Gb[0][_tri(N, fa, sa)]
        c, s, t, rot = _rot(G0[p, p], G0[q, q], g, tol)
        dp, dq = (G0[p, p] - t * g, G0[q, q] + t * g) if rot else (G0[p, p], G0[q, q])
        Gb[1][_tri(N, _pos_next(W, fa), _pos_next(W, sa))] = 0.0 if rot else g
        rec[0][a] = (c, s, dp, dq)
    blocks = []
    for a in range(W):
        for b in range(a + 1, W):
            pa = [R if a == 0 else a - 1, 2 * W - 2 - a]
            pb = [b - 1, 2 * W - 2 - b]
            duty = []
            for e in range(4):
                mt = _next_meeting(W, pa[e >> 1], pb[e & 1])
                if mt >= 0:
                    x, y = pa[e >> 1], pb[e & 1]
                    duty.append((e, mt, _tri(N, _pos_next(W, _pos_next(W, x)),
                                             _pos_next(W, _pos_next(W, y)))))
            blocks.append((a, b, pa, pb, duty, [0.0, 0.0]))
    emu_rots = [[rec[0][a][:2] for a in range(W)]]
    for gs in range(R):
        b, nb = gs & 1, (gs & 1) ^ 1
        for (a, bb, pa, pb, duty, pend) in blocks:
            if gs > 0:
                for k, (_, _, addr) in enumerate(duty):
                    Gb[nb][addr] = pend[k]
            g = [Gb[b][_tri(N, pa[e >> 1], pb[e & 1])] for e in range(4)]
            ca, sa = rec[b][a][:2]
            cb, sb = rec[b][bb][:2]
            h00, h01 = ca * g[0] - sa * g[2], ca * g[1] - sa * g[3]
            h10, h11 = sa * g[0] + ca * g[2], sa * g[1] + ca * g[3]
            h = [cb * h00 - sb * h01, sb * h00 + cb * h01, cb * h10 - sb * h11, sb * h10 + cb * h11]
            solved = set()
            for k, (e, mt, _) in enumerate(duty):
                ns, xf = mt >> 1, mt & 1
                dx = rec[b][a][3] if e >> 1 else rec[b][a][2]
                dy = rec[b][bb][3] if e & 1 else rec[b][bb][2]
                df, ds = (dx, dy) if xf else (dy, dx)
                c, s, t, rot = _rot(df, ds, h[e], tol)
                rec[nb][ns] = (c, s, df - t * h[e], ds + t * h[e]) if rot else (c, s, df, ds)
                pend[k] = 0.0 if rot else h[e]
                solved.add(e)
            for e in range(4):
                if e not in solved:
                    Gb[nb][_tri(N, _pos_next(W, pa[e >> 1]), _pos_next(W, pb[e & 1]))] = h[e]
        if gs + 1 < R:
            emu_rots.append([rec[nb][a][:2] for a in range(W)])
    np.testing.assert_allclose(np.array(emu_rots), np.array(ref_rots), rtol=1e-12, atol=1e-14)
    # final diagonal: records of the last step vs the reference G
    lb = (R - 1) & 1
    for a in range(W):
        p, q = _ring_slot(W, a, R - 1)
        np.testing.assert_allclose([rec[lb][a][2], rec[lb][a][3]], [G[p, p], G[q, q]], rtol=1e-12)


# ---- bipartite inner ordering (cross steps): X players fixed at positions
# 0..W-1, the Y player at Y-position p (position W+p) moves to p-1 (mod W)
# every step; slot a pairs positions (a, W+a).  Python twins of block.hip
# BipOrder, and the same position-space emulation as above.
def _bip_players(W, a, st):
    return a, W + (a + st) % W


def _bip_pos_next(W, P):
    return P if P < W else W + (P - W - 1) % W


def _bip_next_meeting(W, P1, P2):
    n1, n2 = _bip_pos_next(W, P1), _bip_pos_next(W, P2)
    if (n1 < W) == (n2 < W):
        return -1
    s1, s2 = n1 % W, n2 % W
    if s1 != s2:
        return -1
    return 2 * s1 + (1 if n1 < W else 0)


@pytest.mark.parametrize("W", [3, 4, 8, 32, 64])
def test_bip_next_step_pairs_are_static(W):
    """Bipartite ordering: every cross pair once per W steps, and the coupling
    of each next-step pair sits in exactly one slot-pair block (at most one per
    block), at a static position."""
    seen = set()
    for st in range(W):
        nxt = {}
        for a in range(W):
            p, q = _bip_players(W, a, st)
            seen.add((p, q))
            p1, q1 = _bip_players(W, a, (st + 1) % W)
            nxt[frozenset((p1, q1))] = (a, p1)
        found = 0
        for a in range(W):
            for b in range(a + 1, W):
                per_block = 0
                pa, pb = [a, W + a], [b, W + b]
                P, Q = _bip_players(W, a, st), _bip_players(W, b, st)
                for e in range(4):
                    x, y = P[e >> 1], Q[e & 1]
                    mt = _bip_next_meeting(W, pa[e >> 1], pb[e & 1])
                    if frozenset((x, y)) in nxt:
                        sl, first = nxt[frozenset((x, y))]
                        assert mt == 2 * sl + (1 if first == x else 0)
                        found += 1
                        per_block += 1
                    else:
                        assert mt == -1
                assert per_block <= 1
        assert found == W
    assert len(seen) == W * W


@pytest.mark.parametrize("W", [3, 4, 8])
def test_bip_position_space_emulation(W):
    """The kernel's position-space data flow with the bipartite ordering
    against a plain player-space Jacobi over the cross pairs: same rotations,
    same final diagonal."""
    N, R = 2 * W, W
    rng = np.random.default_rng(W + 100)
    X = rng.random((3 * N, N))
    G0 = X.T @ X
    tol = 1e-14
    G = G0.copy()
    ref_rots = []
    for st in range(R):
        rots = []
        for a in range(W):
            p, q = _bip_players(W, a, st)
            c, s, t, _ = _rot(G[p, p], G[q, q], G[p, q], tol)
            rots.append((c, s))
            J = np.eye(N)
            J[p, p], J[p, q], J[q, p], J[q, q] = c, s, -s, c
            dpp, dqq, gpq = G[p, p], G[q, q], G[p, q]
            G = J.T @ G @ J
            if t != 0.0:
                G[p, p], G[q, q] = dpp - t * gpq, dqq + t * gpq
                G[p, q] = G[q, p] = 0.0
        ref_rots.append(rots)
    nxt = lambda P: _bip_pos_next(W, P)  # noqa: E731
    Gb = [np.zeros(N * (N - 1) // 2), np.zeros(N * (N - 1) // 2)]
    for r in range(N):
        for c in range(r + 1, N):
            Gb[0][_tri(N, r, c)] = G0[r, c]  # pos0 is the identity
    rec = [dict(), dict()]
    for a in range(W):
        fa, sa = a, W + a
        g = Gb[0][_tri(N, fa, sa)]
        c, s, t, rot = _rot(G0[fa, fa], G0[sa, sa], g, tol)
        dp, dq = (G0[fa, fa] - t * g, G0[sa, sa] + t * g) if rot else (G0[fa, fa], G0[sa, sa])
        Gb[1][_tri(N, nxt(fa), nxt(sa))] = 0.0 if rot else g
        rec[0][a] = (c, s, dp, dq)
    blocks = []
    for a in range(W):
        for b in range(a + 1, W):
            pa, pb = [a, W + a], [b, W + b]
            duty = []
            for e in range(4):
                mt = _bip_next_meeting(W, pa[e >> 1], pb[e & 1])
                if mt >= 0:
                    x, y = pa[e >> 1], pb[e & 1]
                    duty.append((e, mt, _tri(N, nxt(nxt(x)), nxt(nxt(y)))))
            blocks.append((a, b, pa, pb, duty, [0.0]))
    emu_rots = [[rec[0][a][:2] for a in range(W)]]
    for gs in range(R):
        b, nb = gs & 1, (gs & 1) ^ 1
        for (a, bb, pa, pb, duty, pend) in blocks:
            if gs > 0:
                for k, (_, _, addr) in enumerate(duty):
                    Gb[nb][addr] = pend[k]
            g = [Gb[b][_tri(N, pa[e >> 1], pb[e & 1])] for e in range(4)]
            ca, sa = rec[b][a][:2]
            cb, sb = rec[b][bb][:2]
            h00, h01 = ca * g[0] - sa * g[2], ca * g[1] - sa * g[3]
            h10, h11 = sa * g[0] + ca * g[2], sa * g[1] + ca * g[3]
            h = [cb * h00 - sb * h01, sb * h00 + cb * h01, cb * h10 - sb * h11, sb * h10 + cb * h11]
            solved = set()
            for k, (e, mt, _) in enumerate(duty):
                ns, xf = mt >> 1, mt & 1
                dx = rec[b][a][3] if e >> 1 else rec[b][a][2]
                dy = rec[b][bb][3] if e & 1 else rec[b][bb][2]
                df, ds = (dx, dy) if xf else (dy, dx)
                c, s, t, rot = _rot(df, ds, h[e], tol)
                rec[nb][ns] = (c, s, df - t * h[e], ds + t * h[e]) if rot else (c, s, df, ds)
                pend[k] = 0.0 if rot else h[e]
                solved.add(e)
            for e in range(4):
                if e not in solved:
                    Gb[nb][_tri(N, nxt(pa[e >> 1]), nxt(pb[e & 1]))] = h[e]
        if gs + 1 < R:
            emu_rots.append([rec[nb][a][:2] for a in range(W)])
    np.testing.assert_allclose(np.array(emu_rots), np.array(ref_rots), rtol=1e-12, atol=1e-14)
    lb = (R - 1) & 1
    for a in range(W):
        p, q = _bip_players(W, a, R - 1)
        np.testing.assert_allclose([rec[lb][a][2], rec[lb][a][3]], [G[p, p], G[q, q]], rtol=1e-12)


def _deal_tool():
    import importlib.util
    import os
    p = os.path.join(os.path.dirname(__file__), "..", "tools", "evd_deal_opt.py")
    spec = importlib.util.spec_from_file_location("evd_deal_opt", p)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _header_table(name):
    import os
    import re
    p = os.path.join(os.path.dirname(__file__), "..", "svd-jacobi-mpi-cuda_amd", "csrc", "hip",
                     "evd_deal_tables.hpp")
    txt = open(p).read()
    body = re.search(name + r"\[\d+\] = \{(.*?)\};", txt, re.S).group(1)
    return [int(x, 16) for x in re.findall(r"0x[0-9a-f]{4}", body)]


@pytest.mark.parametrize("W", [32, 64])
def test_evd_deal_table_valid_and_cheaper(W):
    """The generated fp32 bipartite EVD dealing (csrc/hip/evd_deal_tables.hpp,
    tools/evd_deal_opt.py): duty blocks of next-step slots 0..W-1 first, every
    slot-pair block exactly once, and fewer modelled LDS cycles per step than
    the round-2 dealing (PMC: bank-conflict share 40 -> 20 %, profiles/r2_deal)."""
    T = _deal_tool()
    vals = _header_table(f"kEvdDealF32_W{W}_bip")
    NT = T.NT
    duty, rest = T.round2_deal(W, T.BIP)
    blks = [None if v == 0xffff else (v >> 8, v & 255) for v in vals]
    assert blks[:W] == duty
    dealt = [b for b in blks if b is not None]
    assert sorted(dealt) == sorted(duty + rest) and len(set(dealt)) == W * (W - 1) // 2
    maxoff = len(vals) // NT
    slots = [[blks[j * NT + t] for t in range(NT)] for j in range(maxoff)]
    c_opt, _ = T.deal_cost(W, T.BIP, slots)
    c_r2, _ = T.deal_cost(W, T.BIP, T.slots_from(duty, rest, W))
    assert c_opt < 0.8 * c_r2, (c_opt, c_r2)


@pytest.mark.parametrize("nb", [4, 8, 16, 64])
def test_quad_round_robin_covers_once(nb):
    pr = S.quad_round_robin(nb)
    modes = S.quad_round_robin_modes(nb)
    assert pr.shape == (nb - 1, nb // 2, 2) and len(modes) == nb - 1
    S.check_quad_steps(pr, modes)
    seen = set()
    for st in pr:
        assert sorted(st.ravel().tolist()) == list(range(nb))
        seen |= {(min(a, b), max(a, b)) for a, b in st.tolist()}
    assert len(seen) == nb * (nb - 1) // 2
    assert pr[0].tolist() == [[2 * i, 2 * i + 1] for i in range(nb // 2)]


@pytest.mark.parametrize("h", [2, 4, 8])
def test_quad_bipartite_covers_once(h):
    xs, ys = list(range(h)), list(range(100, 100 + h))
    pr = S.quad_bipartite(xs, ys)
    S.check_quad_steps(pr, S.quad_bipartite_modes(h))
    assert {(a, b) for st in pr for a, b in st.tolist()} == {(x, y) for x in xs for y in ys}


@pytest.mark.parametrize("nb", [4, 8, 12, 64, 256])
def test_quad_round_robin_native_equals_python(nb):
    assert np.array_equal(S.quad_round_robin(nb), S.quad_round_robin_py(nb))


@pytest.mark.parametrize("h", [2, 4, 8, 64])
def test_quad_bipartite_native_equals_python(h):
    xs = list(range(3, 3 + h))
    ys = list(range(100, 100 + 2 * h, 2))
    assert np.array_equal(S.quad_bipartite(xs, ys), S.quad_bipartite_py(xs, ys))


def test_check_quad_steps_rejects_wrong_orientation():
    pr = S.quad_round_robin(8)
    bad = pr.copy()
    bad[2, 0] = bad[2, 0, ::-1]
    with pytest.raises(ValueError):
        S.check_quad_steps(bad, S.quad_round_robin_modes(8))
    with pytest.raises(ValueError):
        S.check_quad_steps(pr, [1, 5, 4] + [4, 5] * 2)
