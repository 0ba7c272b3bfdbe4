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
