"""Chained (two-stream) sweep plans: coverage and CPU equivalence."""
import pytest
import torch

import svdj
from svdj.parallel import Communicator, DistributedBlockJacobi
from svdj.parallel import schedule as S


@pytest.mark.parametrize("P,k", [(1, 2), (1, 4), (2, 2), (3, 4), (4, 2)])
def test_chained_plan_covers_every_pair_once(P, k):
    t = S.tournament(P)
    plans = S.chained_sweep_plan(P, k)
    phys = [[int(t.held[0, g, 0]), int(t.held[0, g, 1])] for g in range(P)]
    seen = set()
    for r in range(t.rounds):
        if r > 0:
            old = [list(x) for x in phys]
            for g in range(P):
                src = int(t.recv_from[r, g])
                phys[g][int(t.xslot[r, g])] = old[src][int(t.xslot[r, src])]
        for g in range(P):
            for phase in plans[r]:
                used = [set(), set()]
                for c, chain in enumerate(phase):
                    for st in chain.pairs:
                        blocks = st.reshape(-1).tolist()
                        assert len(blocks) == len(set(blocks))
                        used[c].update(blocks)
                        for a, b in st:
                            ga = phys[g][a // k] * k + a % k
                            gb = phys[g][b // k] * k + b % k
                            key = (min(ga, gb), max(ga, gb))
                            assert key not in seen
                            seen.add(key)
                assert not (used[0] & used[1]), "chains of a phase must be independent"
    nb = 2 * P * k
    assert len(seen) == nb * (nb - 1) // 2


def test_chained_plan_odd_k_falls_back():
    assert S.chained_sweep_plan(2, 3) is None


def test_chained_solver_cpu_matches_single_chain():
    A = svdj.utils.inputs.random_dense(160, 128, dtype=torch.float64, seed=8)
    comm = Communicator(backend="gloo", device=torch.device("cpu"), init=False)
    r1 = DistributedBlockJacobi(svdj.SolverConfig(block=32, chains=1), comm).solve(A)
    r2 = DistributedBlockJacobi(svdj.SolverConfig(block=32, chains=2), comm).solve(A)
    ref = torch.linalg.svdvals(A)
    for r in (r1, r2):
        rep = svdj.utils.metrics.verify(A, r.U, r.S, r.V, ref)
        assert r.converged and rep["residual_rel"] < 1e-12 and rep["orth_u_fro"] < 1e-11
