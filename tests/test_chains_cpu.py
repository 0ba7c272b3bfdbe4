"""Two-chain (pipelined) solver: CPU equivalence with the single-chain path.

Plan coverage of the pipelined sweep is checked in test_pipeline_cpu.py."""
import torch

import svdj
from svdj.parallel import Communicator, DistributedBlockJacobi


def test_chained_solver_cpu_matches_single_chain():
    A = svdj.utils.inputs.random_dense(160, 128, dtype=torch.float64, seed=8)
    comm = Communicator(backend="gloo", device=torch.device("cpu"), init=False)
    r1 = DistributedBlockJacobi(svdj.SolverConfig(block=32, chains=1), comm).solve(A)
    r2 = DistributedBlockJacobi(svdj.SolverConfig(block=32, chains=2), comm).solve(A)
    ref = torch.linalg.svdvals(A)
    for r in (r1, r2):
        rep = svdj.utils.metrics.verify(A, r.U, r.S, r.V, ref)
        assert r.converged and rep["residual_rel"] < 1e-12 and rep["orth_u_fro"] < 1e-11
