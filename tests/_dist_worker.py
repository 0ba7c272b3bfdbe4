"""Worker for multi-process (gloo) distributed tests; launched by torchrun."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdj  # noqa: E402
from svdj.parallel import Communicator, DistributedBlockJacobi  # noqa: E402


def main():
    m, n, W, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    mode = sys.argv[5] if len(sys.argv) > 5 else "root"
    comm = Communicator(backend="gloo", device=torch.device("cpu"))
    cfg = svdj.SolverConfig(block=W, dtype=torch.float64, max_inner_sweeps=1,
                            precondition="qr" if mode.endswith("qr") else "none")
    solver = DistributedBlockJacobi(cfg, comm)
    A = svdj.utils.inputs.random_dense(m, n, dtype=torch.float64, seed=9)
    if mode in ("root", "rootqr"):
        res = solver.solve(A if comm.rank == 0 else None)
    else:
        res = solver.solve(None, m=m, n=n, dtype=torch.float64,
                           generator=lambda c0, c1: A[:, c0:c1])
    if comm.rank == 0:
        rep = svdj.utils.metrics.verify(A, res.U, res.S, res.V, torch.linalg.svdvals(A))
        rep.update(sweeps=res.sweeps, converged=res.converged, world=comm.world)
        with open(out, "w") as f:
            json.dump(rep, f)
    comm.destroy()


if __name__ == "__main__":
    main()
