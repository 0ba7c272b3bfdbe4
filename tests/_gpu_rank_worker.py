"""Worker of the one-GPU multi-rank tests (tests/test_gpu_multirank.py).

Launched by torchrun with every rank on cuda:0 (SVDJ_SHARED_GPU=1); the
backend comes from SVDJ_COMM_BACKEND (nccl = RCCL through per-rank host ids,
or gloo, host-synchronised).  Solves one fixed matrix with the pipelined
distributed solver and writes rank 0's gathered (U, S, V) plus run info to
the output file, so runs over different backends can be compared bitwise.

argv: n W chains mode(otf|root|qr|qrbf16) out.pt   (qrbf16: tall bf16 input, the bf16
problem mode -- BASELINE config 4's kind of job)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdj  # noqa: E402
from svdj.parallel import Communicator, DistributedBlockJacobi  # noqa: E402


def main():
    n, W, chains, mode, out = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4],
                               sys.argv[5])
    comm = Communicator(timeout_s=120)
    dev = comm.device
    timing = os.environ.get("SVDJ_TEST_TIMING", "1") == "1"
    cfg = svdj.SolverConfig(block=W, dtype=torch.float32, chains=chains, comm_timing=timing,
                            precondition="none", progress=True,
                            exchange=os.environ.get("SVDJ_TEST_EXCHANGE", "auto"),
                            quad=os.environ.get("SVDJ_TEST_QUAD", "auto"))
    solver = DistributedBlockJacobi(cfg, comm)
    g = torch.Generator(device=dev).manual_seed(5)
    m = 4 * n if mode in ("qr", "qrbf16") else n
    if mode in ("qr", "qrbf16"):  # tall: row-distributed CholeskyQR2 + Jacobi on R
        cfg.precondition = "qr"
    A = torch.rand(m, n, generator=g, device=dev, dtype=torch.float32)
    pdtype = torch.float32
    if mode == "qrbf16":  # bf16 data, fp32 master copies, bf16 matrix cores
        A = A.to(torch.bfloat16)
        pdtype = cfg.dtype = torch.bfloat16
    if mode == "root":
        res = solver.solve(A if comm.rank == 0 else None, gather=True)
    else:
        res = solver.solve(None, m=m, n=n, dtype=pdtype,
                           generator=lambda c0, c1: A[:, c0:c1], gather=True)
    if comm.rank == 0:
        torch.save({"U": res.U.cpu(), "S": res.S.cpu(), "V": res.V.cpu(), "A": A.cpu(),
                    "sweeps": res.sweeps, "converged": res.converged, "history": res.history,
                    "backend": comm.backend, "world": comm.world,
                    "exchange": res.info.get("exchange"), "mma": res.info.get("mma"),
                    "inner_order": res.info.get("inner_order"), "quad": res.info.get("quad"),
                    "comm": json.dumps(res.info.get("comm"))}, out)
    comm.destroy()


if __name__ == "__main__":
    main()
