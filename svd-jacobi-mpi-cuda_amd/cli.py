"""Command-line driver -- the reference's ``main`` (reference main.cu:1426-1676).

    python tools/svd_jacobi.py N [--m M] [options]                     # 1 GPU / CPU
    torchrun --nproc-per-node 8 tools/svd_jacobi.py N [options]        # 8 GPUs (RCCL)

Reference behaviour kept:
  * argv[1] = n (square by default, main.cu:1452-1453); ``--m`` allows m >= n;
  * default input = the reference's upper-triangular U(0,1) from
    std::default_random_engine(1000000), bit-exact (main.cu:1558-1567), generated
    on the root rank (root-owned input, like the reference);
  * prints "Dimensions, height: .., width: ..", "SVD MPI+OMP time with U,V
    calculation: <s>" and "||A-USVt||_F: <x>" and writes the
    reporte-dimension-<n>-time-<ts>.txt report (main.cu:1539-1669);
  * ``--test1`` runs the reference's embedded "Test 1" (a 1000 x 1000 single-GPU
    solve + residual, main.cu:1461-1534) -- seeded and on the root rank only
    (the reference ran it on every rank with a non-deterministic seed).
Fixed / added: a real stopping test, ``--verify`` (orthogonality of U and V and
sigma against an independent oracle -- the reference's residual alone is
vacuous), a JSON record, ``--dtype`` / ``--method`` / tolerance / checkpoint
flags (config.add_cli_args).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch


def _input(kind: str, m: int, n: int, seed: int, dtype):
    from .utils import inputs

    if kind == "triu":
        return inputs.reference_triu(n, m, seed)
    if kind == "dense":
        return inputs.reference_dense(n, m, seed)
    if kind == "uniform":
        return inputs.random_dense(m, n, dtype=torch.float64, seed=seed)
    if kind == "normal":
        return inputs.random_dense(m, n, dtype=torch.float64, seed=seed, dist="normal")
    raise ValueError(kind)


def _residual(A, res) -> float:
    R = A.double() - (res.U.double() * res.S.double()) @ res.V.double().t()
    return float(R.norm())


def main(argv=None) -> int:
    from . import api, config
    from .parallel import Communicator, DistributedBlockJacobi
    from .utils import metrics, report

    p = argparse.ArgumentParser(prog="svd_jacobi", description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("n", type=int, help="matrix width (and height unless --m)")
    p.add_argument("--m", type=int, default=None)
    p.add_argument("--input", default="triu", choices=["triu", "dense", "uniform", "normal"])
    p.add_argument("--seed", type=int, default=1000000)
    p.add_argument("--cpu", action="store_true", help="run on the CPU (oracle / torch ref)")
    p.add_argument("--verify", action="store_true")
    p.add_argument("--test1", action="store_true")
    p.add_argument("--report-dir", default=".")
    p.add_argument("--no-report", action="store_true")
    p.add_argument("--json", default=None)
    config.add_cli_args(p)
    a = p.parse_args(argv)
    cfg = config.config_from_args(a)
    if cfg.dtype is None:
        cfg.dtype = torch.float64  # the reference is fp64

    world = int(os.environ.get("WORLD_SIZE", "1"))
    use_gpu = torch.cuda.is_available() and not a.cpu
    comm = Communicator(device=None if use_gpu else torch.device("cpu"),
                        backend=None if use_gpu else "gloo") if world > 1 else None
    rank = comm.rank if comm else 0
    dev = (comm.device if comm else (torch.device("cuda:0") if use_gpu else torch.device("cpu")))
    m, n = a.m or a.n, a.n
    workers = world if use_gpu else (os.cpu_count() or 1)

    if rank == 0:
        print(f"Number of workers: {workers}")
        print(f"Dimensions, height: {m}, width: {n}")
        if a.test1:  # reference "Test 1": 1000 x 1000 single-device solve
            A1 = _input("uniform", 1000, 1000, 1, torch.float64).to(dev)
            r1 = api.svd(A1, config=cfg, device=dev)
            print(f"Test 1: sweeps {r1.sweeps}, time {r1.seconds:.4f} s, "
                  f"||A-USVt||_F: {_residual(A1, r1):.3e}")

    A = _input(a.input, m, n, a.seed, torch.float64) if rank == 0 else None
    t0 = time.perf_counter()
    if comm is not None:
        solver = DistributedBlockJacobi(cfg, comm)
        res = solver.solve(A.to(dev) if A is not None else None)
    else:
        res = api.svd(A.to(dev), config=cfg, device=dev)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    if rank == 0:
        print(f"SVD MPI+OMP time with U,V calculation: {secs}")
        resid = _residual(A.to(res.U.device), res)
        print(f"||A-USVt||_F: {resid}")
        print(f"sweeps: {res.sweeps} converged: {res.converged} method: {res.method}")
        acc = None
        if a.verify:
            ref = torch.linalg.svdvals(A.double())
            acc = metrics.verify(A.to(res.U.device), res.U, res.S, res.V, ref)
            print("verify:", {k: f"{v:.3e}" for k, v in acc.items()})
        if not a.no_report:
            path = report.write_reference_report(a.report_dir, m, n, secs, resid, workers)
            print(f"report: {path}")
        if a.json:
            report.write_json(a.json, report.run_record(res, m, n, world if use_gpu else 0, acc,
                                                        {"wall_seconds": secs}))
    if comm is not None:
        comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
