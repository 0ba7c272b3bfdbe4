#!/usr/bin/env python3
"""Headline benchmark: dense one-sided Jacobi SVD to convergence on N MI355X.

Metric (BASELINE.json): GFLOP/s + time-to-converge (sweeps to ||off|| < tol),
N x N dense SVD at 1/2/4/8 MI355X.  One "step" = one complete SVD solve
(A -> U, sigma, V with AllVec/AllVec, every sweep until a sweep applies no
rotation) of a synthetic random dense U(0,1) matrix, fp32, distributed as a
column-block tournament over the N GPUs (one process per GPU, RCCL).

GFLOP/s counts the reference's algorithmic work per sweep,
n(n-1)/2 * (12 m + 6 n), times the sweeps actually
executed, divided by the measured wall time of the solve; the value is the
whole-job aggregate.  Strong scaling: the matrix size is fixed as N grows.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--n 16384]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = ("GFLOP/s + time-to-converge (sweeps to ||off||<tol), N×N dense SVD at "
                   "1/2/4/8 MI355X")


def verify_distributed(res, gen, m, n, comm, dtype):
    """Accuracy of the (distributed) result, after the timed region.

    Every rank regenerates A (same seeded generator) and checks its own
    columns: ||A V_loc - U_loc S_loc||_F^2 and ||[U_loc|V_loc]^T[..] - I||_F^2,
    summed over ranks (fp32 GEMMs, accurate to ~1e-6 relative).  Padding
    columns (global index >= n) are excluded."""
    geo = res.info["geometry"]
    B = geo["B"]
    held = res.info["held"]
    A = torch.cat([gen(c0, min(c0 + B, n)) for c0 in range(0, n, B)], dim=1).to(dtype)
    At, Vt, S = res.U, res.V, res.S
    cols = []
    for s, sb in enumerate(held):
        for j in range(B):
            if sb * B + j < n:
                cols.append(s * B + j)
    idx = torch.tensor(cols, device=At.device, dtype=torch.long)
    U = At[idx, :m].t()
    V = Vt[idx, :n].t()
    sig = S[idx]
    R = A @ V - U * sig
    eye = torch.eye(len(cols), device=At.device, dtype=dtype)
    parts = torch.stack([R.double().pow(2).sum(), A.double().pow(2).sum() / comm.world,
                         (V.t() @ V - eye).double().pow(2).sum(),
                         (U.t() @ U - eye).double().pow(2).sum()])
    if comm.distributed:
        import torch.distributed as dist
        dist.all_reduce(parts)
    parts = parts.cpu()
    return {"residual_rel": float((parts[0] / parts[1]).sqrt()),
            "orth_v_blockdiag_fro": float(parts[2].sqrt()),
            "orth_u_blockdiag_fro": float(parts[3].sqrt())}


def main():
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--n", "--size", dest="n", type=int, default=16384)
    p.add_argument("--m", type=int, default=None)
    p.add_argument("--dtype", default="fp32", choices=["fp32", "fp64", "bf16"])
    p.add_argument("--precondition", default="auto", choices=["none", "qr", "auto"],
                   help="QR-precondition tall inputs (m >= 2n); flops then count QR + GEMM")
    p.add_argument("--block", type=int, default=None)
    p.add_argument("--max-sweeps", type=int, default=60)
    p.add_argument("--inner", type=int, default=1)
    p.add_argument("--chains", type=int, default=2)
    p.add_argument("--no-stagger", action="store_true",
                   help="issue the two step chains independently (lockstep) instead of offset")
    p.add_argument("--mma", default="auto", choices=["auto", "native", "bf16x6", "bf16x3"],
                   help="block apply matrix cores (auto = native f32/f64 MFMA; bf16x6/bf16x3 "
                        "split modes are faster but not fp32-accurate on every input)")
    p.add_argument("--json-out", default=None)
    p.add_argument("--no-verify", action="store_true",
                   help="skip the post-timing accuracy check")
    a = p.parse_args()

    import svdj
    from svdj.parallel import Communicator, DistributedBlockJacobi

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 with "
                         "torch.distributed.run --nproc-per-node N")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    comm = Communicator()
    dtype = {"fp32": torch.float32, "fp64": torch.float64, "bf16": torch.bfloat16}[a.dtype]
    work = torch.float64 if dtype == torch.float64 else torch.float32
    n = a.n
    m = a.m or n
    cfg = svdj.SolverConfig(dtype=dtype, block=a.block, max_sweeps=a.max_sweeps,
                            max_inner_sweeps=a.inner, chains=a.chains, mma=a.mma,
                            stagger=not a.no_stagger,
                            precondition=a.precondition)
    solver = DistributedBlockJacobi(cfg, comm)
    dev = comm.device

    GB = 256  # generator block: the matrix is fixed regardless of how callers chunk it

    def gen(c0, c1):  # synthetic random dense U(0,1), columns c0..c1-1 of ONE fixed matrix
        parts = []
        for b0 in range(c0 // GB * GB, c1, GB):
            g = torch.Generator(device=dev).manual_seed(1234 + b0)
            blk = torch.rand(m, GB, generator=g, dtype=work, device=dev)
            parts.append(blk[:, max(c0 - b0, 0):min(c1 - b0, GB)])
        return torch.cat(parts, dim=1).to(dtype)

    def one():
        return solver.solve(None, m=m, n=n, dtype=dtype, generator=gen, gather=False)

    for _ in range(a.warmup):
        one()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    results = [one() for _ in range(a.steps)]
    comm.barrier()
    torch.cuda.synchronize()
    elapsed = comm.max_over_ranks(time.perf_counter() - t0)

    sweeps = [r.sweeps for r in results]
    conv = all(r.converged for r in results)
    flops = sum(r.info["flops"] for r in results)
    gflops = flops / elapsed / 1e9
    ms = elapsed / a.steps * 1e3
    geo = results[-1].info["geometry"]
    acc = None if a.no_verify else verify_distributed(results[-1], gen, m, n, comm, work)
    if comm.rank == 0:
        line = {
            "metric": BASELINE_METRIC,
            "value": round(gflops, 2),
            "unit": "GFLOP/s",
            "n_gpus": a.gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": "synthetic random dense U(0,1), seeded per column block",
            "config": {
                "model": f"{m}x{n} {a.dtype} block one-sided Jacobi SVD (AllVec), to convergence",
                "global_batch": 1,
                "seq_len": n,
                "parallelism": f"colblock{a.gpus} (2 super-blocks/GPU, RCCL tournament)",
                "block_W": geo["W"],
                "super_block_B": geo["B"],
                "mma": results[-1].info.get("mma", a.mma),
                "precondition": results[-1].info.get("precondition", "none"),
                "chains": a.chains,
                "staggered": not a.no_stagger,
            },
            "sweeps": sweeps,
            "converged": conv,
            "time_to_converge_s": round(ms / 1e3, 4),
            "off_history_last": [float("%.3e" % h) for h in results[-1].history[-3:]],
            "comm_seconds_rank0": round(results[-1].info["comm_seconds"], 4),
            "accuracy": acc,
        }
        print(json.dumps(line), flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                json.dump(line, f)
    comm.destroy()


if __name__ == "__main__":
    main()
