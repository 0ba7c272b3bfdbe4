"""Kernel-level micro benchmark of one block-Jacobi sweep (development aid).

Times one sweep of block steps (gram -> evd -> apply) on a random n x n
matrix for several inner-sweep counts; inner=0 isolates the EVD's fixed cost
(assembly / metric / launch) from its per-Jacobi-sweep cost.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdj  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=4096)
p.add_argument("--block", type=int, default=32)
p.add_argument("--dtype", default="fp32")
p.add_argument("--inner", default="0,1,2")
p.add_argument("--reps", type=int, default=3)
p.add_argument("--mma", default="native")
a = p.parse_args()
K = svdj.ops.kernels
dt = torch.float32 if a.dtype == "fp32" else torch.float64
dev = torch.device("cuda:0")
n, W = a.n, a.block
nb = n // W
pairs = torch.from_numpy(svdj.parallel.schedule.round_robin(nb)).to(dev)
modes = [0] * (nb - 1)
A0 = torch.rand(n, n, dtype=dt, device=dev)
for inner in [int(x) for x in a.inner.split(",")]:
    times = []
    for _ in range(a.reps):
        At = A0.clone()
        Vt = torch.zeros(n, n, dtype=dt, device=dev)
        K.set_identity(Vt, n)
        D = K.col_norms2(At, n)
        metric = K.new_metric(dev)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        K.block_steps(At, Vt, D, n, pairs, W, modes, 1e-30 if inner > 0 else 1e30, inner, metric,
                      mma=a.mma)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    per_step = min(times) / (nb - 1) * 1e3
    print(json.dumps({"n": n, "W": W, "dtype": a.dtype, "inner": inner, "mma": a.mma, "sweep_ms": round(min(times), 3),
                      "us_per_step": round(per_step, 2)}), flush=True)
