"""Single-stream block sweep timing for EVD A/B runs (development aid).

Runs one block-Jacobi sweep (round robin over n/W blocks, first step full)
on ONE stream, so no two kernels overlap: under ``rocprofv3 --kernel-trace
--stats`` the per-kernel averages are isolated latencies.  Prints one JSON
line with the wall time of the timed sweeps.  ``SVDJ_HIP_LIB`` selects a
variant library (tools build them with _build.build_hip_variant).
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
p.add_argument("--m", type=int, default=None)
p.add_argument("--block", type=int, default=32)
p.add_argument("--dtype", default="fp32")
p.add_argument("--sweeps", type=int, default=2)
p.add_argument("--order", default="bipartite", choices=["cyclic", "bipartite"])
a = p.parse_args()
K = svdj.ops.kernels
dt = torch.float32 if a.dtype == "fp32" else torch.float64
dev = torch.device("cuda:0")
n, W = a.n, a.block
m = a.m or n
nb = n // W
pairs = torch.from_numpy(svdj.parallel.schedule.round_robin(nb)).to(dev)
modes = [1] + [0] * (nb - 2)
g = torch.Generator(device=dev).manual_seed(1)
At = torch.rand(n, m, dtype=dt, device=dev, generator=g)
Vt = torch.zeros(n, n, dtype=dt, device=dev)
K.set_identity(Vt, n)
D = K.col_norms2(At, m)
tol = svdj.utils.metrics.default_tol(dt, m)
metric = K.new_metric(dev)
K.block_steps(At, Vt, D, m, pairs, W, modes, tol, 1, metric, inner_order=a.order)  # warm
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.sweeps):
    K.block_steps(At, Vt, D, m, pairs, W, modes, tol, 1, metric, inner_order=a.order)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.sweeps
print(json.dumps({"n": n, "m": m, "W": W, "dtype": a.dtype, "ms_per_sweep": round(ms, 3),
                  "steps": nb - 1, "pairs_per_step": nb // 2,
                  "us_per_step": round(ms * 1e3 / (nb - 1), 2),
                  "lib": os.environ.get("SVDJ_HIP_LIB", "default")}))
