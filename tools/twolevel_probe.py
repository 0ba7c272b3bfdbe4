"""Two-level block Jacobi probe (development aid): time, sweeps and accuracy of
models/twolevel.py on a random dense U(0,1) matrix, one device."""
import argparse
import json
import math
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import svdj  # noqa: E402
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from twolevel_exp import TwoLevel  # noqa: E402
from svdj.ops import kernels as K  # noqa: E402
from svdj.utils.layout import pack_columns, pad_rows  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--sizes", default="4096")
p.add_argument("--W", type=int, default=64)
p.add_argument("--Wb", type=int, default=512)
p.add_argument("--reps", type=int, default=1)
p.add_argument("--verify", action="store_true")
p.add_argument("--device", default="cuda:0")
p.add_argument("--inner-order", default="bipartite")
p.add_argument("--max-sweeps", type=int, default=60)
a = p.parse_args()
dev = torch.device(a.device)
dt = torch.float32
for n in [int(x) for x in a.sizes.split(",")]:
    m = n
    A = svdj.utils.inputs.random_dense(m, n, dtype=dt, device=dev, seed=1)
    m_pad, n_v = pad_rows(m), pad_rows(n)
    ncols = -(-n // (2 * a.Wb)) * 2 * a.Wb
    n_v = pad_rows(ncols)
    tl = TwoLevel(ncols, m_pad, n_v, a.W, a.Wb, dt, dev)
    tol = math.sqrt(m) * torch.finfo(dt).eps
    for rep in range(a.reps):
        At = pack_columns(A, dt, dev, ncols, m_pad)
        Vt = torch.zeros(ncols, n_v, dtype=dt, device=dev)
        K.set_identity(Vt, ncols)
        metric = K.new_metric(dev)
        K.set_norm_floor(metric, dt, m_pad)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        prog = (lambda s, mx, nr, nf: print(f"  sweep {s}: off {mx:.2e} rot {nr} fail {nf} "
                                            f"{time.perf_counter() - t0:.3f}s", file=sys.stderr,
                                            flush=True))
        sweeps, hist = tl.solve(At, Vt, tol, a.max_sweeps, metric, inner_order=a.inner_order, progress=prog)
        S = K.finalize(At, m_pad)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t = time.perf_counter() - t0
        out = {"n": n, "W": a.W, "Wb": a.Wb, "sweeps": sweeps, "sec": round(t, 4),
               "gflops_alg": round(svdj.utils.metrics.gflops(m, n, sweeps, t), 1), "rep": rep}
        if a.verify and rep == a.reps - 1:
            U = At[:n, :m].t()
            V = Vt[:n, :n].t()
            ref = torch.linalg.svdvals(A.double()) if n <= 8192 else None
            out.update(svdj.utils.metrics.verify(A, U, S[:n], V, ref))
        print(json.dumps(out), flush=True)
