"""Threshold strategies for the block sweep (development aid, CPU, fp32).

Runs the block one-sided Jacobi of the flagship path (W-column blocks, round-robin
steps, first step of a sweep full, the rest cross-only) with the torch reference
kernels (ops.reference.block_step) and prints, per sweep, the distribution of
the per-pair coupling max|c_ij|/sqrt(d_i d_j) and how many pairs were applied.
Starting points: eigpre / eigpre64 (V0 = eigenvectors of the Gram), blkpreK (eigenvectors
of K diagonal super-block Grams), rt / rt32 (xGEJSV-style Jacobi on R^T of A = QR without V,
V recovered by a triangular solve).
A strategy sets the skip threshold of sweep k from the history; the cost model
is the number of applied pairs (each costs one read+write of 2W columns of A
and V) plus one Gram read per pair.
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdj  # noqa: E402

R = svdj.ops.reference
p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=2048)
p.add_argument("--W", type=int, default=64)
p.add_argument("--strategy", default="base")
p.add_argument("--c", type=float, default=1e-2)
p.add_argument("--k0", type=int, default=4)
p.add_argument("--max-sweeps", type=int, default=40)
a = p.parse_args()
torch.set_num_threads(8)
n, W = a.n, a.W
nb = n // W
A = svdj.utils.inputs.random_dense(n, n, dtype=torch.float64, seed=1).float()
At = A.t().contiguous()
Vt = torch.eye(n, dtype=torch.float32)
if a.strategy.startswith("blkpre"):
    # eigenvectors of the fp32 Gram of each of nblk column super-blocks
    nblk = int(a.strategy[6:])
    Q = torch.zeros(n, n)
    bs = n // nblk
    for i in range(nblk):
        sl = slice(i * bs, (i + 1) * bs)
        _, Qi = torch.linalg.eigh(A[:, sl].t() @ A[:, sl])
        Q[sl, sl] = Qi.flip(1)
    At = (A @ Q).t().contiguous()
    Vt = Q.t().contiguous()
    a.strategy = "base"
Qqr = None
if a.strategy.startswith("rt"):
    # xGEJSV-style: A = QR (fp64), Jacobi on X = R^T without V; V_x by a triangular
    # solve (rt: fp64 solve, rt32: fp32 solve)
    Qqr, Rqr = torch.linalg.qr(A.double())
    At = Rqr.float().contiguous()          # rows of At = columns of X = R^T
    Vt = None
    solve32 = a.strategy == "rt32"
    a.strategy = "base"
if a.strategy.startswith("eigpre"):
    # eigenvectors of the fp32 Gram as the starting V (A1 = A Q, V0 = Q)
    G = A.t() @ A
    if a.strategy == "eigpre64":
        _, Q = torch.linalg.eigh(G.double())
        Q = Q.float()
    else:
        _, Q = torch.linalg.eigh(G)
    Q = Q.flip(1).contiguous()
    At = (A @ Q).t().contiguous()
    Vt = Q.t().contiguous()
    a.strategy = "base"
D = (At.double() ** 2).sum(1).float()
tol = math.sqrt(n) * torch.finfo(torch.float32).eps
rr = torch.from_numpy(svdj.parallel.schedule.round_robin(nb).copy())
hist = []
applied_total = 0
gram_total = 0
prev_q = None
for sw in range(a.max_sweeps):
    offs = []
    if a.strategy == "base" or sw < a.k0 or prev_q is None:
        tau = tol
    elif a.strategy == "median":      # skip pairs below c x the previous sweep's median coupling
        tau = max(tol, a.c * prev_q[0.5])
    elif a.strategy == "q90":
        tau = max(tol, a.c * prev_q[0.9])
    else:
        raise SystemExit(a.strategy)
    applied = 0
    for s in range(rr.shape[0]):
        pairs = rr[s]
        full = s == 0
        ar = torch.arange(W)
        ci = pairs[:, 0].long()[:, None] * W + ar
        cj = pairs[:, 1].long()[:, None] * W + ar
        C = At[ci] @ At[cj].transpose(1, 2)
        den = D[ci].clamp(min=0).sqrt()[:, :, None] * D[cj].clamp(min=0).sqrt()[:, None, :]
        off = (C.abs() / den.clamp(min=1e-30)).amax((1, 2))
        offs.append(off)
        _, nrot = R.block_step(At, Vt, D, pairs, W, full, tol if full else tau, 1, order="cross")
        applied += nrot if not full else pairs.shape[0]
        gram_total += pairs.shape[0]
    offs = torch.cat(offs).double()
    q = {x: float(torch.quantile(offs, x)) for x in (0.1, 0.5, 0.9)}
    q["max"] = float(offs.max())
    prev_q = q
    applied_total += applied
    # convergence: a sweep at the final tolerance that rotates nothing
    conv = tau == tol and applied == 0
    print(json.dumps({"sweep": sw + 1, "tau": "%.2e" % tau, "applied": applied,
                      "pairs": int(offs.numel()),
                      "q10": "%.2e" % q[0.1], "q50": "%.2e" % q[0.5], "q90": "%.2e" % q[0.9],
                      "max": "%.2e" % q["max"]}), flush=True)
    if tau == tol and all(float(o.max()) < tol for o in [offs]):
        break
if Qqr is not None:
    Xf = At.double().t()                   # X_final = X V_x = U_x S
    Sx = Xf.norm(dim=0)
    Ux = Xf / Sx
    if solve32:
        Vx = torch.linalg.solve_triangular(Rqr.t().float(), Xf.float(), upper=False).double()
    else:
        Vx = torch.linalg.solve_triangular(Rqr.t(), Xf, upper=False)   # R^T V_x = X_final
    Ad = (Qqr @ Vx) * Sx                   # A = Q R = (Q V_x) S U_x^T: columns U_A S
    Vd = Ux
else:
    Ad, Vd = At.double().t(), Vt.double().t()
S = Ad.norm(dim=0)
U = Ad / S
res = float((A.double() - U @ torch.diag(S) @ Vd.t()).norm() / A.double().norm())
sv = torch.linalg.svdvals(A.double())
err = float((torch.sort(S, descending=True).values - sv).abs().max() / sv[0])
print(json.dumps({"strategy": a.strategy, "c": a.c, "k0": a.k0, "sweeps": sw + 1,
                  "applied_pairs": applied_total, "gram_pairs": gram_total,
                  "cost_units": applied_total * 4 + gram_total,
                  "residual": "%.2e" % res, "sigma_err": "%.2e" % err,
                  "orth_v": "%.2e" % float((Vd.t() @ Vd - torch.eye(n, dtype=torch.float64)).abs().max())}),
      flush=True)
