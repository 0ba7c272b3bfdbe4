"""Numerics probe of the block apply X <- X Q per matrix-core mode (dev aid).

1. one apply vs an fp64 product of the same fp32 inputs: max / rms relative
   error and the mean signed error (bias) in units of fp32 eps;
2. drift: 200 random orthogonal Q applied to an orthonormal X (what V sees),
   ||X^T X - I||_max after each 50.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdj  # noqa: E402

K = svdj.ops.kernels
dev = torch.device("cuda:0")
eps = torch.finfo(torch.float32).eps
g = torch.Generator().manual_seed(0)


def rand_q(N):
    q, _ = torch.linalg.qr(torch.randn(N, N, generator=g, dtype=torch.float64))
    return q


for W in (32, 64):
    N, rows = 2 * W, 4096
    X0 = torch.rand(N, rows, generator=g, dtype=torch.float64).float()
    Q = rand_q(N).float()
    ref = (Q.double().t() @ X0.double())  # (X Q)^T = Q^T X^T
    out = {"W": W}
    for mma in ("native", "bf16x6", "bf16x3"):
        Xt = X0.to(dev).contiguous()
        K.apply_q(Xt, Q.to(dev).contiguous(), W, mma)
        err = (Xt.double().cpu() - ref) / (ref.abs() + 1e-30)
        scale = ref.abs().max()
        e_abs = (Xt.double().cpu() - ref)
        out[mma] = {"max_rel_eps": round(float(err.abs().max()) / eps, 2),
                    "rms_abs_over_max_eps": round(float(e_abs.pow(2).mean().sqrt() / scale) / eps, 3),
                    "bias_over_max_eps": round(float(e_abs.mean() / scale) / eps, 4)}
        # drift on an orthonormal panel
        V = torch.linalg.qr(torch.randn(rows, N, generator=g, dtype=torch.float64))[0].t()
        Vt = V.float().to(dev).contiguous()
        drift = []
        for it in range(200):
            K.apply_q(Vt, rand_q(N).float().to(dev).contiguous(), W, mma)
            if (it + 1) % 50 == 0:
                v = Vt.double().cpu()
                drift.append(float((v @ v.t() - torch.eye(N, dtype=torch.float64)).abs().max()))
        out[mma]["orth_drift"] = ["%.2e" % d for d in drift]
    print(json.dumps(out), flush=True)

# 3. Jacobi-like late-stage drift: one dominant column (x1000), Q = near-identity
#    rotations; track each column norm against an fp64 replay of the same Qs.
for W in (32, 64):
    N, rows = 2 * W, 2048
    X0 = torch.rand(N, rows, generator=g, dtype=torch.float64) * 0.1
    X0[3] = torch.rand(rows, generator=g, dtype=torch.float64) * 100.0
    X0 = X0.float()
    Qs = []
    for it in range(400):
        S = torch.randn(N, N, generator=g, dtype=torch.float64) * 1e-3
        Qs.append(torch.linalg.matrix_exp(S - S.t()).float())
    out = {"W": W, "probe": "dominant-column drift (rel err of column norms after 400 applies)"}
    ref = X0.double()
    for Q in Qs:
        ref = Q.double().t() @ ref
    rn = ref.norm(dim=1)
    for mma in ("native", "bf16x6"):
        Xt = X0.to(dev).contiguous()
        for Q in Qs:
            K.apply_q(Xt, Q.to(dev).contiguous(), W, mma)
        e = (Xt.double().cpu().norm(dim=1) - rn) / rn
        out[mma] = {"dominant_eps": round(float(e[3]) / eps, 2), "max_abs_eps": round(float(e.abs().max()) / eps, 2),
                    "mean_eps": round(float(e.mean()) / eps, 3)}
    print(json.dumps(out), flush=True)
