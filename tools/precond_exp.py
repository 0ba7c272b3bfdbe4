"""Square-matrix QR preconditioning experiment (dev aid): sweeps and time of
the block solver on A versus on R^T from A = QR (Drmac-Veselic style; one-sided
Jacobi on R^T, then U = Q V_R, V = U_R).

    python tools/precond_exp.py n [n ...]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import svdj  # noqa: E402

dev = torch.device("cuda", 0)
for n in [int(x) for x in sys.argv[1:]]:
    g = torch.Generator(device=dev).manual_seed(1234)
    A = torch.rand(n, n, generator=g, device=dev)

    def timed(f):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = f()
        torch.cuda.synchronize()
        return r, time.perf_counter() - t0

    svdj.svd(A, method="block")  # warm
    res, t_plain = timed(lambda: svdj.svd(A, method="block"))
    (Q, R), t_qr = timed(lambda: torch.linalg.qr(A))
    (Q, R), t_qr = timed(lambda: torch.linalg.qr(A))
    Rt = R.t().contiguous()
    res2, t_j = timed(lambda: svdj.svd(Rt, method="block"))
    _, t_gemm = timed(lambda: Q @ res2.V)
    print(f"n={n}: plain {res.sweeps} sweeps {t_plain:.3f} s | QR {t_qr:.3f} s + Jacobi(R^T) "
          f"{res2.sweeps} sweeps {t_j:.3f} s + U=QV {t_gemm:.3f} s = {t_qr + t_j + t_gemm:.3f} s",
          flush=True)
