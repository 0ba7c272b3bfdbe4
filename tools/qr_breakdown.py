"""Time the pieces of the tall-skinny preconditioner (models/precondition.py)
on one GPU: CholeskyQR2 (2 x [Gram, Cholesky, TRSM], R product) and the final
U = Q U_R GEMM, each bracketed by HIP events, median of --reps runs.

Usage: python tools/qr_breakdown.py [--m 32768] [--n 8192] [--dtype fp32]
Prints one JSON line: ms per piece, the executed TFLOP/s of the m x n x n
pieces (full GEMM for the Gram, m n^2 for a TRSM), and the total.
"""
import argparse
import json
import statistics

import torch


def timed(fn, reps):
    out, ts = None, []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return out, statistics.median(ts)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=32768)
    p.add_argument("--n", type=int, default=8192)
    p.add_argument("--dtype", default="fp32", choices=["fp32", "fp64"])
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    dt = torch.float32 if a.dtype == "fp32" else torch.float64
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.rand(a.m, a.n, device="cuda", dtype=dt, generator=g)
    ms = {}
    Q, R = A, None
    for it in range(2):
        G, ms[f"gram{it}"] = timed(lambda: Q.t() @ Q, a.reps)
        (L, info), ms[f"chol{it}"] = timed(lambda: torch.linalg.cholesky_ex(G), a.reps)
        assert int(info) == 0
        Qn, ms[f"trsm{it}"] = timed(
            lambda: torch.linalg.solve_triangular(L.t(), Q, upper=True, left=False), a.reps)
        if R is not None:
            R, ms["r_product"] = timed(lambda: L.t() @ R, a.reps)
        else:
            R = L.t()
        Q = Qn
    UR = torch.linalg.qr(torch.rand(a.n, a.n, device="cuda", dtype=dt, generator=g))[0]
    _, ms["u_gemm"] = timed(lambda: Q @ UR, a.reps)
    # deferred form used by the solvers (precondition.apply_q): Q is never
    # formed, U = Q1 (L2^-T U_R) -- an n x n TRSM instead of trsm1
    _, ms["nn_trsm_deferred"] = timed(
        lambda: torch.linalg.solve_triangular(L.t(), UR, upper=True), a.reps)
    mnn = 2.0 * a.m * a.n * a.n  # executed flops of the full GEMMs; a TRSM is half
    tf = {k: (mnn / 2 if k.startswith("trsm") else mnn) / (v * 1e-3) / 1e12
          for k, v in ms.items() if k.startswith(("gram", "trsm", "u_gemm"))}
    orth = float((Q.t() @ Q - torch.eye(a.n, device="cuda", dtype=dt)).norm())
    print(json.dumps({"m": a.m, "n": a.n, "dtype": a.dtype, "ms": {k: round(v, 3) for k, v in ms.items()},
                      "total_ms": round(sum(ms.values()) - ms["nn_trsm_deferred"], 3),
                      "total_deferred_ms": round(sum(ms.values()) - ms["trsm1"], 3),
                      "tflops_useful": {k: round(v, 1) for k, v in tf.items()},
                      "q_orth_fro": orth}))


if __name__ == "__main__":
    main()
