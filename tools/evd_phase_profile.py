"""Per-phase cycle split of the block EVD kernel (dev aid; needs a library
built with -DSVDJ_EVD_PROFILE, selected through SVDJ_HIP_LIB).

Slots (pair 0, wave 0 lane 0 and the last wave's lane 0): per step
0 = block update (+ next-step solves in wave 0), 1 = Q rotation + DPP shift
(Q waves), 2 = whole step incl. the barrier; per kernel 4 = setup (assembly,
pre-pass, prologue), 5 = all sweeps."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdj  # noqa: E402

K = svdj.ops.kernels
fn = svdj.ops.hip_lib().svdj_debug_evd_profile
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
dev = torch.device("cuda:0")
names = {0: "update_solve", 1: "q_dpp", 2: "step_total", 4: "setup_per_kernel",
         5: "sweeps_per_kernel"}
import argparse  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=0, help="rows (default 64 W)")
ap.add_argument("--pairs", type=int, default=32, help="pairs per step")
ap.add_argument("--order", default="bipartite", choices=["cyclic", "bipartite"])
ap.add_argument("--cases", default="fp32:32,fp32:64,fp64:32")
args = ap.parse_args()
for case in args.cases.split(","):
    dname, Wn = case.split(":")
    dt, W = (torch.float32 if dname == "fp32" else torch.float64), int(Wn)
    if True:
        n = 2 * args.pairs * W
        m = args.m or n
        At = torch.rand(n, m, device=dev, dtype=dt)
        Vt = torch.zeros(n, n, device=dev, dtype=dt)
        K.set_identity(Vt, n)
        D = K.col_norms2(At, m)
        pairs = torch.from_numpy(svdj.parallel.schedule.round_robin(n // W)).to(dev)
        buf = (C.c_ulonglong * 16)()
        K.block_steps(At, Vt, D, m, pairs[:8], W, [1] + [0] * 7, 1e-30, 1, K.new_metric(dev),
                      inner_order=args.order)
        torch.cuda.synchronize()
        fn(buf, 1)
        cross = pairs[8:16]
        K.block_steps(At, Vt, D, m, cross, W, [0] * int(cross.shape[0]), 1e-30, 1,
                      K.new_metric(dev), inner_order=args.order)
        torch.cuda.synchronize()
        fn(buf, 1)
        steps = int(cross.shape[0]) * (W if args.order == "bipartite" else 2 * W - 1)
        out = {"dtype": str(dt), "W": W, "m": m, "pairs": args.pairs, "order": args.order}
        for who, off in (("wave0", 0), ("lastwave", 8)):
            out[who] = {v: round(buf[off + k] / (steps if k < 4 else int(cross.shape[0])), 1)
                        for k, v in names.items()}
        print(json.dumps(out), flush=True)
