"""Isolated cross-Gram timing, register-fragment vs LDS-staged kernel (dev aid).

    python tools/gram_iso.py [m]
"""
import sys

import os
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import svdj

K = svdj.ops.kernels
m = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
W = 64
dev = torch.device("cuda", 0)
for npairs, rows in ((64, 2048), (64, 1024), (8, 256), (8, 512), (32, 512)):
    At = torch.rand(2 * npairs * W, m, device=dev)
    pairs = torch.arange(2 * npairs, dtype=torch.int32).view(npairs, 2)
    out = {}
    for kern in ("reg", "lds4", "lds3", "lds2", "reg", "lds4", "lds3", "lds2"):
        kw = dict(kernel="lds", depth=int(kern[3])) if kern.startswith("lds") else dict(kernel="reg")
        for _ in range(3):
            K.gram_cross(At, m, pairs, W, rows, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            K.gram_cross(At, m, pairs, W, rows, **kw)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        out[kern] = us
    gb = 2 * npairs * W * m * 4 / 1e9
    print(f"m={m} pairs={npairs} rows/chunk={rows}: " + ", ".join(
        f"{k} {v:.1f} us ({gb / v * 1e3:.2f} TB/s)" for k, v in out.items()), flush=True)
