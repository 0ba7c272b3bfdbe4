"""Per-step timing probe at the 1-GPU flagship geometry (development aid).

Prints, as JSON lines:
  * the device copy bandwidth (read + write) of a 2 GiB fp32 tensor, the
    practical HBM ceiling the block steps are held against;
  * the time of S block steps of P pairs (W = 64 columns per block, m rows)
    on one stream, fresh pairs every step (round-robin steps), split-bf16
    apply, cross EVD -- per step and as achieved bytes/s of the data the step
    must move (Gram read of A + apply read/write of A and V).
Run under ``rocprofv3 --kernel-trace --stats`` for the per-kernel split.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdj  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--m", type=int, default=16384)
p.add_argument("--nb", type=int, default=256, help="blocks of W columns")
p.add_argument("--pairs", type=int, default=64, help="pairs per step")
p.add_argument("--steps", type=int, default=24)
p.add_argument("--reps", type=int, default=3)
p.add_argument("--mma", default="bf16x6")
p.add_argument("--quad", action="store_true", help="quad steps (modes 4/5) on quad_round_robin pairs")
p.add_argument("--no-copy", action="store_true")
a = p.parse_args()
K = svdj.ops.kernels
dev = torch.device("cuda:0")
W = 64

x = torch.empty(2 ** 29 if not a.no_copy else 1, dtype=torch.float32, device=dev).uniform_()
y = torch.empty_like(x)
best = 1e9
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    y.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1))
print(json.dumps({"probe": "copy", "bytes": 2 * x.numel() * 4, "ms": round(best, 3),
                  "TB_s": round(2 * x.numel() * 4 / best / 1e9, 3)}), flush=True)
best = 1e9
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    x.sum()
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1))
print(json.dumps({"probe": "read (torch sum)", "bytes": x.numel() * 4, "ms": round(best, 3),
                  "TB_s": round(x.numel() * 4 / best / 1e9, 3)}), flush=True)
del x, y

n, m = a.nb * W, a.m
sch = svdj.parallel.schedule
rr = sch.quad_round_robin(a.nb) if a.quad else sch.round_robin(a.nb)  # (nb - 1, nb / 2, 2)
pairs = torch.from_numpy(rr[1:1 + a.steps, :a.pairs].copy()).to(dev)
modes = [4, 5] * (a.steps // 2) if a.quad else [0] * a.steps
g = torch.Generator(device=dev).manual_seed(1)
A0 = torch.rand(n, m, dtype=torch.float32, device=dev, generator=g)
for rep in range(a.reps):
    At = A0.clone()
    Vt = torch.zeros(n, n, dtype=torch.float32, device=dev)
    K.set_identity(Vt, n)
    D = K.col_norms2(At, m)
    metric = K.new_metric(dev)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    K.block_steps(At, Vt, D, m, pairs, W, modes, 1e-30, 1, metric, mma=a.mma,
                  inner_order="cross")
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    per = ms / a.steps
    moved = a.pairs * 2 * W * 4 * (m + 2 * m + 2 * n)  # Gram read A; apply r/w A and V
    print(json.dumps({"probe": "steps", "rep": rep, "m": m, "n": n, "pairs": a.pairs, "mma": a.mma, "quad": a.quad,
                      "us_per_step": round(per * 1e3, 1), "TB_s_needed_bytes": round(moved / per / 1e9, 3),
                      "rotated": K.read_metric(metric)[1]}), flush=True)
