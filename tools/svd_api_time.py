"""Time the public entry point svdj.svd(A) on the bench's input (development aid).

VERDICT r5 #2: svd() must run the engine bench.py times.  This builds bench.py's
exact matrix (make_generator: U(0,1), seeded per 256-column block), then times
``svdj.svd(A)`` (input already on the device, U, S, V returned in the
reference's layout) and ``svdj.svd(A, extra={"engine": "steps"})``; prints one
JSON line per engine with seconds, sweeps and the residual.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import svdj  # noqa: E402
from bench import make_generator  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=16384)
p.add_argument("--reps", type=int, default=2)
p.add_argument("--engines", default="pipeline,steps")
a = p.parse_args()
dev = torch.device("cuda", 0)
n = a.n
gen = make_generator(n, dev, torch.float32, torch.float32)
A = torch.cat([gen(c0, min(c0 + 1024, n)) for c0 in range(0, n, 1024)], dim=1)
for eng in a.engines.split(","):
    for rep in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = svdj.svd(A, extra={"engine": eng})
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rel = float((A @ res.V - res.U * res.S).norm() / A.norm())
        print(json.dumps({"engine": eng, "rep": rep, "n": n, "seconds": round(dt, 4),
                          "solver_seconds": round(res.seconds, 4), "sweeps": res.sweeps,
                          "quad": res.info.get("quad"), "merged": res.info.get("merged_chains"),
                          "residual_rel": rel}), flush=True)
        del res
