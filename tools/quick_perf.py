"""Quick single-GPU timing sweep (development aid)."""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import svdj  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--sizes", default="1024,2048,4096")
p.add_argument("--method", default="block")
p.add_argument("--dtype", default="fp32")
p.add_argument("--block", type=int, default=None)
p.add_argument("--inner", type=int, default=1)
p.add_argument("--mma", default="auto")
p.add_argument("--verify", action="store_true")
a = p.parse_args()
dt = torch.float32 if a.dtype == "fp32" else torch.float64
dev = torch.device("cuda:0")
for n in [int(x) for x in a.sizes.split(",")]:
    A = svdj.utils.inputs.random_dense(n, n, dtype=dt, device=dev, seed=1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = svdj.svd(A, method=a.method, dtype=dt, block=a.block, max_inner_sweeps=a.inner,
                   mma=a.mma)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    out = {"n": n, "method": a.method, "dtype": a.dtype, "sweeps": res.sweeps, "sec": round(t, 4),
           "solver_sec": round(res.seconds, 4),
           "gflops_alg": round(svdj.utils.metrics.gflops(n, n, res.sweeps, t), 1),
           "block": res.info.get("block"), "mma": a.mma, "hist": ["%.1e" % h for h in res.history]}
    if a.verify:
        ref = torch.linalg.svdvals(A.double())
        out.update(svdj.utils.metrics.verify(A, res.U, res.S, res.V, ref))
    print(json.dumps(out), flush=True)
