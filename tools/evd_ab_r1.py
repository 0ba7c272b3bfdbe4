"""evd_ab.py for the round-1 library (its svdj_block_steps has no tol_mode
argument): same single-stream sweep, for before/after kernel timings.
Usage: SVDJ_HIP_LIB=.../libsvdj_hip_r1.so python tools/evd_ab_r1.py --n 4096 --block 32"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdj  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=4096)
p.add_argument("--block", type=int, default=32)
p.add_argument("--sweeps", type=int, default=2)
a = p.parse_args()
lib = C.CDLL(os.environ["SVDJ_HIP_LIB"])
vp, ci, cd = C.c_void_p, C.c_int, C.c_double
lib.svdj_block_steps.argtypes = [ci, ci, ci, vp, ci, vp, ci, ci, vp, vp, ci, ci,
                                 C.POINTER(C.c_int32), cd, ci, vp, C.c_size_t, vp, ci, vp]
lib.svdj_block_workspace_bytes.restype = C.c_size_t
lib.svdj_block_workspace_bytes.argtypes = [ci, ci, ci, ci]
dev = torch.device("cuda:0")
n, W = a.n, a.block
nb = n // W
pairs = torch.from_numpy(svdj.parallel.schedule.round_robin(nb)).to(dev)
modes = (C.c_int32 * (nb - 1))(*([1] + [0] * (nb - 2)))
g = torch.Generator(device=dev).manual_seed(1)
At = torch.rand(n, n, device=dev, generator=g)
Vt = torch.eye(n, device=dev)
D = (At.double() ** 2).sum(1).float()
ws = torch.empty(int(lib.svdj_block_workspace_bytes(0, W, nb // 2, n)), dtype=torch.uint8, device=dev)
metric = torch.zeros(2, dtype=torch.int32, device=dev)
tol = svdj.utils.metrics.default_tol(torch.float32, n)
st = vp(torch.cuda.current_stream().cuda_stream)


def sweep():
    rc = lib.svdj_block_steps(0, W, n, vp(At.data_ptr()), n, vp(Vt.data_ptr()), n, n,
                              vp(D.data_ptr()), vp(pairs.data_ptr()), nb // 2, nb - 1, modes, tol, 1,
                              vp(ws.data_ptr()), ws.numel(), vp(metric.data_ptr()), 0, st)
    assert rc == 0, rc


sweep()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.sweeps):
    sweep()
e1.record()
torch.cuda.synchronize()
print(json.dumps({"n": n, "W": W, "ms_per_sweep": round(e0.elapsed_time(e1) / a.sweeps, 3),
                  "lib": "round-1"}))
