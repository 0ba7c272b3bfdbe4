"""Per-phase cycle split of the block EVD kernel (dev aid; needs a library
built with -DSVDJ_EVD_PROFILE, selected through SVDJ_HIP_LIB)."""
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
names = ["ph1_solve", "bar1_wait", "ph2_update", "bar2_wait", "dpp_shift"]
for W in (32, 64):
    n = 64 * W
    At = torch.rand(n, n, device=dev)
    Vt = torch.zeros(n, n, device=dev)
    K.set_identity(Vt, n)
    D = K.col_norms2(At, n)
    pairs = torch.from_numpy(svdj.parallel.schedule.round_robin(n // W)).to(dev)
    buf = (C.c_ulonglong * 16)()
    fn(buf, 1)
    K.block_steps(At, Vt, D, n, pairs[:8], W, [1] + [0] * 7, 1e-30, 1, K.new_metric(dev))
    torch.cuda.synchronize()
    fn(buf, 1)
    steps = 8 * (2 * W - 1)
    print(json.dumps({"W": W, "wave0_cycles_per_step": {k: round(buf[i] / steps, 1) for i, k in enumerate(names)},
                      "lastwave_cycles_per_step": {k: round(buf[8 + i] / steps, 1) for i, k in enumerate(names)}}))
