"""Prints the accuracy figures the GPU tests bound (dev aid for setting test
tolerances a few times above the measured values)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdj  # noqa: E402

cuda = torch.device("cuda:0")
m, n = 520, 384
A = svdj.utils.inputs.random_dense(m, n, dtype=torch.float64, seed=3)
ref = torch.linalg.svdvals(A)
for method, dtype, mma in [("block", torch.float32, "native"), ("block", torch.float32, "bf16x6"),
                           ("block", torch.float64, "native"), ("scalar", torch.float32, "native"),
                           ("scalar", torch.float64, "native")]:
    res = svdj.svd(A.to(cuda), method=method, dtype=dtype, mma=mma)
    rep = svdj.utils.metrics.verify(A.to(cuda), res.U, res.S, res.V, ref)
    print(json.dumps({"test": "end_to_end", "method": method, "dtype": str(dtype), "mma": mma,
                      "sweeps": res.sweeps, "converged": res.converged,
                      **{k: rep[k] for k in ("residual_rel", "sigma_max_abs_err_over_smax",
                                             "orth_u_fro", "orth_v_fro")}}))
A = svdj.utils.inputs.random_dense(512, 512, dtype=torch.float32, device=cuda, seed=2)
for m_ in ("block", "scalar"):
    res = svdj.svd(A, method=m_)
    rep = svdj.utils.metrics.verify(A, res.U, res.S, res.V, torch.linalg.svdvals(A.double().cpu()))
    print(json.dumps({"test": "drivers_512", "method": m_, "sweeps": res.sweeps,
                      **{k: rep[k] for k in ("residual_rel", "orth_u_fro", "orth_v_fro")}}))
