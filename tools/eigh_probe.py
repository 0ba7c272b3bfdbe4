"""Timing of the dense symmetric eigensolvers torch reaches on this box
(development aid): torch.linalg.eigh of the fp32 Gram A^T A with each
available linalg backend, for the eigenvector-preconditioned Jacobi option."""
import json
import sys
import time

import torch

dev = torch.device("cuda:0")
sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4096,8192,16384").split(",")]
backs = ["default"]
for b in ("magma", "cusolver"):
    try:
        torch.backends.cuda.preferred_linalg_library(b)
        backs.append(b)
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"backend": b, "error": str(e)[:200]}), flush=True)
torch.backends.cuda.preferred_linalg_library("default")
for n in sizes:
    A = torch.rand(n, n, device=dev)
    G = A.t() @ A
    torch.cuda.synchronize()
    for b in backs:
        torch.backends.cuda.preferred_linalg_library(b)
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            try:
                lam, Q = torch.linalg.eigh(G)
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"n": n, "backend": b, "error": str(e)[:200]}), flush=True)
                break
            dt = time.perf_counter() - t0
            orth = float((Q.t() @ Q - torch.eye(n, device=dev)).abs().max())
            print(json.dumps({"n": n, "backend": b, "rep": rep, "s": round(dt, 3), "orth": orth}),
                  flush=True)
        if n >= 16384 and dt > 60:
            break
    torch.backends.cuda.preferred_linalg_library("default")
    del A, G
