"""Worker for multi-process (gloo) distributed tests; launched by torchrun."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdj  # noqa: E402
from svdj.parallel import Communicator, DistributedBlockJacobi  # noqa: E402


def main():
    m, n, W, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    mode = sys.argv[5] if len(sys.argv) > 5 else "root"
    comm = Communicator(backend="gloo", device=torch.device("cpu"),
                        timeout_s=float(os.environ.get("SVDJ_TEST_TIMEOUT", "600")))
    cfg = svdj.SolverConfig(block=W, dtype=torch.float64, max_inner_sweeps=1,
                            precondition="qr" if "qr" in mode else "none")
    if mode == "fault":  # rank 1 dies after sweep 1; rank 0 must fail, not hang
        cfg.extra["fault_exit"] = (1, 1)
        mode = "root"
    solver = DistributedBlockJacobi(cfg, comm)
    A = svdj.utils.inputs.random_dense(m, n, dtype=torch.float64, seed=9)
    if mode == "roundtrip":  # reference test_local_matrix_distribution_* parity
        U = solver.roundtrip(A if comm.rank == 0 else None, m, n)
        if comm.rank == 0:
            with open(out, "w") as f:
                json.dump({"max_err": float((U - A).abs().max()), "world": comm.world}, f)
        comm.destroy()
        return
    if mode == "isend":  # reference test_MPI_Isend_Recv parity: ring exchange
        x = torch.full((5,), float(comm.rank), dtype=torch.float64)
        y = torch.empty(5, dtype=torch.float64)
        nxt, prv = (comm.rank + 1) % comm.world, (comm.rank - 1) % comm.world
        for w in comm.isendrecv([(x, nxt)], [(y, prv)]):
            w.wait()
        ok = bool((y == prv).all())
        t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64)
        import torch.distributed as dist
        dist.all_reduce(t)
        if comm.rank == 0:
            with open(out, "w") as f:
                json.dump({"ok_ranks": float(t[0]), "world": comm.world}, f)
        comm.destroy()
        return
    if mode == "ordsum":  # rank-ordered sum: slabbed (bounded memory) == whole, same bits
        g = torch.Generator().manual_seed(100 + comm.rank)
        x = torch.randn(37, 53, generator=g, dtype=torch.float64)
        whole = comm.ordered_sum_(x.clone(), max_bytes=1 << 30)
        slab = comm.ordered_sum_(x.clone(), max_bytes=8 * comm.world * 5)  # 5 elements per slab
        xt = x.clone().t()  # non-contiguous
        slab_t = comm.ordered_sum_(xt, max_bytes=8 * comm.world * 7)
        ref = None
        for h in range(comm.world):
            y = torch.randn(37, 53, generator=torch.Generator().manual_seed(100 + h),
                            dtype=torch.float64)
            ref = y.clone() if ref is None else ref.add_(y)
        if comm.rank == 0:
            with open(out, "w") as f:
                json.dump({"slab_eq_whole": bool(torch.equal(slab, whole)),
                           "whole_eq_ref": bool(torch.equal(whole, ref)),
                           "slab_t_eq": bool(torch.equal(slab_t.t(), whole)),
                           "world": comm.world}, f)
        comm.destroy()
        return
    if mode == "localsvd":  # svd() inside a distributed job solves this rank's matrix alone
        B = svdj.utils.inputs.random_dense(m, n, dtype=torch.float64, seed=50 + comm.rank)
        res = svdj.svd(B, method="block", device="cpu", block=W, extra={"engine": "pipeline"})
        ref = torch.linalg.svdvals(B)
        err = float((res.S.sort(descending=True).values - ref).abs().max() / ref[0])
        resid = float((B @ res.V - res.U * res.S).norm() / B.norm())
        t = torch.tensor([max(err, resid)], dtype=torch.float64)
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if comm.rank == 0:
            with open(out, "w") as f:
                json.dump({"max_err": float(t[0]), "engine": res.info["engine"],
                           "converged": res.converged, "world": comm.world}, f)
        comm.destroy()
        return
    if mode == "calib":  # startup exchange calibration: same choice on every rank, data intact
        from svdj.parallel.pipeline import calibrate_exchange
        from svdj.parallel.schedule import tournament
        tour = tournament(comm.world)
        choice, summary = calibrate_exchange(comm, tour, [(8, 300), (8, 256)], torch.float64,
                                             torch.device("cpu"), reps=1)
        flag = torch.tensor([1.0 if choice == "spread" else 0.0], dtype=torch.float64)
        import torch.distributed as dist
        lo, hi = flag.clone(), flag.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        if comm.rank == 0:
            with open(out, "w") as f:
                json.dump({"choice": choice, "summary": summary, "agree": float(lo[0]) == float(hi[0]),
                           "world": comm.world}, f)
        comm.destroy()
        return
    if mode == "exchcmp":  # spread (relayed over all links) vs direct exchange: same bits
        got = {}
        for ex in ("direct", "spread"):
            cfg.exchange = ex
            res = DistributedBlockJacobi(cfg, comm).solve(A if comm.rank == 0 else None)
            got[ex] = res
        if comm.rank == 0:
            d, s_ = got["direct"], got["spread"]
            with open(out, "w") as f:
                json.dump({"u_diff": float((d.U - s_.U).abs().max()),
                           "s_diff": float((d.S - s_.S).abs().max()),
                           "v_diff": float((d.V - s_.V).abs().max()),
                           "sweeps": [d.sweeps, s_.sweeps],
                           "exchange": [d.info["exchange"], s_.info["exchange"]],
                           "relayed": s_.info["comm"]["bytes_relayed"],
                           "exchanges": [d.info["comm"]["exchanges"], s_.info["comm"]["exchanges"]],
                           "timing": [d.info["comm"]["timing"], s_.info["comm"]["timing"]],
                           "comm_ms_absent": "comm_ms" not in d.info["comm"],
                           "world": comm.world}, f)
        comm.destroy()
        return
    if mode == "otf":  # on-the-fly generated input through the public API
        res = svdj.svd_on_the_fly(m, n, lambda c0, c1: A[:, c0:c1], comm=comm,
                                  dtype=torch.float64, config=cfg)
        if comm.rank == 0:
            rep = svdj.utils.metrics.verify(A, res.U, res.S, res.V, torch.linalg.svdvals(A))
            rep.update(sweeps=res.sweeps, converged=res.converged, world=comm.world)
            with open(out, "w") as f:
                json.dump(rep, f)
        comm.destroy()
        return
    if mode == "genqr_rows":  # row-distributed QR output: U row block, full S and V
        import torch.distributed as dist
        res = solver.solve(None, m=m, n=n, dtype=torch.float64,
                           generator=lambda c0, c1: A[:, c0:c1], gather=False)
        r0, r1 = res.info["u_rows"]
        U, S, V = res.U, res.S, res.V
        parts = torch.stack([(A[r0:r1] @ V - U * S).pow(2).sum(), A[r0:r1].pow(2).sum()])
        UtU = U.t() @ U
        dist.all_reduce(parts)
        dist.all_reduce(UtU)
        if comm.rank == 0:
            eye = torch.eye(n, dtype=torch.float64)
            ref = torch.linalg.svdvals(A)
            with open(out, "w") as f:
                json.dump({"residual_rel": float((parts[0] / parts[1]).sqrt()),
                           "orth_u_fro": float((UtU - eye).norm()),
                           "orth_v_fro": float((V.t() @ V - eye).norm()),
                           "sigma_err": float((torch.sort(S, descending=True).values - ref).abs().max()
                                              / ref[0]),
                           "rows": [r0, r1], "converged": res.converged, "world": comm.world}, f)
        comm.destroy()
        return
    if mode in ("root", "rootqr"):
        res = solver.solve(A if comm.rank == 0 else None)
    else:
        res = solver.solve(None, m=m, n=n, dtype=torch.float64,
                           generator=lambda c0, c1: A[:, c0:c1])
    if comm.rank == 0:
        rep = svdj.utils.metrics.verify(A, res.U, res.S, res.V, torch.linalg.svdvals(A))
        rep.update(sweeps=res.sweeps, converged=res.converged, world=comm.world)
        with open(out, "w") as f:
            json.dump(rep, f)
    comm.destroy()


if __name__ == "__main__":
    main()
