#!/usr/bin/env python3
"""Headline benchmark: dense one-sided Jacobi SVD to convergence on N MI355X.

Metric (BASELINE.json): GFLOP/s + time-to-converge (sweeps to ||off|| < tol),
N x N dense SVD at 1/2/4/8 MI355X.  One "step" = one complete SVD solve
(A -> U, sigma, V with AllVec/AllVec, every sweep until a sweep applies no
rotation) of a synthetic random dense U(0,1) matrix, fp32, distributed as a
column-block tournament over the N GPUs (one process per GPU, RCCL).

GFLOP/s counts the reference's algorithmic work per sweep,
n(n-1)/2 * (12 m + 6 n), times the sweeps actually
executed, divided by the measured wall time of the solve; the value is the
whole-job aggregate.  Strong scaling: the matrix size is fixed as N grows.

Input/output placement:
  default       every rank generates its own columns inside the timed region
                (on-the-fly input) and keeps its U/V/sigma columns;
  --root-owned  rank 0 holds A before the timed region; the timed region
                includes the scatter to all ranks and the gather of U, sigma
                and V back to rank 0 (the reference's timing, main.cu:1586-1611).

Simulation (one process, no RCCL): ``--simulate-P P --simulate-rank g`` runs
rank g's exact per-GPU plan of a P-GPU job with every exchange replaced by a
device swap of the real message sizes (parallel/comm.py SimCommunicator), for
a fixed number of sweeps; it reports the per-GPU time per sweep.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--n 16384]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

# What each matrix-core mode of the block apply computes (reported in the JSON line).
MMA_NUMERICS = {
    "native": "IEEE f32/f64 MFMA products and sums",
    "bf16x6": ("fp32 data, fp32 accumulation: every fp32 operand split exactly into 3 RNE bf16 "
               "parts, the 6 products of order < 3 on bf16 MFMA (dropped terms < 2^-26 relative), "
               "delta form X + X(Q - I) with the identity added in fp32; accuracy block = the "
               "check (README 'Matrix-core modes')"),
    "bf16x3": "bf16 problem mode: 2-way bf16 split (~2^-17), fp32 master copies",
}

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = ("GFLOP/s + time-to-converge (sweeps to ||off||<tol), N×N dense SVD at "
                   "1/2/4/8 MI355X")


def _global_columns(res, n, comm):
    """Indices (rows of At / Vt / S) of this rank's real columns and their
    global column ids, in slot order (padding columns >= n dropped)."""
    B = res.info["geometry"]["B"]
    loc, glob = [], []
    for s_, sb in enumerate(res.info["held"]):
        for j in range(B):
            if sb * B + j < n:
                loc.append(s_ * B + j)
                glob.append(sb * B + j)
    return loc, glob


def verify_distributed(res, gen, m, n, comm, dtype):
    """Accuracy of the distributed result, after the timed region.

    Every rank regenerates A (same seeded generator) and checks its own
    columns: ||A V_loc - U_loc S_loc||_F^2.  Orthogonality is FULL: U and V
    are all-gathered in global column order and each rank forms its row
    block U_loc^T U (V_loc^T V) of the n x n Gram, minus the identity;
    the squared norms are summed over ranks (fp32 GEMMs, ~1e-6 relative)."""
    loc, glob = _global_columns(res, n, comm)
    A = gen(0, n).to(dtype)
    dev = A.device
    idx = torch.tensor(loc, device=res.U.device, dtype=torch.long)
    U = res.U[idx, :m].t().to(dev)
    V = res.V[idx, :n].t().to(dev)
    sig = res.S[idx].to(dev)
    gidx = torch.tensor(glob, device=dev, dtype=torch.long)
    # all-gather (global id, column) of every rank's U and V columns
    Ufull = torch.zeros(n, m, dtype=dtype, device=dev)
    Vfull = torch.zeros(n, n, dtype=dtype, device=dev)
    if comm.world == 1:  # no gather copies (65536^2: 17 GB per matrix)
        Ufull[gidx] = U.t()
        Vfull[gidx] = V.t()
    else:
        cnt = comm.allgather(torch.tensor([len(glob)], dtype=torch.int64, device=dev)).cpu().reshape(-1)
        mx = int(cnt.max())
        pad_u = torch.zeros(mx, m, dtype=dtype, device=dev)
        pad_v = torch.zeros(mx, n, dtype=dtype, device=dev)
        pad_g = torch.full((mx,), -1, dtype=torch.int64, device=dev)
        pad_u[:len(glob)], pad_v[:len(glob)], pad_g[:len(glob)] = U.t(), V.t(), gidx
        Uall, Vall, Gall = comm.allgather(pad_u), comm.allgather(pad_v), comm.allgather(pad_g)
        del pad_u, pad_v
        for h in range(comm.world):
            c = int(cnt[h])
            Ufull[Gall[h, :c]] = Uall[h, :c]
            Vfull[Gall[h, :c]] = Vall[h, :c]
        del Uall, Vall
    # Gram rows in column chunks (65536^2: a whole n x n Gram and its fp64
    # square would need ~100 GB next to A, U, V)
    ch = max(1, min(len(glob), (1 << 28) // max(n, 1)))
    sq = torch.zeros(3, dtype=torch.float64, device=dev)  # residual, V, U
    mxu = torch.zeros((), dtype=torch.float64, device=dev)
    mxv = torch.zeros((), dtype=torch.float64, device=dev)
    for c0 in range(0, len(glob), ch):
        c1 = min(len(glob), c0 + ch)
        eye_rows = torch.zeros(c1 - c0, n, dtype=dtype, device=dev)
        eye_rows[torch.arange(c1 - c0, device=dev), gidx[c0:c1]] = 1
        Rc = A @ V[:, c0:c1] - U[:, c0:c1] * sig[c0:c1]
        EV = V[:, c0:c1].t() @ Vfull.t() - eye_rows
        EU = U[:, c0:c1].t() @ Ufull.t() - eye_rows
        sq += torch.stack([Rc.double().pow(2).sum(), EV.double().pow(2).sum(),
                           EU.double().pow(2).sum()])
        mxu = torch.maximum(mxu, EU.abs().max().double())
        mxv = torch.maximum(mxv, EV.abs().max().double())
        del Rc, EV, EU, eye_rows
    a2 = sum(A[:, c0:c0 + 4096].double().pow(2).sum() for c0 in range(0, n, 4096))
    parts = torch.stack([sq[0], a2 / comm.world, sq[1], sq[2]])
    parts = comm.allreduce_sum_(parts.to(comm_device(comm, dev))).cpu()
    # largest single entry |u_i^T u_j - delta_ij|: the stop test bounds the
    # final couplings by tol (sqrt(m) eps), so the Frobenius norm grows ~ n tol
    mx = comm.allgather(torch.stack([mxu, mxv])).cpu().amax(0)
    return {"residual_rel": float((parts[0] / parts[1]).sqrt()),
            "orth_v_fro": float(parts[2].sqrt()), "orth_u_fro": float(parts[3].sqrt()),
            "orth_u_max_abs": float(mx[0]), "orth_v_max_abs": float(mx[1]),
            "orth_scope": "full n x n Gram (all-gathered)"}


def comm_device(comm, dev):
    """Device of the tensors the communicator reduces (host for gloo)."""
    return torch.device("cpu") if getattr(comm, "backend", "") == "gloo" else dev


def verify_rows(res, gen, m, n, comm, dtype):
    """QR-preconditioned (tall) result: U is this rank's row block, sigma and
    V are complete on every rank.  ||A V - U S||_F / ||A||_F over all row
    blocks, ||U^T U - I||_F (U^T U all-reduced) and ||V^T V - I||_F."""
    r0, r1 = res.info["u_rows"]
    A = torch.cat([gen(c0, min(c0 + 1024, n))[r0:r1] for c0 in range(0, n, 1024)], dim=1).to(dtype)
    U, S, V = res.U.to(dtype), res.S.to(dtype), res.V.to(dtype)
    eye = torch.eye(n, device=A.device, dtype=dtype)
    UtU = U.t() @ U
    parts = torch.stack([(A @ V - U * S).double().pow(2).sum(), A.double().pow(2).sum()])
    if comm.distributed:
        import torch.distributed as dist
        dist.all_reduce(parts)
        dist.all_reduce(UtU)
    parts = parts.cpu()
    return {"residual_rel": float((parts[0] / parts[1]).sqrt()),
            "orth_u_fro": float((UtU - eye).double().norm()),
            "orth_v_fro": float((V.t() @ V - eye).double().norm())}


class _ticker:
    """A stderr line every 30 s while a long silent call runs (the fp64
    oracle), so a job watchdog does not take the run for hung."""

    def __init__(self, what):
        self.what = what

    def __enter__(self):
        import threading
        self.t0, self.stop = time.time(), threading.Event()

        def run():
            while not self.stop.wait(30):
                print(f"[bench] {self.what}: {time.time() - self.t0:.0f} s", file=sys.stderr,
                      flush=True)
        self.th = threading.Thread(target=run, daemon=True)
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.th.join()


def sigma_check(res, gen, m, n, comm):  # noqa: C901
    """max |sigma - sigma_ref| / sigma_ref_max against an fp64 oracle
    (torch.linalg.svdvals of the regenerated A in fp64 on the device,
    rocSOLVER), after the timed region.  Every rank's sigma columns are
    all-gathered first (padding columns dropped)."""
    if res.info.get("distributed_output") is True:
        B = res.info["geometry"]["B"]
        ids = comm.allgather(torch.tensor(res.info["held"], device=res.S.device)).cpu()
        S_all = comm.allgather(res.S[:2 * B])
        sig = torch.zeros(2 * B * comm.world, dtype=torch.float64, device=res.S.device)
        for h in range(comm.world):
            for s_ in range(2):
                sb = int(ids[h, s_])
                sig[sb * B:(sb + 1) * B] = S_all[h, s_ * B:(s_ + 1) * B].double()
        sig = sig[:n]
    else:
        sig = res.S.double()
    if comm.rank != 0:
        return None
    A = gen(0, n).double()
    with _ticker(f"sigma oracle: fp64 svdvals of {m}x{n}"):  # minutes at n >= 8192
        ref = torch.linalg.svdvals(A)
        if ref.is_cuda:
            torch.cuda.synchronize()
    got = torch.sort(sig, descending=True).values
    return float((got - ref).abs().max() / ref[0])


def verify_root(res, A, dtype):
    """Rank 0, root-owned output: full ||A V - U S|| / ||A|| and orthogonality."""
    U, S, V = res.U.to(dtype), res.S.to(dtype), res.V.to(dtype)
    A = A.to(dtype)
    eye = torch.eye(S.shape[0], device=A.device, dtype=dtype)
    r = (A @ V - U * S).double().norm() / A.double().norm()
    return {"residual_rel": float(r),
            "orth_v_fro": float((V.t() @ V - eye).double().norm()),
            "orth_u_fro": float((U.t() @ U - eye).double().norm())}


def make_generator(m, dev, work, dtype):
    GB = 256  # generator block: the matrix is fixed regardless of how callers chunk it

    def gen(c0, c1):  # synthetic random dense U(0,1), columns c0..c1-1 of ONE fixed matrix
        parts = []
        for b0 in range(c0 // GB * GB, c1, GB):
            g = torch.Generator(device=dev).manual_seed(1234 + b0)
            blk = torch.rand(m, GB, generator=g, dtype=work, device=dev)
            parts.append(blk[:, max(c0 - b0, 0):min(c1 - b0, GB)])
        return torch.cat(parts, dim=1).to(dtype)

    return gen


def simulate(a, cfg, dtype, work):
    """Per-GPU time of rank g's plan in a P-GPU job, on one GPU."""
    import svdj
    from svdj.parallel import DistributedBlockJacobi, SimCommunicator

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    P, g = a.simulate_P, a.simulate_rank
    n = a.n
    m = a.m or n
    from svdj.models import precondition as pre
    m_it = n if pre.use_qr(cfg, m, n) else m  # rows of the matrix the sweeps run on
    gen = make_generator(m, dev, work, dtype)
    seed_gen = torch.Generator(device=dev).manual_seed(99)
    made = []

    def seed(pos, like):  # other ranks' super-block halves: [A half, D half, V half]
        if pos == 0:
            t = torch.zeros_like(like)
            t[:, :m_it] = torch.rand(like.shape[0], m_it, generator=seed_gen, device=dev,
                                     dtype=work).to(like.dtype)
            made.append(t)
            return t
        if pos == 1:  # squared norms of the matching A half
            return made.pop(0).double().pow(2).sum(1).to(like.dtype)
        return torch.zeros_like(like)

    comm = SimCommunicator(P, g, dev, seed_fn=seed, link_gbps=a.sim_link_gbps,
                           exchange=a.exchange)
    cfg.max_sweeps = a.sim_sweeps
    cfg.comm_timing = True
    solver = DistributedBlockJacobi(cfg, comm)

    def one():
        return solver.solve(None, m=m, n=n, dtype=dtype, generator=gen, gather=False)

    one()  # warmup (compiles nothing; allocates workspaces and the ring)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = one()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    geo = res.info["geometry"]
    line = {
        "metric": "simulated per-GPU time per sweep (rank plan of a P-GPU job on one GPU)",
        "value": round(el / res.sweeps * 1e3, 3), "unit": "ms/sweep", "higher_is_better": False,
        "simulated_P": P, "simulated_rank": g, "sweeps_run": res.sweeps,
        "solve_s": round(el, 4), "dtype": a.dtype,
        "config": {"model": f"{m}x{n} {a.dtype}", "block_W": geo["W"], "super_block_B": geo["B"],
                   "chains": a.chains, "inner_order": res.info.get("inner_order", a.inner_order),
                   "link_gbps_model": a.sim_link_gbps, "exchange": comm.exchange,
                   "quad_steps": bool(res.info.get("quad", False))},
        "comm": res.info.get("comm"),
        "qr_seconds": res.info.get("qr_seconds"),
        "sim_bytes_per_exchange": comm.bytes_moved // max(comm.exchanges, 1),
        "note": "exchanges swap with simulated peers (device copies of the real sizes); "
                "numerics are not those of the real job -- timing only",
    }
    print(json.dumps(line), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(line, f)


class _HostComm:
    """The gloo host group of --engine native (verification only: the solve
    itself talks RCCL from C++)."""

    backend = "gloo"

    def __init__(self, rank, world):
        self.rank, self.world = rank, world

    distributed = property(lambda self: self.world > 1)

    def allgather(self, t):
        if self.world == 1:
            return t.unsqueeze(0).clone()
        import torch.distributed as dist
        h = t.detach().cpu().contiguous()
        out = [torch.empty_like(h) for _ in range(self.world)]
        dist.all_gather(out, h)
        return torch.stack(out).to(t.device)

    def allreduce_sum_(self, t):
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(t)
        return t


def run_native(a, dtype, work):
    """--engine native: the C++ distributed solver (libsvdj_dist.so,
    csrc/dist/svdj_dist.cpp) inside the bench process -- the same tournament,
    half-exchange pipeline and block kernels as the Python executor, with the
    sweep issued from C++ (RCCL ncclSend/ncclRecv on its own comm stream,
    HIP events for every dependency).  torch.distributed runs on gloo here,
    for the host-side barriers and the max over ranks only."""
    import ctypes as C
    import datetime

    import torch.distributed as dist

    import svdj
    from svdj.ops import _native as NAT
    from svdj.ops import kernels as K
    from svdj.parallel.comm import default_timeout_s, env_world
    from svdj.utils.metrics import algorithmic_flops_per_sweep, default_tol
    from svdj.models.block import choose_mma

    rank, world, local = env_world()
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if dtype not in (torch.float32, torch.float64):
        raise SystemExit("--engine native: fp32 or fp64")
    shared = os.environ.get("SVDJ_SHARED_GPU") == "1"
    dev = torch.device("cuda", 0 if shared else local)
    torch.cuda.set_device(dev)
    # the solver's streams first: HIP binds streams to hardware queues in
    # creation order, RCCL creates its own at communicator init
    sa, sb, sc = (torch.cuda.Stream(dev) for _ in range(3))
    timeout = a.comm_timeout or default_timeout_s()
    if shared:
        os.environ["NCCL_HOSTID"] = f"svdj-shared-gpu-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=timeout))
    comm = _HostComm(rank, world)

    def barrier():
        if world > 1:
            dist.barrier()

    lib = NAT.dist_lib()

    def check(rc, what):
        if rc < 0:
            raise RuntimeError(f"{what}: {lib.svdj_dist_last_error().decode()}")

    def say(msg):
        if a.progress:
            print(f"[bench native rank {rank}] {msg}", file=sys.stderr, flush=True)

    id_path = f"/tmp/svdj_bench_{os.environ.get('MASTER_PORT', '0')}_{world}.id"
    if rank == 0 and os.path.exists(id_path):
        os.remove(id_path)
    barrier()
    nccl = C.c_void_p()
    say(f"RCCL init via {id_path}")
    check(lib.svdj_dist_comm_init(rank, world, id_path.encode(), float(timeout), C.byref(nccl)),
          "svdj_dist_comm_init")
    n = a.n
    m = a.m or n
    dcode = 1 if dtype == torch.float64 else 0
    W = a.block or lib.svdj_dist_choose_block(dcode, world, m, n)
    geo = [C.c_int32() for _ in range(4)]
    check(lib.svdj_dist_geometry(world, m, n, W, dcode, *[C.byref(g) for g in geo]), "svdj_dist_geometry")
    B, ncols, m_pad, n_v = (g.value for g in geo)
    held0 = (C.c_int32 * 2)()
    check(lib.svdj_dist_initial_held(world, rank, held0), "svdj_dist_initial_held")
    ncs = lib.svdj_dist_storage_cols(world, B)  # 2B + B of receive spares when P > 1
    At = torch.zeros(ncs, m_pad, dtype=dtype, device=dev)
    Vt = torch.zeros(ncs, n_v, dtype=dtype, device=dev)
    D = torch.zeros(ncs, dtype=dtype, device=dev)
    S = torch.empty(2 * B, dtype=dtype, device=dev)
    gen = make_generator(m, dev, work, dtype)
    hist = (C.c_double * a.max_sweeps)()
    p = NAT.DistProblem()
    p.rank, p.world, p.comm, p.dtype = rank, world, nccl, dcode
    p.W, p.m_pad, p.n_v, p.B = W, m_pad, n_v, B
    p.At, p.Vt, p.D = At.data_ptr(), Vt.data_ptr(), D.data_ptr()
    p.tol = a.tol if a.tol is not None else default_tol(dtype, m)
    mma = a.mma if a.mma != "auto" else choose_mma(dtype, W)
    p.tol_mode, p.max_sweeps, p.mma = 0, a.max_sweeps, K.mma_code(mma, dtype)
    p.inner_order = {"cyclic": 0, "bipartite": 1, "cross": 2, "auto": 3}[a.inner_order]
    p.stream_a, p.stream_b, p.stream_comm = sa.cuda_stream, sb.cuda_stream, sc.cuda_stream
    p.hist = C.cast(hist, C.POINTER(C.c_double))
    p.exchange = {"auto": 0, "direct": 1, "spread": 2}[a.exchange]
    p.timeout_s = float(timeout)
    p.comm_timing = 1 if a.comm_timing else 0
    p.progress = 1 if a.progress else 0
    p.stop_rule = K.STOP_RULES[a.stop_rule]
    p.quad = {"auto": 0, "on": 1, "off": 2}[a.quad]
    p.fault_rank, p.fault_sweep = -1, -1
    if a.inject_fault:
        p.fault_rank, p.fault_sweep = (int(x) for x in a.inject_fault.split(":"))
    hnd = C.c_void_p()  # persistent: workspaces, pair lists, events allocated once
    check(lib.svdj_dist_handle_create(C.byref(p), C.byref(hnd)), "svdj_dist_handle_create")
    p.handle = hnd

    def one():  # input generation (this rank's columns), V = I, norms, sweeps, U / sigma
        with torch.cuda.stream(sa):
            At.zero_()
            for s_ in range(2):
                c0 = held0[s_] * B
                c1 = min(c0 + B, n)
                if c1 > c0:
                    At[s_ * B:s_ * B + (c1 - c0), :m] = gen(c0, c1).t()
                K.set_identity(Vt[s_ * B:(s_ + 1) * B], B, c0)
            K.col_norms2(At, m_pad, out=D)
        p.held[0], p.held[1] = held0[0], held0[1]
        say(f"solve (W={W}, B={B}, m_pad={m_pad}, n_v={n_v})")
        rc = lib.svdj_dist_solve(C.byref(p), C.c_void_p(S.data_ptr()))
        if rc == -300:  # watchdog: a peer died or hung; the communicator is aborted
            print(f"[bench native rank {rank}] {lib.svdj_dist_last_error().decode()}",
                  file=sys.stderr, flush=True)
            os._exit(3)
        check(rc, "svdj_dist_solve")
        return p.sweeps, int(p.converged)

    for _ in range(a.warmup):
        one()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sweeps, conv, reasons = [], True, set()
    for _ in range(a.steps):
        sw, cv = one()
        sweeps.append(sw)
        conv = conv and cv > 0
        reasons.add({1: "no_rotation", 2: "second_order"}.get(cv, "not_converged"))
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
    flops = sum(algorithmic_flops_per_sweep(m, n) * s_ for s_ in sweeps)
    acc = None
    if not a.no_verify:
        class _Res:
            pass
        res = _Res()
        res.U, res.V, res.S = At, Vt, S
        res.info = {"geometry": {"B": B}, "held": [int(p.held[0]), int(p.held[1])],
                    "distributed_output": True}
        acc = verify_distributed(res, gen, m, n, comm, work)
        if want_sigma(a, n):
            err = sigma_check(res, gen, m, n, comm)
            if rank == 0:
                acc["sigma_max_rel_err_vs_fp64_oracle"] = err
    if rank == 0:
        ms = el / a.steps * 1e3
        line = {
            "metric": BASELINE_METRIC, "value": round(flops / el / 1e9, 2), "unit": "GFLOP/s",
            "n_gpus": a.gpus, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": a.dtype,
            "data": "synthetic random dense U(0,1), seeded per column block; generated on the fly per rank",
            "config": {"model": f"{m}x{n} {a.dtype} block one-sided Jacobi SVD (AllVec), to convergence",
                       "global_batch": 1, "seq_len": n,
                       "parallelism": f"colblock{a.gpus} (2 super-blocks/GPU, RCCL tournament)",
                       "engine": "native C++ (libsvdj_dist)", "block_W": W, "super_block_B": B,
                       "mma": mma, "mma_numerics": MMA_NUMERICS.get(mma, ""),
                       "precondition": "none", "chains": 2,
                       "inner_order": {0: "cyclic", 1: "bipartite", 2: "cross"}.get(
                           int(p.inner_order_used), a.inner_order),
                       "exchange": {1: "direct", 2: "spread"}.get(int(p.exchange_used), "direct"),
                       "root_owned": False,
                       "quad_steps": bool(p.quad_used), "merged_chains": bool(p.merged_used),
                       "stop_rule": a.stop_rule},
            "sweeps": sweeps, "converged": conv, "stop_reason": sorted(reasons),
            "time_to_converge_s": round(ms / 1e3, 4),
            "off_history_last": [float("%.3e" % hist[i]) for i in range(max(0, p.sweeps - 3), p.sweeps)],
            "comm": ({"exchanges": int(p.exchanges), "bytes_sent": int(p.bytes_sent),
                      "timing": bool(a.comm_timing),
                      **({"exchange_choice": (
                          f"measured at handle creation: direct {p.calib_direct_ms:.3f} ms, spread "
                          f"{p.calib_spread_ms:.3f} ms per half exchange -> "
                          f"{'spread' if int(p.exchange_used) == 2 else 'direct'}")}
                         if p.calib_direct_ms > 0 else {}),
                      **({"comm_ms": round(p.comm_ms, 3), "exposed_comm_ms": round(p.exposed_comm_ms, 3)}
                         if a.comm_timing else {})} if world > 1 else None),
            "world": world, "rccl_ranks": world,
            "accuracy": acc,
        }
        print(json.dumps(line), flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                json.dump(line, f)
    lib.svdj_dist_handle_destroy(hnd)
    lib.svdj_dist_comm_destroy(nccl)
    if world > 1:
        dist.destroy_process_group()


def work_estimate(counts, m_pad, seconds):
    """Executed matrix-core work and HBM traffic of the quad kernels per
    solve, next to the algorithmic GFLOP/s (the headline is the
    reference's scalar-Jacobi flop count, which is not what the MFMAs
    execute).  counts = [apply MFMAs, apply tiles, quad Grams, of which on 2
    bf16 parts] summed over ranks: one v_mfma_f32_32x32x16_bf16 = 32768 flops;
    an apply tile is 32 rows x 256 columns of A or V read and written (64 KiB);
    a quad Gram reads 256 columns of m_pad rows and issues 288 MFMAs (in
    32x32x16 units) per 32-row slab, 144 on 2 parts.  Averaged
    over the whole time to converge, so these are lower bounds on the quad
    kernels' own rates (the EVD chain and the single steps that open each
    sweep are in the time but not in the counts)."""
    mf_apply, tiles, gq, gq2 = counts
    mf_gram = (gq - gq2) * (m_pad / 32.0) * 288.0 + gq2 * (m_pad / 32.0) * 144.0
    flops = (mf_apply + mf_gram) * 32768.0
    nbytes = tiles * 65536.0 + gq * m_pad * 256.0 * 4.0
    if seconds <= 0 or flops <= 0:
        return None
    return {"basis": "quad-step kernels only (split-bf16 apply + quad Gram), device-counted; "
                     "per solve, averaged over the time to converge",
            "mfma_bf16_tflop_per_solve": round(flops / 1e12, 3),
            "executed_mfma_tflops": round(flops / seconds / 1e12, 1),
            "hbm_gb_per_solve": round(nbytes / 1e9, 1),
            "hbm_tb_per_s": round(nbytes / seconds / 1e12, 3),
            "apply_mfma": int(mf_apply), "apply_tiles": int(tiles), "quad_grams": int(gq),
            "quad_grams_2part": int(gq2)}


def want_sigma(a, n) -> bool:
    """sigma vs the fp64 oracle: by default whenever n <= 8192 (rocSOLVER
    svdvals of the regenerated A in fp64, after timing); --check-sigma forces
    it, --no-sigma-check skips it."""
    if a.no_sigma_check:
        return False
    return bool(a.check_sigma) or n <= 8192


def svdj_default_inner() -> str:
    import svdj
    return svdj.SolverConfig().inner_order


def main():
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--n", "--size", dest="n", type=int, default=16384)
    p.add_argument("--m", type=int, default=None)
    p.add_argument("--dtype", default="fp32", choices=["fp32", "fp64", "bf16"])
    p.add_argument("--precondition", default="auto", choices=["none", "qr", "auto"],
                   help="QR-precondition tall inputs (m >= 2n); flops then count QR + GEMM")
    p.add_argument("--block", type=int, default=None)
    p.add_argument("--max-sweeps", type=int, default=60)
    p.add_argument("--inner", type=int, default=1)
    p.add_argument("--tol", type=float, default=None,
                   help="rotation threshold (default sqrt(m) eps of the problem dtype)")
    p.add_argument("--chains", type=int, default=2, choices=[1, 2])
    p.add_argument("--inner-order", default=svdj_default_inner(),
                   choices=["auto", "cyclic", "bipartite", "cross"],
                   help="EVD ordering of the block cross steps")
    p.add_argument("--mma", default="auto", choices=["auto", "native", "bf16x6", "bf16x3"],
                   help="block apply matrix cores (auto = bf16x6 for fp32 W=64 steps, f32/f64 "
                        "MFMA otherwise; bf16x6 = 3-way bf16 split at fp32 accuracy, bf16x3 = "
                        "2-way split, ~2^-17)")
    p.add_argument("--root-owned", action="store_true",
                   help="A on rank 0 before timing; scatter + gather of U,S,V timed")
    p.add_argument("--progress", action="store_true", help="one line per sweep on stderr")
    p.add_argument("--comm-timeout", type=float, default=None,
                   help="communication timeout in s: a peer that stops answering ends the "
                        "job non-zero after this long (default SVDJ_COMM_TIMEOUT or 300)")
    p.add_argument("--comm-timing", action="store_true",
                   help="bracket every exchange and task with timing events and report "
                        "comm_ms / exposed_comm_ms (adds events; off for headline runs)")
    p.add_argument("--inject-fault", default=None, metavar="RANK:SWEEP",
                   help="failure-detection test: that rank exits abruptly after that sweep")
    p.add_argument("--exchange", default="auto", choices=["auto", "direct", "spread"],
                   help="half super-block transfer: one link (direct) or all links, relayed "
                        "(spread); auto = spread from 4 GPUs")
    p.add_argument("--quad", default="auto", choices=["auto", "on", "off"],
                   help="fused two-step quad block steps (fp32 W=64 split-bf16; auto: off)")
    p.add_argument("--stop-rule", default="second_order", choices=["second_order", "no_rotation"],
                   help="also end after a sweep of noise-level rotations (second_order, "
                        "csrc/include/svdj_stop.h) or only after a sweep without rotations")
    p.add_argument("--simulate-P", type=int, default=0)
    p.add_argument("--simulate-rank", type=int, default=0)
    p.add_argument("--sim-sweeps", type=int, default=3)
    p.add_argument("--sim-link-gbps", type=float, default=0.0,
                   help="model each exchange's link time at this GB/s (0: device copy only)")
    p.add_argument("--engine", default="python", choices=["python", "native"],
                   help="distributed executor: torch.distributed + Python issue (python), or "
                        "the C++ solver libsvdj_dist with RCCL called directly (native)")
    p.add_argument("--json-out", default=None)
    p.add_argument("--no-verify", action="store_true",
                   help="skip the post-timing accuracy check")
    p.add_argument("--check-sigma", action="store_true",
                   help="compare sigma with an fp64 oracle (svdvals) even when n > 8192")
    p.add_argument("--no-sigma-check", action="store_true",
                   help="skip the sigma check that runs by default for n <= 8192")
    a = p.parse_args()

    import svdj
    from svdj.parallel import Communicator, DistributedBlockJacobi

    dtype = {"fp32": torch.float32, "fp64": torch.float64, "bf16": torch.bfloat16}[a.dtype]
    work = torch.float64 if dtype == torch.float64 else torch.float32
    cfg = svdj.SolverConfig(dtype=dtype, block=a.block, max_sweeps=a.max_sweeps, tol=a.tol,
                            max_inner_sweeps=a.inner, chains=a.chains, mma=a.mma,
                            precondition=a.precondition,
                            inner_order=a.inner_order,
                            progress=a.progress, comm_timing=a.comm_timing, exchange=a.exchange,
                            quad=a.quad, stop_rule=a.stop_rule)
    if a.inject_fault:
        r_, s_ = (int(x) for x in a.inject_fault.split(":"))
        cfg.extra["fault_exit"] = (r_, s_)
    if a.comm_timeout is None:
        a.comm_timeout = float(os.environ.get("SVDJ_COMM_TIMEOUT", "300"))
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    if a.simulate_P:
        simulate(a, cfg, dtype, work)
        return
    if a.engine == "native":
        run_native(a, dtype, work)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 with "
                         "torch.distributed.run --nproc-per-node N")
    comm = Communicator(timeout_s=a.comm_timeout)
    solver = DistributedBlockJacobi(cfg, comm)
    dev = comm.device
    from svdj.parallel.schedule import tournament
    tour = tournament(comm.world)
    partners = set(tour.send_to[:, comm.rank].tolist()) | set(tour.recv_from[:, comm.rank].tolist())
    ready = comm.readiness(partners)
    if comm.rank == 0 and comm.distributed:
        print(f"[bench] world {ready['world']} over {ready.get('rccl_ranks')} RCCL ranks, devices "
              f"{ready.get('devices')}, P2P to tournament partners {ready.get('p2p_partners')}",
              file=sys.stderr, flush=True)
    n = a.n
    m = a.m or n
    gen = make_generator(m, dev, work, dtype)

    A_root = None
    if a.root_owned and comm.rank == 0:
        A_root = gen(0, n)

    def one():
        if a.root_owned:
            return solver.solve(A_root if comm.rank == 0 else None, gather=True)
        return solver.solve(None, m=m, n=n, dtype=dtype, generator=gen, gather=False)

    for _ in range(a.warmup):
        one()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # Only the last solve's outputs are kept (earlier ones are released as the
    # next solve starts); sweeps / convergence / flops are accumulated as scalars.
    sweeps, conv, flops, last, reasons = [], True, 0.0, None, set()
    for _ in range(a.steps):
        last = None
        last = one()
        sweeps.append(last.sweeps)
        conv = conv and last.converged
        reasons.add(last.info.get("stop_reason") or "not_converged")
        flops += last.info["flops"]
    comm.barrier()
    torch.cuda.synchronize()
    elapsed = comm.max_over_ranks(time.perf_counter() - t0)

    gflops = flops / elapsed / 1e9
    ms = elapsed / a.steps * 1e3
    geo = last.info["geometry"]
    acc = None
    if not a.no_verify:
        if a.root_owned:
            acc = verify_root(last, A_root, work) if comm.rank == 0 else None
        elif last.info.get("precondition") == "qr":
            acc = verify_rows(last, gen, m, n, comm, work)
        else:
            acc = verify_distributed(last, gen, m, n, comm, work)
    # sigma vs the fp64 oracle; on the QR path sigma is complete on every rank
    # (the oracle is svdvals of the whole m x n A)
    if not a.no_verify and want_sigma(a, n):
        if a.root_owned:
            err = None
            if comm.rank == 0:
                ref = torch.linalg.svdvals(A_root.double())
                got = torch.sort(last.S.double(), descending=True).values
                err = float((got - ref).abs().max() / ref[0])
        else:
            err = sigma_check(last, gen, m, n, comm)
        if comm.rank == 0:
            acc = dict(acc or {}, sigma_max_rel_err_vs_fp64_oracle=err)
    # work the quad kernels actually did in the last solve, summed over ranks
    # (apply MFMAs and tiles counted on the device, quad Grams on the host)
    wk = last.info.get("work") or {}
    wt = torch.tensor([float(wk.get("apply_mfma", 0)), float(wk.get("apply_tiles", 0)),
                       float(wk.get("gram_quads", 0)), float(wk.get("gram_quads2", 0))],
                      dtype=torch.float64, device=comm.device)
    comm.allreduce_sum_(wt)
    work_est = work_estimate(wt.cpu().tolist(), int(wk.get("m_pad", m)), ms / 1e3)
    if comm.rank == 0:
        line = {
            "metric": BASELINE_METRIC,
            "value": round(gflops, 2),
            "unit": "GFLOP/s",
            "n_gpus": a.gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": "synthetic random dense U(0,1), seeded per column block" +
                    ("; root-owned A, scatter+gather timed" if a.root_owned
                     else "; generated on the fly per rank"),
            "config": {
                "model": f"{m}x{n} {a.dtype} block one-sided Jacobi SVD (AllVec), to convergence",
                "global_batch": 1,
                "seq_len": n,
                "parallelism": f"colblock{a.gpus} (2 super-blocks/GPU, RCCL tournament)",
                "block_W": geo["W"],
                "super_block_B": geo["B"],
                "mma": last.info.get("mma", a.mma),
                "mma_numerics": MMA_NUMERICS.get(last.info.get("mma", a.mma), ""),
                "precondition": last.info.get("precondition", "none"),
                "chains": a.chains,
                "inner_order": last.info.get("inner_order", a.inner_order),
                "root_owned": a.root_owned,
                "exchange": last.info.get("exchange", a.exchange),
                "quad_steps": bool(last.info.get("quad", False)),
                "merged_chains": bool(last.info.get("merged_chains", False)),
                "stop_rule": a.stop_rule,
            },
            "sweeps": sweeps,
            "converged": conv,
            "stop_reason": sorted(reasons),
            "time_to_converge_s": round(ms / 1e3, 4),
            "off_history_last": [float("%.3e" % h) for h in last.history[-3:]],
            "comm": last.info.get("comm"),
            "world": ready.get("world"), "devices": ready.get("devices"),
            "rccl_ranks": ready.get("rccl_ranks"), "p2p_partners": ready.get("p2p_partners"),
            "accuracy": acc,
            "work_estimate": work_est,
        }
        print(json.dumps(line), flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                json.dump(line, f)
    comm.destroy()


if __name__ == "__main__":
    main()
