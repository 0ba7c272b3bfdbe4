"""Multi-process distributed block Jacobi on CPU (gloo), world 1..4 and 8."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, m, n, W, tmp_path, mode="root"):
    out = tmp_path / f"res_{world}_{mode}.json"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "_dist_worker.py"), str(m), str(n), str(W), str(out), mode]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return json.loads(out.read_text())


@pytest.mark.parametrize("world,m,n", [(1, 140, 128), (2, 160, 128), (3, 200, 190), (4, 300, 256),
                                        (8, 200, 192)])
def test_distributed_block_jacobi_gloo(world, m, n, tmp_path):
    rep = _run(world, m, n, 32, tmp_path)
    assert rep["converged"] and rep["world"] == world
    assert rep["residual_rel"] < 1e-12, rep
    assert rep["sigma_max_abs_err_over_smax"] < 1e-12, rep
    assert rep["orth_u_fro"] < 1e-10 and rep["orth_v_fro"] < 1e-10, rep


def test_distributed_generator_input(tmp_path):
    rep = _run(2, 150, 128, 32, tmp_path, mode="gen")
    assert rep["converged"] and rep["residual_rel"] < 1e-12, rep


@pytest.mark.parametrize("mode", ["rootqr", "genqr"])
def test_distributed_qr_preconditioned(mode, tmp_path):
    rep = _run(2, 300, 128, 32, tmp_path, mode=mode)
    assert rep["converged"] and rep["residual_rel"] < 1e-12, rep
    assert rep["orth_u_fro"] < 1e-10 and rep["sigma_max_abs_err_over_smax"] < 1e-12, rep


@pytest.mark.parametrize("world", [2, 3])
def test_ordered_sum_slabs_are_bitwise_whole(world, tmp_path):
    """the rank-ordered Gram sum of the distributed QR gathers in
    slabs of bounded size; the additions per element are unchanged, so the
    slabbed sum is the same bits as the whole one and as rank-order adds."""
    rep = _run(world, 10, 10, 32, tmp_path, mode="ordsum")
    assert rep["slab_eq_whole"] and rep["whole_eq_ref"] and rep["slab_t_eq"], rep


def test_svd_inside_distributed_job_is_local(tmp_path):
    """svd() on a rank of a running job solves that rank's own matrix on a
    world-1 Communicator.local (it must not join the job's process group)."""
    rep = _run(2, 150, 128, 32, tmp_path, mode="localsvd")
    assert rep["engine"] == "pipeline" and rep["converged"], rep
    assert rep["max_err"] < 1e-12, rep


@pytest.mark.parametrize("world", [2, 3])
def test_local_matrix_distribution_roundtrip(world, tmp_path):
    """Scatter root-owned A to the resident super-blocks and gather it back."""
    rep = _run(world, 130, 100, 32, tmp_path, mode="roundtrip")
    assert rep["max_err"] == 0.0 and rep["world"] == world


@pytest.mark.parametrize("world", [2, 4])
def test_isend_irecv_ring(world, tmp_path):
    rep = _run(world, 8, 8, 32, tmp_path, mode="isend")
    assert rep["ok_ranks"] == world


@pytest.mark.parametrize("world,m,n", [(4, 300, 256), (5, 340, 320)])
def test_spread_exchange_matches_direct(world, m, n, tmp_path):
    """parallel/spread.py: every half relayed over all links in two phases
    delivers exactly the direct exchange's data, so the solves are bitwise
    equal (and the relays really carried bytes)."""
    rep = _run(world, m, n, 32, tmp_path, mode="exchcmp")
    assert rep["exchange"] == ["direct", "spread"] and rep["relayed"] > 0, rep
    assert rep["u_diff"] == 0.0 and rep["s_diff"] == 0.0 and rep["v_diff"] == 0.0, rep
    assert rep["sweeps"][0] == rep["sweeps"][1]
    # exchanges are counted with timing off: per sweep
    # every rank sends each of its two halves once per round after round 0
    assert rep["timing"] == [False, False] and rep["comm_ms_absent"], rep
    per_sweep = 2 * (2 * world - 2)
    assert rep["exchanges"][0] == rep["exchanges"][1] == per_sweep * rep["sweeps"][0], rep


@pytest.mark.parametrize("world", [4, 5])
def test_exchange_calibration_agrees_across_ranks(world, tmp_path):
    """pipeline.calibrate_exchange (exchange auto on RCCL from 4 GPUs) over
    gloo: both exchange variants of the first tournament round run to
    completion (no op mismatch in the relayed phases) and every rank
    reaches the same decision."""
    rep = _run(world, 0, 0, 0, tmp_path, mode="calib")
    assert rep["world"] == world and rep["agree"], rep
    assert rep["choice"] in ("direct", "spread") and rep["summary"].startswith("measured"), rep


def test_spread_ops_deliver_every_chunk_once():
    """Simulate the two phases of spread_ops for every rank of every
    tournament round at P = 3..8: each directed pair's sends and receives
    match one to one in order and size, relays forward what they received,
    and every rank ends with exactly the message its sender sent."""
    import numpy as np

    from svdj.parallel.schedule import tournament
    from svdj.parallel.spread import spread_ops

    for P in range(3, 9):
        tour = tournament(P)
        sizes, flags = [37, 5, 23], [True, False, True]
        for r in range(1, tour.rounds):
            send_to = [int(x) for x in tour.send_to[r]]
            ops = [spread_ops(g, send_to, sizes, flags) for g in range(P)]
            out = {g: [np.arange(n) + 1000 * g + 100 * mi for mi, n in enumerate(sizes)]
                   for g in range(P)}
            inc = {g: [np.full(n, -1) for n in sizes] for g in range(P)}
            relay = {g: {} for g in range(P)}

            def run(phase):
                sends = {}
                for g in range(P):
                    for mi, (a, b), peer, where in getattr(ops[g], f"p{phase}_send"):
                        data = out[g][mi][a:b] if where == "out" else relay[g][(mi, where[1])]
                        sends.setdefault((g, peer), []).append((mi, data.copy()))
                for g in range(P):
                    recvd = {}
                    for mi, (a, b), peer, where in getattr(ops[g], f"p{phase}_recv"):
                        q = sends[(peer, g)]
                        i = recvd.get(peer, 0)
                        recvd[peer] = i + 1
                        smi, data = q[i]
                        assert smi == mi and len(data) == b - a
                        if where == "in":
                            inc[g][mi][a:b] = data
                        else:
                            relay[g][(mi, where[1])] = data
                    for peer, cnt in recvd.items():
                        assert cnt == len(sends[(peer, g)])

            run(1)
            run(2)
            for g in range(P):
                src = send_to.index(g)
                for mi in range(3):
                    assert (inc[g][mi] == out[src][mi]).all(), (P, r, g, mi)


def test_svd_on_the_fly_api(tmp_path):
    rep = _run(2, 170, 128, 32, tmp_path, mode="otf")
    assert rep["converged"] and rep["residual_rel"] < 1e-12, rep


def test_simulated_rank_plan_cpu():
    """SimCommunicator: one process runs rank g's plan of a P-rank job; every
    exchange swaps real-sized halves with simulated peers."""
    import torch

    import svdj
    from svdj.parallel import DistributedBlockJacobi, SimCommunicator

    P, g, n = 4, 1, 256
    A = svdj.utils.inputs.random_dense(n, n, dtype=torch.float64, seed=3)

    def seed(pos, like):
        return torch.rand(like.shape, dtype=like.dtype) if pos != 1 else torch.ones_like(like)

    comm = SimCommunicator(P, g, torch.device("cpu"), seed_fn=seed)
    cfg = svdj.SolverConfig(block=32, dtype=torch.float64, max_sweeps=2)
    res = DistributedBlockJacobi(cfg, comm).solve(None, m=n, n=n, dtype=torch.float64,
                                                  generator=lambda c0, c1: A[:, c0:c1],
                                                  gather=False)
    assert res.sweeps == 2
    # 2P-2 exchanges per sweep, each split in two halves
    assert comm.exchanges == 2 * 2 * (2 * P - 2)
    geo = res.info["geometry"]
    half = geo["B"] // 2
    assert comm.bytes_moved == comm.exchanges * half * 8 * (geo["m_pad"] + 1 + geo["n_v"])


@pytest.mark.parametrize("world", [2, 4])
def test_row_distributed_cholqr2(world, tmp_path):
    """Tall-skinny: row-distributed CholeskyQR2 (local Gram + all-reduce,
    replicated Cholesky, local TRSM), Jacobi on the replicated R, U = Q U_R
    per row block; checked globally (all-reduced) on every rank's rows."""
    rep = _run(world, 400, 96, 32, tmp_path, mode="genqr_rows")
    assert rep["converged"] and rep["world"] == world
    assert rep["residual_rel"] < 1e-12 and rep["orth_u_fro"] < 1e-10, rep
    assert rep["orth_v_fro"] < 1e-10 and rep["sigma_err"] < 1e-12, rep


def test_dead_peer_fails_survivor_fast(tmp_path):
    """Failure detection, Python engine: rank 1 exits
    abruptly after sweep 1 (SolverConfig.extra fault_exit, like a crashed
    peer).  The ranks are started directly, not by torchrun (whose agent
    would kill the survivor itself): rank 0 must exit non-zero on its own,
    well within the communicator timeout, instead of hanging."""
    import time
    port = _free_port()
    out = tmp_path / "fault.json"
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(os.environ, OMP_NUM_THREADS="1", RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   SVDJ_TEST_TIMEOUT="60")
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(HERE, "_dist_worker.py"), "200", "192", "32", str(out),
             "fault"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    try:
        outs = [p.communicate(timeout=180) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    el = time.time() - t0
    assert procs[1].returncode == 17, outs[1][1][-2000:]
    assert procs[0].returncode not in (0, None), outs[0][1][-2000:]
    assert el < 120, el
    assert not out.exists()
