"""Sweep-level checkpoint / resume (CPU, single rank)."""
import torch

import svdj
from svdj.parallel import Communicator, DistributedBlockJacobi


def test_checkpoint_resume_matches_uninterrupted(tmp_path):
    A = svdj.utils.inputs.random_dense(96, 64, dtype=torch.float64, seed=21)
    comm = Communicator(backend="gloo", device=torch.device("cpu"), init=False)
    ref = DistributedBlockJacobi(svdj.SolverConfig(block=32), comm).solve(A)
    # interrupted run: stop after 3 sweeps, checkpoint every sweep
    cfg = svdj.SolverConfig(block=32, max_sweeps=3, checkpoint_dir=str(tmp_path),
                            checkpoint_every=1)
    part = DistributedBlockJacobi(cfg, comm).solve(A)
    assert part.sweeps == 3 and not part.converged
    assert (tmp_path / "svdj_ckpt_rank0.pt").exists()
    cfg2 = svdj.SolverConfig(block=32, checkpoint_dir=str(tmp_path), checkpoint_every=1)
    res = DistributedBlockJacobi(cfg2, comm).solve(A)
    assert res.converged and res.sweeps == ref.sweeps
    assert res.history[:3] == part.history
    torch.testing.assert_close(res.S, ref.S, rtol=0, atol=0)
    assert not (tmp_path / "svdj_ckpt_rank0.pt").exists()


def test_tracing_and_reports(tmp_path):
    from svdj.utils import report, tracing

    with tracing.trace_range("unit"):
        tracing.mark("m")
    pt = tracing.PhaseTimer("cpu")
    with pt.phase("x"):
        sum(range(1000))
    assert "x" in pt.summary()
    A = svdj.utils.inputs.random_dense(40, 32, seed=1)
    res = svdj.svd(A)
    acc = svdj.utils.metrics.verify(A, res.U, res.S, res.V)
    rec = report.run_record(res, 40, 32, 0, acc)
    p = report.write_json(str(tmp_path / "r.json"), rec)
    assert p.endswith("r.json") and rec["sweeps"] == res.sweeps
    txt = report.write_reference_report(str(tmp_path), 40, 32, res.seconds, acc["residual_fro"], 1)
    body = open(txt).read()
    assert "SVD MPI+OMP time with U,V calculation:" in body and "||A-USVt||_F:" in body
    assert "reporte-dimension-40-time-" in txt
