"""GPU end-to-end: native driver, CLI driver, distributed solver at world 1,
determinism, checkpoint on device (needs MI355X)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_driver_block_and_scalar(tmp_path):
    exe = os.path.join(ROOT, "svd-jacobi-mpi-cuda_amd", "bin", "svdj_main")
    if not os.path.exists(exe):
        import svdj  # noqa: F401
        import importlib
        importlib.import_module("svd-jacobi-mpi-cuda_amd._build").build_driver()
    for method in ("block", "scalar"):
        r = subprocess.run([exe, "256", "--input", "dense", "--method", method, "--verify",
                            "--report-dir", str(tmp_path)], capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        out = r.stdout
        assert "SVD MPI+OMP time with U,V calculation" in out
        resid = float(out.split("||A-USVt||_F:")[1].split()[0])
        orth = float(out.split("||U^TU-I||_F:")[1].split()[0])
        assert resid < 1e-9 and orth < 1e-9, out
    assert any(p.name.startswith("reporte-dimension-256") for p in tmp_path.iterdir())


def test_native_driver_engines_agree(tmp_path):
    """svdj_main's block engines: the default pipeline (libsvdj_dist's plan at
    world 1, no RCCL communicator: the engine bench.py and svd() run) and the
    single-stream round robin both verify, in fp32 with W = 64 (split-bf16
    apply) and fp64, at a size where a chain step holds several pairs."""
    exe = os.path.join(ROOT, "svd-jacobi-mpi-cuda_amd", "bin", "svdj_main")
    for dt, lim in (("f32", 2e-4), ("f64", 1e-9)):
        for eng in ("pipeline", "steps"):
            r = subprocess.run([exe, "1100", "--m", "1200", "--input", "dense", "--dtype", dt,
                                "--engine", eng, "--verify", "--no-report"],
                               capture_output=True, text=True, timeout=300)
            assert r.returncode == 0, r.stdout + r.stderr
            out = r.stdout
            assert ("engine: pipeline" in out) == (eng == "pipeline"), out
            resid = float(out.split("||A-USVt||_F:")[1].split()[0])
            anorm = 1200 * 1100 / 3.0  # ||U(0,1)||_F^2 ~ mn / 3
            assert resid / anorm ** 0.5 < lim, out


def test_cli_driver_gpu(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "svd_jacobi.py"), "200",
                        "--input", "dense", "--verify", "--report-dir", str(tmp_path),
                        "--json", str(tmp_path / "r.json")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "converged: True" in r.stdout
    assert (tmp_path / "r.json").exists()


def test_distributed_world1_gpu_matches_svdvals(svdj, cuda):
    from svdj.parallel import Communicator, DistributedBlockJacobi

    comm = Communicator(device=cuda, init=False)
    A = svdj.utils.inputs.random_dense(700, 512, dtype=torch.float64, seed=4).to(cuda)
    res = DistributedBlockJacobi(svdj.SolverConfig(dtype=torch.float32, block=32), comm).solve(A)
    rep = svdj.utils.metrics.verify(A, res.U, res.S, res.V, torch.linalg.svdvals(A.cpu()))
    # measured ~1.4e-7 / ~5e-5 / ~4e-4 at this size (tools/measure_test_accuracy.py)
    assert res.converged and rep["sigma_max_abs_err_over_smax"] < 1e-6, rep
    assert rep["orth_v_fro"] < 3e-4 and rep["orth_u_fro"] < 2e-3, rep


def test_block_solver_deterministic(svdj, cuda):
    A = svdj.utils.inputs.random_dense(512, 512, dtype=torch.float32, device=cuda, seed=5)
    r1 = svdj.svd(A, method="block")
    r2 = svdj.svd(A, method="block")
    assert r1.sweeps == r2.sweeps
    assert torch.equal(r1.S, r2.S) and torch.equal(r1.U, r2.U) and torch.equal(r1.V, r2.V)


def test_checkpoint_resume_gpu(svdj, cuda, tmp_path):
    from svdj.parallel import Communicator, DistributedBlockJacobi

    comm = Communicator(device=cuda, init=False)
    A = svdj.utils.inputs.random_dense(256, 256, dtype=torch.float32, device=cuda, seed=6)
    ref = DistributedBlockJacobi(svdj.SolverConfig(block=32), comm).solve(A)
    DistributedBlockJacobi(svdj.SolverConfig(block=32, max_sweeps=2, checkpoint_dir=str(tmp_path),
                                              checkpoint_every=1), comm).solve(A)
    res = DistributedBlockJacobi(svdj.SolverConfig(block=32, checkpoint_dir=str(tmp_path),
                                                   checkpoint_every=1), comm).solve(A)
    assert res.sweeps == ref.sweeps and torch.equal(res.S, ref.S)


def test_tall_skinny_bf16_qr_gpu(svdj, cuda):
    """Config-4 shape class on one GPU: tall bf16 input, QR preconditioning,
    fp32 working copies, bf16 matrix cores (bf16x3) for the apply."""
    A = svdj.utils.inputs.random_dense(2048, 512, dtype=torch.float32, device=cuda,
                                       seed=14).to(torch.bfloat16)
    res = svdj.svd(A, method="block", precondition="qr")
    assert res.converged and res.info["precondition"] == "qr" and res.info["mma"] == "bf16x3"
    assert res.U.dtype == torch.bfloat16 and res.U.shape == (2048, 512)
    rep = svdj.utils.metrics.verify(A.double(), res.U, res.S, res.V,
                                    torch.linalg.svdvals(A.double().cpu()))
    assert rep["sigma_max_abs_err_over_smax"] < 1e-4, rep
    assert rep["residual_rel"] < 2e-2, rep


def test_qr_preconditioned_fp32_gpu(svdj, cuda):
    A = svdj.utils.inputs.random_dense(3000, 640, dtype=torch.float32, device=cuda, seed=15)
    res = svdj.svd(A, method="block", precondition="qr")
    plain = svdj.svd(A, method="block", precondition="none")
    ref = torch.linalg.svdvals(A.double().cpu())
    for r in (res, plain):
        rep = svdj.utils.metrics.verify(A, r.U, r.S, r.V, ref)
        assert r.converged and rep["residual_rel"] < 1e-4 and rep["sigma_max_abs_err_over_smax"] < 1e-5, rep


def test_bench_native_engine_matches_python_engine(tmp_path):
    """bench.py --engine native (libsvdj_dist in the bench process, RCCL
    world 1) runs the same solve as the Python executor: same sweeps, same
    accuracy figures, bench JSON contract fields present."""
    out = {}
    for eng in ("native", "python"):
        js = tmp_path / f"{eng}.json"
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--engine", eng,
                            "--size", "1024", "--steps", "1", "--warmup", "0", "--json-out", str(js)],
                           capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, MASTER_PORT=str(29950 + len(out))))
        assert r.returncode == 0, r.stderr[-2000:]
        out[eng] = json.loads(js.read_text())
    nat, py = out["native"], out["python"]
    for k in ("metric", "value", "unit", "n_gpus", "ms_per_step", "config", "sweeps"):
        assert k in nat
    assert nat["config"]["engine"].startswith("native")
    assert nat["sweeps"] == py["sweeps"] and nat["converged"]
    assert nat["accuracy"]["residual_rel"] < 1e-5
    assert abs(nat["accuracy"]["residual_rel"] - py["accuracy"]["residual_rel"]) < 1e-9


def test_bench_rank_plan_simulation(tmp_path):
    """bench.py --simulate-P 4: rank 0's plan of a 4-GPU job on one GPU (the
    sim communicator: exchanges as device copies, no exchange calibration)
    prints its ms-per-sweep JSON line."""
    js = tmp_path / "sim.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--simulate-P", "4",
                        "--n", "2048", "--sim-sweeps", "1", "--json-out", str(js)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["unit"] == "ms/sweep" and d["simulated_P"] == 4 and d["value"] > 0, d


def test_merged_issue_is_bitwise_the_two_chain_solve(svdj, cuda, monkeypatch):
    """One GPU, 64 pairs per chain step (16384 columns, W = 64): the merged
    128-pair launches (PipelineExecutor.run_merged; the default there until
    the shared-GPU apply grid of round 6) give
    bitwise the two-chain result -- same pairs in the same step order and the
    Gram keeps the 64-pair row chunking.  One sweep of a 16384 x 16384 input."""
    from svdj.parallel import Communicator, DistributedBlockJacobi

    comm = Communicator(device=cuda, init=False)
    g = torch.Generator(device=cuda).manual_seed(3)
    A = torch.rand(16384, 16384, generator=g, device=cuda)
    out = {}
    for merge in ("1", "0"):
        monkeypatch.setenv("SVDJ_DEBUG", f"merge={merge}")
        cfg = svdj.SolverConfig(dtype=torch.float32, block=64, max_sweeps=1)
        res = DistributedBlockJacobi(cfg, comm).solve(A)
        assert res.info["merged_chains"] == (merge == "1"), res.info
        out[merge] = (res.U.clone(), res.S.clone(), res.V.clone(), list(res.history))
        del res
    for i in range(3):
        assert torch.equal(out["1"][i], out["0"][i])
    assert out["1"][3] == out["0"][3]
