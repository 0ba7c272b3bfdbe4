"""Native distributed solver (csrc/dist/svdj_dist.cpp) through its fork launcher
bin/svdj_dist_main: RCCL tournament, no Python and no torch in the ranks.

On the one-GPU box the ranks share cuda:0 (--shared-gpu: each rank its own
NCCL_HOSTID, socket transport on loopback); the plan, the grouped
ncclSend/ncclRecv exchanges and the all-reduced stop test are the ones an
8-GPU node runs.  The launcher verifies ||A - U S V^T||_F / ||A||_F and
orthogonality in fp64 on rank 0 after gathering every rank's columns
(reference main.cu:1630-1660 computes the same residual)."""
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "svd-jacobi-mpi-cuda_amd", "bin", "svdj_dist_main")


def _exe():
    if not os.path.exists(EXE):
        import importlib
        importlib.import_module("svd-jacobi-mpi-cuda_amd._build").build_dist()
    return EXE


def _value(out, key):
    return float(out.split(key)[1].split()[0])


@pytest.mark.parametrize("np_,n,dtype,extra", [
    (1, 300, "f64", []),
    (2, 1000, "f64", ["--input", "dense"]),
    (4, 1024, "f32", ["--input", "dense"]),
    (2, 700, "f64", ["--m", "900", "--input", "dense", "--block", "64"]),
])
def test_native_dist_launcher(np_, n, dtype, extra):
    cmd = [_exe(), str(n), "--np", str(np_), "--dtype", dtype, "--verify", "--timeout", "120",
           *extra]
    if np_ > 1:
        cmd.append("--shared-gpu")
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=170, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "SVD MPI+OMP time with U,V calculation" in out
    assert re.search(r"converged: [12]\b", out), out
    rel = _value(out, "||A-USVt||_F/||A||_F:")
    ou = _value(out, "||U^TU-I||_F:")
    ov = _value(out, "||V^TV-I||_F:")
    if dtype == "f64":
        assert rel < 1e-11 and ou < 1e-10 and ov < 2e-10, out
    else:
        assert rel < 2e-5 and ou < 5e-2 and ov < 2e-3, out


def test_native_dist_rank_failure_stops_job():
    """An invalid problem on every rank (block width 48) must end the whole
    job with a non-zero status, not hang the other ranks."""
    r = subprocess.run([_exe(), "256", "--np", "2", "--shared-gpu", "--block", "48",
                        "--timeout", "60"], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0


def test_native_dead_peer_watchdog():
    """Failure detection, native engine: rank 1 exits abruptly after sweep 2
    (--inject-fault 1:2) and the launcher does NOT stop the other rank
    (--keep-going), so rank 0's own watchdog (RCCL async error, or no sweep
    finished within --timeout) must abort its communicator and exit 3 --
    within the timeout, not hang in a receive from the dead peer."""
    import time
    t0 = time.time()
    r = subprocess.run([_exe(), "1024", "--np", "2", "--shared-gpu", "--dtype", "f32",
                        "--input", "dense", "--inject-fault", "1:2", "--keep-going",
                        "--timeout", "20"], capture_output=True, text=True, timeout=150)
    el = time.time() - t0
    out = r.stdout + r.stderr
    assert r.returncode != 0, out[-3000:]
    assert "fault injection: rank 1" in out, out[-3000:]
    assert "[rank 0]" in out and "watchdog" in out.lower(), out[-3000:]
    assert el < 110, (el, out[-3000:])


def test_native_persistent_handle_repeat_solves():
    """Warm-up solves reuse the persistent handle (no per-solve allocation):
    the timed solve after two warm-ups converges to the same accuracy, with
    the exchange timing reported (receive in place, no copy-in)."""
    r = subprocess.run([_exe(), "1024", "--np", "2", "--shared-gpu", "--dtype", "f32",
                        "--input", "dense", "--verify", "--warmup", "2", "--comm-timing",
                        "--timeout", "120"], capture_output=True, text=True, timeout=170)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert re.search(r"converged: [12]\b", out) and "exposed_comm_ms:" in out, out
    assert _value(out, "||A-USVt||_F/||A||_F:") < 2e-5, out


def test_native_dist_reference_triangular_input_converges():
    """The reference's own run (triangular U(0,1) input, fp64, 2 ranks --
    build/runSVDMPICUDAWithoutCMake.slurm:30) converges: the negligible-
    column floor keeps noise-level columns from being rotated forever."""
    r = subprocess.run([_exe(), "1200", "--np", "2", "--shared-gpu", "--dtype", "f64",
                        "--verify", "--timeout", "120"], capture_output=True, text=True,
                       timeout=170)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert re.search(r"converged: [12]\b", out), out
    assert _value(out, "||A-USVt||_F/||A||_F:") < 1e-12, out
    assert _value(out, "||V^TV-I||_F:") < 1e-9, out


def test_native_spread_exchange_matches_direct():
    """Native engine, 4 RCCL ranks: the spread exchange (every half relayed
    over all peers in two grouped phases, svdj_dist_problem.exchange = 2)
    delivers the direct exchange's bits -- same sweeps, same off value, same
    residual to the printed digits."""
    outs = {}
    for ex in ("direct", "spread"):
        r = subprocess.run([_exe(), "1024", "--np", "4", "--shared-gpu", "--dtype", "f32",
                            "--input", "dense", "--verify", "--exchange", ex, "--timeout", "120"],
                           capture_output=True, text=True, timeout=170)
        out = r.stdout + r.stderr
        assert r.returncode == 0 and re.search(r"converged: [12]\b", out), out[-4000:]
        outs[ex] = out
    for key in ("sweeps:", "||A-USVt||_F:", "||U^TU-I||_F:", "||V^TV-I||_F:"):
        assert outs["direct"].split(key)[1].split("\n")[0] == \
            outs["spread"].split(key)[1].split("\n")[0], key


def test_native_auto_exchange_is_measured():
    """Native engine, 4 RCCL ranks, exchange left on auto: the handle times
    one direct and one spread half exchange (max over ranks) and keeps the
    faster; the solve then matches an explicitly direct run to the printed
    digits (both exchanges deliver the same bits)."""
    outs = {}
    for ex in ("auto", "direct"):
        r = subprocess.run([_exe(), "1024", "--np", "4", "--shared-gpu", "--dtype", "f32",
                            "--input", "dense", "--verify", "--exchange", ex, "--timeout", "120"],
                           capture_output=True, text=True, timeout=170)
        out = r.stdout + r.stderr
        assert r.returncode == 0 and re.search(r"converged: [12]\b", out), out[-4000:]
        outs[ex] = out
    m = re.search(r"exchange calibration: direct ([\d.]+) ms, spread ([\d.]+) ms", outs["auto"])
    assert m, outs["auto"][-3000:]
    d, s = float(m.group(1)), float(m.group(2))
    chosen = re.search(r"exchange: (\w+)", outs["auto"]).group(1)
    assert chosen == ("spread" if s < 0.9 * d else "direct"), (d, s, chosen)
    for key in ("sweeps:", "||A-USVt||_F:", "||V^TV-I||_F:"):
        assert outs["auto"].split(key)[1].split("\n")[0] == \
            outs["direct"].split(key)[1].split("\n")[0], key


def test_native_engine_production_default_matches_python(tmp_path):
    """The headline configuration (16384^2 fp32, one GPU) in both engines:
    the native engine takes the same one-GPU issue as the Python executor --
    quad steps on two chains (from 32 pairs the chains stay apart, round 6)
    -- and the same stop rule, so both stop after the same sweep with the
    same accuracy."""
    import json
    import sys
    out = {}
    for eng in ("native", "python"):
        js = tmp_path / f"{eng}.json"
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--engine", eng,
                            "--steps", "1", "--warmup", "1", "--json-out", str(js)],
                           capture_output=True, text=True, timeout=240,
                           env=dict(os.environ, MASTER_PORT=str(29960 + len(out))))
        assert r.returncode == 0, r.stderr[-2000:]
        out[eng] = json.loads(js.read_text())
    nat, py = out["native"], out["python"]
    for d in (nat, py):
        assert d["config"]["quad_steps"] and not d["config"]["merged_chains"], d["config"]
        assert d["converged"] and d["accuracy"]["residual_rel"] < 3e-5, d["accuracy"]
    assert nat["sweeps"] == py["sweeps"], (nat["sweeps"], py["sweeps"])
    assert abs(nat["accuracy"]["residual_rel"] - py["accuracy"]["residual_rel"]) < 1e-8
    assert nat["ms_per_step"] < 1.1 * py["ms_per_step"], (nat["ms_per_step"], py["ms_per_step"])


def test_native_quad_steps_two_ranks():
    """Native engine, 2 RCCL ranks, quad steps forced (--quad on; auto from 32
    pairs per chain step): converges to fp32 accuracy through the exchanges."""
    r = subprocess.run([_exe(), "4096", "--np", "2", "--shared-gpu", "--dtype", "f32",
                        "--input", "dense", "--verify", "--quad", "on", "--timeout", "120"],
                       capture_output=True, text=True, timeout=240)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and re.search(r"converged: [12]\b", out), out[-4000:]
    assert "quad steps" in out, out[-3000:]
    assert _value(out, "||A-USVt||_F/||A||_F:") < 3e-5, out
    assert _value(out, "||V^TV-I||_F:") < 5e-3, out
