"""Multi-rank rehearsal on ONE GPU: 2 ranks share cuda:0 (RCCL refuses a
duplicated GPU, so the exchange runs over gloo with host-synchronised
device tensors).  Exercises the pipelined executor's streams, events and
half-block exchanges, and the blocking path, end to end through bench.py."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("chains", [2, 1])
def test_two_ranks_shared_gpu(chains, tmp_path):
    out = tmp_path / "b.json"
    env = dict(os.environ, SVDJ_SHARED_GPU="1", SVDJ_COMM_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--size", "512", "--steps", "1",
           "--warmup", "0", "--chains", str(chains), "--json-out", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    d = json.loads(out.read_text())
    assert d["converged"] and d["n_gpus"] == 2, d
    assert d["accuracy"]["residual_rel"] < 1e-4, d
