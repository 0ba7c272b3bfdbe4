"""Process-group communicator (one process per GPU).

Replaces the reference's host-staged, root-centred MPI point-to-point star
(reference main.cu:582-680 scatter, 854-936 gather, 942 barrier;
SURVEY.md section 2.4) with torch.distributed:

* backend ``nccl`` (= RCCL on ROCm) for device tensors -- block exchange is
  GPU->GPU over xGMI, grouped send/recv (``batch_isend_irecv``);
* backend ``gloo`` for CPU tensors (CPU-only multi-process tests).

Every rank calls the same sequence; there is no root in the hot loop.  The
convergence value is an all-reduce (max of the off value, sum of rotations),
which the reference computed and dropped (main.cu:710).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


class Communicator:
    """Thin wrapper over a torch.distributed process group."""

    def __init__(self, backend: str | None = None, device: torch.device | None = None,
                 timeout_s: float = 600.0, init: bool = True):
        rank, world, local = env_world()
        if device is None:
            # SVDJ_SHARED_GPU=1: every rank on cuda:0 (rehearsing the multi-rank
            # RCCL path on a one-GPU box; not a performance configuration)
            idx = 0 if os.environ.get("SVDJ_SHARED_GPU") == "1" else local
            device = torch.device("cuda", idx) if torch.cuda.is_available() else torch.device("cpu")
        self.device = torch.device(device)
        if backend is None:
            backend = os.environ.get("SVDJ_COMM_BACKEND") or (
                "nccl" if self.device.type == "cuda" else "gloo")
        self.backend = backend
        self.owns_group = False
        if world > 1 and init and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {}
            if self.device.type == "cuda":
                torch.cuda.set_device(self.device)
                kw["device_id"] = self.device
            dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s),
                                    **kw)
            self.owns_group = True
        self.rank = dist.get_rank() if dist.is_initialized() else rank
        self.world = dist.get_world_size() if dist.is_initialized() else world

    @property
    def distributed(self) -> bool:
        return self.world > 1

    # ---------------------------------------------------------------- p2p
    def sendrecv(self, sends: list, recvs: list):
        """Grouped point-to-point: sends = [(tensor, dst)], recvs = [(tensor, src)]."""
        if not self.distributed:
            raise RuntimeError("sendrecv on a single rank")
        ops = [dist.P2POp(dist.isend, t, d) for t, d in sends if d != self.rank]
        ops += [dist.P2POp(dist.irecv, t, s) for t, s in recvs if s != self.rank]
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()

    def isendrecv(self, sends: list, recvs: list) -> list:
        """Like :meth:`sendrecv` but returns the works without waiting: on the
        GPU the transfer runs on the RCCL stream after the CURRENT stream's
        prior work, and ``work.wait()`` later makes the waiting stream (not
        the host) depend on it -- so compute on other streams overlaps it."""
        if not self.distributed:
            raise RuntimeError("isendrecv on a single rank")
        ops = [dist.P2POp(dist.isend, t, d) for t, d in sends if d != self.rank]
        ops += [dist.P2POp(dist.irecv, t, s) for t, s in recvs if s != self.rank]
        return dist.batch_isend_irecv(ops) if ops else []

    # ---------------------------------------------------------- collectives
    def allreduce_max_sum(self, mx: float | torch.Tensor, cnt: float | torch.Tensor):
        """Returns (global max of mx, global sum of cnt) as python floats."""
        t = torch.stack([torch.as_tensor(mx, dtype=torch.float64).reshape(()).to(self.device),
                         torch.as_tensor(cnt, dtype=torch.float64).reshape(()).to(self.device)])
        if self.distributed:
            a = t[0:1].clone()
            b = t[1:2].clone()
            dist.all_reduce(a, op=dist.ReduceOp.MAX)
            dist.all_reduce(b, op=dist.ReduceOp.SUM)
            t = torch.cat([a, b])
        h = t.cpu()
        return float(h[0]), float(h[1])

    def barrier(self):
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def broadcast(self, t: torch.Tensor, src: int = 0):
        if self.distributed:
            dist.broadcast(t, src)
        return t

    def max_over_ranks(self, x: float) -> float:
        if not self.distributed:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.cpu()[0])

    def destroy(self):
        if self.owns_group and dist.is_initialized():
            dist.destroy_process_group()
            self.owns_group = False
