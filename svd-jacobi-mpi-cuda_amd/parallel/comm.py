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

Two single-GPU rehearsal modes exist besides the production path:

* ``SVDJ_SHARED_GPU=1`` with the nccl backend: P processes share cuda:0 and
  still talk through RCCL.  RCCL refuses two ranks on one device of one host
  ("Duplicate GPU detected"), so each rank declares its own host identity
  (``NCCL_HOSTID``) and the ranks connect through RCCL's socket transport on
  the loopback interface.  The transport is not xGMI, but the torch/RCCL
  stream and event semantics the pipelined exchange relies on are the real
  ones, with no host synchronisation anywhere in the sweep.
* :class:`SimCommunicator`: ONE process plays rank g of a P-rank job; each
  exchange swaps the outgoing half super-block with one held by a simulated
  peer (device copies of exactly the real message sizes, optionally padded to
  the modelled xGMI link time).  It measures the true per-GPU compute time of
  rank g's sweep plan at P = 2, 4, 8 on one GPU.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def default_timeout_s() -> float:
    """Process-group timeout: ``SVDJ_COMM_TIMEOUT`` seconds (default 600;
    bench.py uses 300).  A
    collective or p2p op that does not finish in time makes the RCCL watchdog
    abort the process (TORCH_NCCL_ASYNC_ERROR_HANDLING), so a hung peer ends
    the job with a non-zero exit instead of hanging it."""
    return float(os.environ.get("SVDJ_COMM_TIMEOUT", "600"))


class Communicator:
    """Thin wrapper over a torch.distributed process group."""

    def __init__(self, backend: str | None = None, device: torch.device | None = None,
                 timeout_s: float | None = None, init: bool = True):
        rank, world, local = env_world()
        shared = os.environ.get("SVDJ_SHARED_GPU") == "1"
        if device is None:
            # SVDJ_SHARED_GPU=1: every rank on cuda:0 (rehearsing the multi-rank
            # path on a one-GPU box; not a performance configuration)
            idx = 0 if shared else local
            device = torch.device("cuda", idx) if torch.cuda.is_available() else torch.device("cpu")
        self.device = torch.device(device)
        if backend is None:
            backend = os.environ.get("SVDJ_COMM_BACKEND") or (
                "nccl" if self.device.type == "cuda" else "gloo")
        self.backend = backend
        self.timeout_s = default_timeout_s() if timeout_s is None else float(timeout_s)
        self.owns_group = False
        if world > 1 and init and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # fail fast: a timed-out RCCL op aborts the process
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
            if backend == "nccl" and shared:
                os.environ["NCCL_HOSTID"] = f"svdj-shared-gpu-rank{rank}"
                os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
                os.environ.setdefault("NCCL_IB_DISABLE", "1")
            kw = {}
            if self.device.type == "cuda":
                torch.cuda.set_device(self.device)
                kw["device_id"] = self.device
                # Create torch's stream pool (the solver's chain and comm
                # streams come from it) BEFORE RCCL creates its own streams:
                # HIP binds streams to the GPU_MAX_HW_QUEUES hardware queues
                # in creation order, and two chain streams on one queue run
                # serialised (profiles/r2_native_dist: the native driver
                # measured exactly that until it created its streams first).
                torch.cuda.Stream(self.device)
            dist.init_process_group(backend=backend,
                                    timeout=datetime.timedelta(seconds=self.timeout_s), **kw)
            self.owns_group = True
        self.rank = dist.get_rank() if dist.is_initialized() else rank
        self.world = dist.get_world_size() if dist.is_initialized() else world

    @classmethod
    def local(cls, device) -> "Communicator":
        """A world-1 communicator on ``device`` that never touches a process
        group, even inside a distributed job: the single-GPU solve behind
        ``api.svd`` runs the distributed engine's plan at P = 1 (no
        exchanges, every collective the identity)."""
        c = cls.__new__(cls)
        c.device = torch.device(device)
        c.backend = "nccl" if c.device.type == "cuda" else "gloo"
        c.timeout_s = default_timeout_s()
        c.owns_group = False
        c.rank, c.world = 0, 1
        return c

    @property
    def distributed(self) -> bool:
        return self.world > 1

    @property
    def async_device(self) -> bool:
        """True when p2p on device tensors is stream-ordered (RCCL): the
        exchange is enqueued after the issuing stream's work and completion is
        a stream dependency, never a host wait."""
        return self.backend == "nccl" and self.device.type == "cuda"

    # ------------------------------------------------------------ readiness
    def readiness(self, partners=()) -> dict:
        """Check and report the process -> GPU mapping of a multi-rank job.

        Every rank contributes (host, device index, local device count); the
        ranks must sit on distinct (host, device) pairs -- one process per
        GPU -- unless SVDJ_SHARED_GPU=1 (one-GPU rehearsal).  ``partners``
        (the tournament peers of this rank) are probed for peer access
        (hipDeviceCanAccessPeer: xGMI P2P) when on the same host.  Raises
        RuntimeError on a bad mapping, so a misconfigured 8-GPU launch fails
        before any sweep instead of time-sharing a device."""
        info = {"world": self.world, "backend": self.backend}
        if self.device.type != "cuda":
            return info
        import socket
        import zlib

        host = zlib.crc32(socket.gethostname().encode()) & 0x7FFFFFFF
        idx = self.device.index if self.device.index is not None else 0
        peers = sorted({int(p) for p in partners if 0 <= int(p) < self.world and int(p) != self.rank})
        me = torch.tensor([host, idx, torch.cuda.device_count(), len(peers), 0],
                          dtype=torch.int64, device=self.device)
        rows = self.allgather(me).cpu().tolist() if self.distributed else [me.tolist()]
        shared = os.environ.get("SVDJ_SHARED_GPU") == "1"
        pairs = {(r[0], r[1]) for r in rows}
        if len(pairs) != len(rows) and not shared:
            raise RuntimeError(f"ranks share a GPU (host, device) = "
                               f"{[(r[0], r[1]) for r in rows]}: launch one process per GPU "
                               "(device = cuda:LOCAL_RANK) or set SVDJ_SHARED_GPU=1")
        ok = 0
        for p in peers:
            h, d = rows[p][0], rows[p][1]
            if h == host and d != idx:
                ok += int(torch.cuda.can_device_access_peer(idx, d))
        me[4] = ok
        rows = self.allgather(me).cpu().tolist() if self.distributed else [me.tolist()]
        info.update(devices=[int(r[1]) for r in rows], hosts=len({r[0] for r in rows}),
                    rccl_ranks=dist.get_world_size() if dist.is_initialized() else 1,
                    shared_gpu=shared,
                    p2p_partners=[f"{int(r[4])}/{int(r[3])}" for r in rows])
        return info

    # ---------------------------------------------------------------- p2p
    def _ops(self, sends: list, recvs: list) -> list:
        ops = [dist.P2POp(dist.isend, t, d) for t, d in sends if d != self.rank]
        ops += [dist.P2POp(dist.irecv, t, s) for t, s in recvs if s != self.rank]
        return ops

    def _host_sync(self):
        """gloo on device tensors (the one-GPU rehearsal of the multi-rank
        path) reads and writes them outside stream order: the data must be
        complete before a call and the result before its first use.  RCCL
        (stream-ordered) needs none of this."""
        if self.device.type == "cuda" and not self.async_device:
            torch.cuda.synchronize(self.device)

    def sendrecv(self, sends: list, recvs: list):
        """Grouped point-to-point: sends = [(tensor, dst)], recvs = [(tensor, src)]."""
        if not self.distributed:
            raise RuntimeError("sendrecv on a single rank")
        ops = self._ops(sends, recvs)
        if ops:
            self._host_sync()
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            self._host_sync()

    def isendrecv(self, sends: list, recvs: list) -> list:
        """Like :meth:`sendrecv` but returns the works without waiting: on the
        GPU the transfer runs on the RCCL stream after the CURRENT stream's
        prior work, and ``work.wait()`` later makes the waiting stream (not
        the host) depend on it -- so compute on other streams overlaps it."""
        if not self.distributed:
            raise RuntimeError("isendrecv on a single rank")
        ops = self._ops(sends, recvs)
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

    def allreduce_stop(self, mx, ms, cnt, cnt2):
        """(global max of mx, global max of ms, global sums of cnt and cnt2)
        as python floats: the block path's per-sweep stop-test values."""
        t = torch.stack([torch.as_tensor(x, dtype=torch.float64).reshape(()).to(self.device)
                         for x in (mx, ms, cnt, cnt2)])
        if self.distributed:
            a = t[0:2].clone()
            b = t[2:4].clone()
            self._host_sync()  # gloo reads device tensors outside stream order
            dist.all_reduce(a, op=dist.ReduceOp.MAX)
            dist.all_reduce(b, op=dist.ReduceOp.SUM)
            self._host_sync()
            t = torch.cat([a, b])
        h = t.cpu()
        return float(h[0]), float(h[1]), float(h[2]), float(h[3])

    def allreduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over ranks (device tensors: RCCL, stream-ordered)."""
        if self.distributed:
            self._host_sync()
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            self._host_sync()
        return t

    # temporary bytes ordered_sum_ may hold at once (world x slab)
    ORDERED_SUM_BYTES = 256 << 20

    def ordered_sum_(self, t: torch.Tensor, max_bytes: int | None = None) -> torch.Tensor:
        """In-place sum over ranks added in rank order, t_0 + t_1 + ..., on
        every rank (all-gather, then local adds): bitwise the same result on
        any backend and ring, unlike a floating all-reduce.  The all-gather
        runs over slabs of t's flat view so that at most ``max_bytes``
        (default ORDERED_SUM_BYTES) of gathered copies exist at once: a whole
        n x n Gram gathered from P ranks would need P n^2 elements (n = 65536
        fp64 at P = 8: 256 GB).  Slabbing does not change any element's
        additions, so the result is the same bits."""
        if not self.distributed:
            return t
        cap = self.ORDERED_SUM_BYTES if max_bytes is None else int(max_bytes)
        flat = t.view(-1) if t.is_contiguous() else t.contiguous().view(-1)
        per = max(1, cap // max(1, self.world * flat.element_size()))
        for s0 in range(0, flat.numel(), per):
            sl = flat[s0:s0 + per]
            parts = self.allgather(sl)
            sl.copy_(parts[0])
            for h in range(1, self.world):
                sl.add_(parts[h])
        if not t.is_contiguous():
            t.copy_(flat.view_as(t))
        return t

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        """(world, *t.shape) stack of every rank's ``t`` (RCCL all-gather)."""
        flat = t.contiguous().reshape(-1)
        out = torch.empty(self.world * flat.numel(), dtype=t.dtype, device=t.device)
        if self.distributed:
            self._host_sync()
            dist.all_gather_into_tensor(out, flat)
            self._host_sync()
        else:
            out.copy_(flat)
        return out.view((self.world,) + tuple(t.shape))

    def barrier(self):
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def broadcast(self, t: torch.Tensor, src: int = 0):
        if self.distributed:
            self._host_sync()
            dist.broadcast(t, src)
            self._host_sync()
        return t

    def max_over_ranks(self, x: float) -> float:
        if not self.distributed:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        self._host_sync()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        self._host_sync()
        return float(t.cpu()[0])

    def destroy(self):
        if self.owns_group and dist.is_initialized():
            dist.destroy_process_group()
            self.owns_group = False


class _StreamWork:
    """Completion handle of a simulated exchange: ``wait()`` makes the
    CURRENT stream wait for it (the RCCL work semantics)."""

    def __init__(self, event: torch.cuda.Event | None):
        self.event = event

    def wait(self):
        if self.event is not None:
            torch.cuda.current_stream().wait_event(self.event)


class SimCommunicator:
    """Rank ``rank`` of a simulated ``world``-rank job, in one process.

    Collectives are local (the simulated peers are taken to agree), and
    every exchange is a swap with a simulated peer: the received tensor is
    one the simulated ring sent earlier (initially ``seed_fn(pos, like)`` for
    message slot ``pos`` -- other columns of the same matrix), and the sent
    tensor joins the ring.  The ring holds ``2*world - 2`` entries per message shape, like the
    super-blocks held by the other ranks, so a received half was never paired
    with this rank's blocks in the current round and the EVDs keep real
    rotation work.  The numerics are therefore NOT those of the real job
    (sweep counts do not converge like it); use this for per-sweep time.

    ``link_gbps`` > 0 pads every exchange on the comm stream with a device
    spin of the modelled transfer time (bytes of the larger direction over
    the link bandwidth), so the overlap with compute can be studied.  With
    ``exchange="spread"`` the modelled time is that of the two relayed phases
    over all links (parallel/spread.py, 2/(P-1) of the direct time); the
    device copies stay direct.
    """

    backend = "sim"

    def __init__(self, world: int, rank: int, device: torch.device, seed_fn=None,
                 link_gbps: float = 0.0, exchange: str = "direct"):
        if not (0 <= rank < world):
            raise ValueError(f"rank {rank} not in world {world}")
        self.world, self.rank = int(world), int(rank)
        self.device = torch.device(device)
        self.timeout_s = 0.0
        self.owns_group = False
        self.seed_fn = seed_fn
        self.link_gbps = float(link_gbps)
        from .spread import modelled_time_factor, resolve_exchange
        self.exchange = resolve_exchange(exchange, self.world)
        self.link_factor = modelled_time_factor(self.world) if self.exchange == "spread" else 1.0
        self._ring: dict = {}
        self.bytes_moved = 0
        self.exchanges = 0

    distributed = property(lambda self: self.world > 1)
    async_device = property(lambda self: self.device.type == "cuda")

    def _swap(self, sends: list, recvs: list):
        nbytes = 0
        for pos, ((st, _), (rt, _)) in enumerate(zip(sends, recvs)):
            key = (pos, tuple(rt.shape), rt.dtype)  # one ring per message slot
            ring = self._ring.setdefault(key, [])
            depth = max(2 * self.world - 2, 1)
            while len(ring) < depth:
                ring.append(self.seed_fn(pos, rt) if self.seed_fn else torch.zeros_like(rt))
            src = ring.pop(0)
            rt.copy_(src)
            src.copy_(st)  # reuse the storage for the outgoing tensor
            ring.append(src)
            nbytes += st.numel() * st.element_size()
        self.bytes_moved += nbytes
        self.exchanges += 1
        if self.link_gbps > 0 and self.device.type == "cuda":
            from ..ops import kernels as K
            K.spin_ns(self.device, nbytes * self.link_factor / (self.link_gbps * 1e9) * 1e9)

    def sendrecv(self, sends: list, recvs: list):
        self._swap(sends, recvs)

    def isendrecv(self, sends: list, recvs: list) -> list:
        self._swap(sends, recvs)
        if self.device.type != "cuda":
            return []
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return [_StreamWork(ev)]

    def allreduce_max_sum(self, mx, cnt):
        return float(torch.as_tensor(mx).double()), float(torch.as_tensor(cnt).double())

    def allreduce_stop(self, mx, ms, cnt, cnt2):
        return tuple(float(torch.as_tensor(x).double()) for x in (mx, ms, cnt, cnt2))

    def allreduce_sum_(self, t):
        """The sum over ``world`` ranks is modelled as ``world`` copies of this
        rank's tensor.  For a square (Gram) tensor a small ridge keeps it as
        well conditioned as the real all-reduced Gram of a tall matrix (one
        row block alone can be square and ill-conditioned, which would push
        the simulated CholeskyQR2 onto its Householder fallback): cost-only."""
        t.mul_(self.world)
        if t.dim() == 2 and t.shape[0] == t.shape[1]:
            t.diagonal().add_(t.diagonal().mean() * 1e-2)
        return t

    def allgather(self, t):
        return torch.stack([t.clone() for _ in range(self.world)])

    def barrier(self):
        pass

    def broadcast(self, t, src: int = 0):
        return t

    def max_over_ranks(self, x: float) -> float:
        return float(x)

    def destroy(self):
        pass
