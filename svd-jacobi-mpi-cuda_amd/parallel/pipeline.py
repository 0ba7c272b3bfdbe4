"""Half-block pipelined sweep: RCCL exchange overlapped with compute.

The tournament (schedule.tournament) replaces ONE resident super-block per
GPU between rounds.  Done as a whole (parallel/distributed.py ``_exchange``)
the exchange sits between rounds with the GPU idle: at n=16384 on 8 GPUs
that is 15 x 134 MB per sweep per GPU over one xGMI link.  The reference's
exchange (rank-0 star, host-staged, reference main.cu:582-680, 854-936) is
fully serial as well.

Here every super-block is handled as two halves and a round's cross work is
four half-pair tasks (I = incoming slot, S = staying slot):

    stream 0:  T00 = I0 x S0   ->  T01 = I0 x S1
    stream 1:  T10 = I1 x S0   ->  T11 = I1 x S1

Half 0 of the next outgoing slot is last touched by T01/T10, half 1 by T11,
so the send/recv of half 0 is issued right after T10 and runs under T11;
half 1 is issued after T11 and runs under the next round's T00' and T01'
(which only need the already-arrived half 0).  Every task waits only on the
events of the tasks that last touched its two halves, so the two compute
streams and the RCCL stream overlap as far as the data dependencies allow.
Round 0 of every sweep also runs the within-super-block round robins
(RR(slot 0) || RR(slot 1)); the last round of a sweep (no exchange after it,
the whole sweep on one GPU) runs the fully parallel order [T00 || T11],
[T01 || T10].  Every block pair of the matrix still meets
exactly once per sweep (checked by tests/test_pipeline_cpu.py).

On CPU tensors (gloo tests) the same item list runs sequentially, with the
exchanges blocking at their trigger points -- identical arithmetic.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np
import torch

from .schedule import (quad_bipartite, quad_bipartite_modes, quad_round_robin,
                       quad_round_robin_modes, round_robin)
from .spread import relay_chunk, resolve_exchange, spread_ops


@dataclass
class Task:
    """One chain of block steps on local block indices."""
    name: str
    pairs: np.ndarray        # (steps, pairs_per_step, 2)
    modes: list
    stream: int
    halves: tuple            # ((slot, part), ...) touched (parts are halves for 2 chains)


@dataclass
class Send:
    """Exchange of part ``half`` of slot ``slot`` before round ``round``."""
    round: int
    slot: int
    half: int


@dataclass
class SweepPlan:
    P: int
    k: int
    items: list = field(default_factory=list)   # Task | Send, in issue order
    parts: int = 2           # a super-block moves in this many parts (= chains)


def _blocks(slot: int, half: int, k: int, parts: int = 2) -> list:
    h = k // parts
    return list(range(slot * k + half * h, slot * k + (half + 1) * h))


def _bipartite(xs: list, ys: list) -> np.ndarray:
    h = len(xs)
    out = np.zeros((h, h, 2), dtype=np.int32)
    for t in range(h):
        for a in range(h):
            out[t, a] = (xs[a], ys[(a + t) % h])
    return out


def sweep_plan(P: int, k: int, xslot: np.ndarray, chains: int = 2, quad: bool = False
               ) -> SweepPlan:
    """Items of one sweep.  ``xslot[r]`` is the slot replaced before round r
    (r >= 1), as produced by schedule.tournament.  (Four chains in quarters
    were measured slower than two at every P in round 2 -- 8-GPU plan 64 ->
    84-88 ms per sweep -- and removed.)  ``quad``: the same block pairs in
    quad order (schedule.quad_round_robin / quad_bipartite, mode 4/5 steps
    fused two at a time, csrc/hip/block.hip "quad step"); needs k % 4 == 0."""
    if chains != 2:
        raise ValueError(f"pipelined sweep: 2 chains, got {chains}")
    if k < 2 or k % 2:
        raise ValueError(f"pipelined sweep needs an even block count per super-block, got {k}")
    if quad and k % 4:
        raise ValueError(f"quad steps need a multiple of 4 blocks per super-block, got {k}")
    plan = SweepPlan(P, k)
    if quad:
        rr, rr_modes = quad_round_robin(k), quad_round_robin_modes(k)
    else:
        rr, rr_modes = round_robin(k), [1] + [0] * (k - 2)
    plan.items.append(Task("rr0", rr.copy(), rr_modes, 0, ((0, 0), (0, 1))))
    plan.items.append(Task("rr1", rr + k, rr_modes, 1, ((1, 0), (1, 1))))
    R = 2 * P - 1
    for r in range(R):
        inc = int(xslot[r]) if r > 0 else 0
        stay = 1 - inc
        h = k // 2

        def task(name, ih, sh, stream):
            xs, ys = _blocks(inc, ih, k), _blocks(stay, sh, k)
            if quad:
                return Task(f"r{r}.{name}", quad_bipartite(xs, ys), quad_bipartite_modes(h), stream,
                            ((inc, ih), (stay, sh)))
            return Task(f"r{r}.{name}", _bipartite(xs, ys), [0] * h, stream, ((inc, ih), (stay, sh)))

        nxt = int(xslot[r + 1]) if r + 1 < R else None
        if nxt is None:
            # nothing to send after this round: the two fully parallel phases
            # [T00 || T11], [T01 || T10]
            plan.items += [task("T00", 0, 0, 0), task("T11", 1, 1, 1), task("T01", 0, 1, 0),
                           task("T10", 1, 0, 1)]
            continue
        plan.items += [task("T00", 0, 0, 0), task("T01", 0, 1, 0), task("T10", 1, 0, 1),
                       Send(r + 1, nxt, 0), task("T11", 1, 1, 1), Send(r + 1, nxt, 1)]
    return plan


def issue_groups(items: list, joint: bool, max_group: int = 2) -> list:
    """The plan's items regrouped for issue: a Task, a Send, or a tuple of up
    to ``max_group`` independent tasks issued jointly (merged into single
    launches on one GPU, :meth:`PipelineExecutor.run_merged`).

    Greedy: a task is grouped with the following tasks (Sends in between are
    skipped) while each runs on a new stream, touches parts disjoint from the
    group's, and no skipped Send concerns its parts; the skipped Sends are
    issued after the group (they only wait on events of earlier users of
    their part, so the delay is host-side only).  For two chains this pairs
    rr0+rr1, T01+T10, the last round's T00+T11 / T01+T10, and T11 of a round
    with T00 of the next across the half-1 Send."""
    out = []
    i, n = 0, len(items)
    while i < n:
        it = items[i]
        if not (joint and isinstance(it, Task)):
            out.append(it)
            i += 1
            continue
        group, streams, parts = [it], {it.stream}, set(it.halves)
        skipped, last, j = [], i, i + 1
        while j < n and len(group) < max_group:
            x = items[j]
            if isinstance(x, Send):
                skipped.append((j, x))
                j += 1
                continue
            if (x.stream in streams or set(x.halves) & parts
                    or any((sd.slot, sd.half) in x.halves for _, sd in skipped)):
                break
            group.append(x)
            streams.add(x.stream)
            parts |= set(x.halves)
            last = j
            j += 1
        out.append(tuple(group) if len(group) > 1 else it)
        out.extend(sd for idx, sd in skipped if idx < last)
        i = last + 1
    return out


def check_plan_coverage(plans: list, tour) -> None:
    """Simulate one sweep on every GPU (``plans[g]`` is GPU g's plan; all have
    the same item structure) on global block ids, from the tournament's
    starting placement; assert that every pair of global blocks meets
    exactly once.  Raises AssertionError."""
    P = len(plans)
    k = plans[0].k
    parts = plans[0].parts
    h = k // parts
    # place[g][slot][part] = (super-block, part) currently resident
    place = [[[(int(tour.held[0, g, s]), hh) for hh in range(parts)] for s in range(2)]
             for g in range(P)]
    met = {}
    n_items = len(plans[0].items)
    assert all(len(p.items) == n_items for p in plans)
    for i in range(n_items):
        its = [p.items[i] for p in plans]
        if isinstance(its[0], Send):
            assert all(isinstance(x, Send) and x.half == its[0].half and x.round == its[0].round
                       for x in its)
            r, hh = its[0].round, its[0].half
            new = [None] * P
            for g in range(P):
                src = int(tour.recv_from[r, g])
                assert int(tour.send_to[r, src]) == g
                new[g] = place[src][its[src].slot][hh]
            for g in range(P):
                place[g][its[g].slot][hh] = new[g]
            continue
        for g in range(P):
            it = its[g]
            for t in range(it.pairs.shape[0]):
                for a, b in it.pairs[t]:
                    ga = _global_block(place[g], int(a), k, h)
                    gb = _global_block(place[g], int(b), k, h)
                    assert ga != gb
                    key = (min(ga, gb), max(ga, gb))
                    met[key] = met.get(key, 0) + 1
    nb = 2 * P * k
    assert len(met) == nb * (nb - 1) // 2, (len(met), nb * (nb - 1) // 2)
    assert all(v == 1 for v in met.values())


def _global_block(place_g, b: int, k: int, h: int) -> int:
    slot, rem = divmod(b, k)
    half, off = divmod(rem, h)
    sb, hh = place_g[slot][half]
    return sb * k + hh * h + off


def _union(iv: list) -> list:
    """Sorted, merged union of (start, end) intervals."""
    out = []
    for a, b in sorted(x for x in iv if x[1] > x[0]):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def exposed_time(waits: list, busy: list) -> float:
    """Measure of the time covered by some wait interval (a compute stream
    idle until an exchange arrives) and by NO busy interval (a task running
    on any compute stream of the rank): each moment counts once, however many
    consumers wait on the arrival and on however many streams."""
    w, b = _union(waits), _union(busy)
    total, j = 0.0, 0
    for ws, we in w:
        t = ws
        while j < len(b) and b[j][1] <= t:
            j += 1
        k = j
        while t < we:
            if k < len(b) and b[k][0] <= t:
                t = max(t, b[k][1])
                k += 1
                continue
            nxt = b[k][0] if k < len(b) else we
            total += min(nxt, we) - t
            t = min(nxt, we)
    return total


class HalfLayout:
    """Where each resident half super-block lives: the rank's storage is a
    row of half buffers (hB columns each): loc[slot][half] is the buffer of
    (slot, half), spare[half] the free buffer that the next exchange of a
    half ``half`` receives into.  An exchange sends from loc[x][h], receives
    into spare[h] and swaps the two -- the received columns are used where
    they landed, no copy (round 2 received into a staging buffer and copied
    it into place: 654 copy dispatches per 8-GPU rank-plan profile).
    Buffers {h, 2 + h, 4 + h} always hold (slot 0, h), (slot 1, h), spare."""

    def __init__(self, spares: bool):
        self.loc = [[0, 1], [2, 3]]
        self.spare = [4, 5] if spares else None

    @property
    def nbuf(self) -> int:
        return 6 if self.spare is not None else 4

    def canonical(self) -> bool:
        return self.loc == [[0, 1], [2, 3]]

    def table(self, k: int) -> np.ndarray:
        """Local block id (slot * k + half * k/2 + j) -> physical block id."""
        hk = k // 2
        t = np.empty(2 * k, dtype=np.int32)
        for s in range(2):
            for h in range(2):
                t[s * k + h * hk:s * k + (h + 1) * hk] = self.loc[s][h] * hk + np.arange(hk)
        return t

    def moves_to_canonical(self) -> list:
        """(src buffer, dst buffer) copies that bring (slot, half) back to
        buffer 2 slot + half, using the spare as scratch (applied in order)."""
        mv = []
        if self.spare is None:
            return mv
        for h in range(2):
            where = {0: self.loc[0][h], 1: self.loc[1][h]}  # slot -> buffer
            free = self.spare[h]
            for _ in range(4):
                todo = [s for s in (0, 1) if where[s] != 2 * s + h]
                if not todo:
                    break
                ready = [s for s in todo if 2 * s + h == free]
                if ready:
                    s = ready[0]
                    mv.append((where[s], free))
                    where[s], free = free, where[s]
                else:  # both slots sit in each other's home: park one in the spare
                    s = todo[0]
                    mv.append((where[s], free))
                    where[s], free = free, where[s]
            self.loc[0][h], self.loc[1][h], self.spare[h] = where[0], where[1], free
        return mv


_EXCHANGE_CACHE: dict = {}


def calibrate_exchange(comm, tour, shapes, dtype, dev, reps: int = 3):
    """("direct" | "spread", summary) for the exchange of half buffers of
    ``shapes`` over this job's links: both variants of the first tournament
    round are timed (one warm-up, ``reps`` timed, barrier + device sync around
    each, the max over ranks), and spread is kept only if it is at least 10 %
    faster.  Every rank reaches the same decision (the times are all-reduced).
    Cached per (world, shapes, dtype): one calibration per solver geometry.
    The spread default rests on a link model (spread.modelled_time_factor) that
    ignores the relay's extra HBM traffic and RCCL op count; this replaces the
    model by a measurement."""
    key = (comm.world, tuple(shapes), str(dtype))
    hit = _EXCHANGE_CACHE.get(key)
    if hit is not None:
        return hit
    P, g, r = comm.world, comm.rank, 1
    dst, src = int(tour.send_to[r, g]), int(tour.recv_from[r, g])
    outs = [torch.zeros(sh, dtype=dtype, device=dev) for sh in shapes]
    ins = [torch.empty_like(t) for t in outs]
    flat_out = [t.reshape(-1) for t in outs]
    flat_in = [t.reshape(-1) for t in ins]
    sizes = [t.numel() for t in flat_out]
    ops = spread_ops(g, tour.send_to[r], sizes, [True] * len(sizes))
    relay = [torch.empty(P, relay_chunk(n, P), dtype=dtype, device=dev) for n in sizes]

    def tensor(op):
        mi, (a, b), peer, where = op
        if where == "out":
            return flat_out[mi][a:b], peer
        if where == "in":
            return flat_in[mi][a:b], peer
        return relay[mi][where[1], :b - a], peer

    variants = {
        "direct": [([(t, dst) for t in outs], [(t, src) for t in ins])],
        "spread": [([tensor(o) for o in ops.p1_send], [tensor(o) for o in ops.p1_recv]),
                   ([tensor(o) for o in ops.p2_send], [tensor(o) for o in ops.p2_recv])],
    }
    def sync():
        if torch.device(dev).type == "cuda":
            torch.cuda.synchronize(dev)

    times = {}
    for name, phases in variants.items():
        best = float("inf")
        for it in range(reps + 1):
            comm.barrier()
            sync()
            t0 = time.perf_counter()
            for ps, pr in phases:
                for w in comm.isendrecv(ps, pr):
                    w.wait()
            sync()
            dt = comm.max_over_ranks(time.perf_counter() - t0)
            if it:
                best = min(best, dt)
        times[name] = best
    choice = "spread" if times["spread"] < 0.9 * times["direct"] else "direct"
    summary = (f"measured at startup: direct {times['direct'] * 1e3:.3f} ms, spread "
               f"{times['spread'] * 1e3:.3f} ms per half exchange -> {choice}")
    _EXCHANGE_CACHE[key] = (choice, summary)
    return choice, summary


class PipelineExecutor:
    """Runs a :class:`SweepPlan` on the resident buffers of one rank.

    Storage: ``At``/``Vt``/``D`` hold :class:`HalfLayout` ``nbuf`` half
    buffers (4, or 6 with the two receive spares of a multi-rank job); the
    plan's local block ids are mapped to buffers at issue time.  Call
    :meth:`canonicalize` before reading the result: it moves the halves back
    to buffer 2 slot + half, i.e. rows [s B, (s+1) B) = slot s.

    ``exchange="spread"`` (parallel/spread.py) moves every half over all
    xGMI links in two relayed phases instead of the one direct link; the
    data that arrives is identical, bit for bit.

    Exchange timing (``timing=True``, device runs with a stream-ordered
    communicator): every half exchange is bracketed on the comm stream by two
    timing events (issue after its producers' events, arrival of both
    directions); every task is bracketed on its stream (start after its waits,
    end), and every consumer records an event just before it waits for an
    arrival.  :meth:`comm_summary` reports ``comm_ms`` (sum of exchange
    spans) and ``exposed_comm_ms``: the time during which some compute stream
    waited for an arrival while no task ran on any compute stream
    (:func:`exposed_time`) -- the part of the exchanges on the critical path."""

    def __init__(self, comm, streams, At, Vt, D, k: int, W: int, tour, timing: bool = False,
                 parts: int = 2, exchange: str = "direct"):
        if parts != 2:
            raise ValueError("the pipelined executor moves super-blocks in halves")
        self.comm, self.streams = comm, streams
        self.At, self.Vt, self.D = At, Vt, D
        self.k, self.W, self.tour = k, W, tour
        self.parts = parts
        self.hB = k // parts * W
        self.layout = HalfLayout(spares=comm.distributed)
        if At.shape[0] != self.layout.nbuf * self.hB or D.shape[0] != At.shape[0]:
            raise ValueError(f"storage must hold {self.layout.nbuf} half buffers of {self.hB} "
                             f"columns, got {At.shape[0]}")
        dev = At.device
        self.cuda = dev.type == "cuda"
        self.dev_pairs = {}  # (item index, buffers of its halves) -> device pairs
        self._groups = {}
        self.comm_stream = torch.cuda.Stream(dev) if self.cuda and comm.distributed else None
        self.stream_ordered = self.cuda and getattr(comm, "async_device", False)
        self.timing = bool(timing) and self.stream_ordered
        self._t0 = None
        self._spans = []     # (issue event, arrival event) per half exchange
        self._waits = []     # (consumer-ready event, arrival event) per consume
        self._busy = []      # (start event, end event) per task
        self.bytes_sent = 0
        self.bytes_relayed = 0
        self.exchanges = 0   # half exchanges issued (counted with or without timing)
        # the simulated communicator models a spread exchange by its time only
        self.exchange_choice = None
        if (exchange == "auto" and comm.world >= 4 and self.stream_ordered
                and getattr(comm, "backend", "") != "sim"):
            # RCCL from 4 GPUs: time both exchanges on this node's links once
            # (first tournament round, the real half-buffer sizes) and keep the
            # faster; the data delivered is bitwise the same either way
            exchange, self.exchange_choice = calibrate_exchange(
                comm, tour, [tuple(At[self._buf(0)].shape)] +
                ([tuple(Vt[self._buf(0)].shape)] if Vt is not None else []), At.dtype, dev)
        self.exchange = resolve_exchange(exchange, comm.world)
        self.spread = self.exchange == "spread" and getattr(comm, "backend", "") != "sim"
        self._relay = {}     # message index -> (P, chunk) relay buffer
        self._spread_ops = {}

    @staticmethod
    def storage_columns(B: int, distributed: bool) -> int:
        """Columns (rows of At) a rank allocates: 2B, plus a spare half per
        half index when exchanges happen."""
        return (3 if distributed else 2) * B

    def _buf(self, b: int) -> slice:
        return slice(b * self.hB, (b + 1) * self.hB)

    def _pairs(self, i: int, task: Task):
        bufs = tuple(self.layout.loc[s][h] for s, h in task.halves)
        key = (i, bufs)
        t = self.dev_pairs.get(key)
        if t is None:
            phys = self.layout.table(self.k)[task.pairs]
            t = torch.from_numpy(np.ascontiguousarray(phys)).to(self.At.device)
            self.dev_pairs[key] = t
        return t

    def _event(self):
        return torch.cuda.Event(enable_timing=self.timing)

    def run_merged(self, plan: SweepPlan, run_steps) -> float:
        """One sweep on ONE rank (no exchanges) with the two chains merged:
        the parallel task pairs of the plan (rr0 + rr1, T00 + T11, T01 + T10;
        ``issue_groups``) become single launches of twice the pairs per step
        on the caller's stream.  Same block pairs in the same step order as
        :meth:`run` (the sweep count is the two-chain plan's), but every
        step's Gram, EVD, Q build and apply cover both chains: the EVD latency
        is paid once per step instead of being left to the other chain to
        hide (on one GPU a 64-pair step alone took 636-655 us, the two
        overlapped chains 678 us per 64 pairs; profiles/r4_steps)."""
        if self.comm.distributed:
            raise RuntimeError("run_merged is the single-rank issue")
        index = {id(it): i for i, it in enumerate(plan.items)}
        for it in issue_groups(plan.items, True):
            tasks = it if isinstance(it, tuple) else (it,)
            if len(tasks) == 2 and list(tasks[0].modes) == list(tasks[1].modes) and \
                    tasks[0].pairs.shape == tasks[1].pairs.shape:
                pairs = torch.cat([self._pairs(index[id(t)], t) for t in tasks], dim=1)
                run_steps(pairs.contiguous(), tasks[0].modes, 0)
                continue
            for t in tasks:
                run_steps(self._pairs(index[id(t)], t), t.modes, 0)
        return 0.0

    def run(self, plan: SweepPlan, run_steps, phys, merge: bool = False) -> float:
        """Execute one sweep.  ``run_steps(pairs, modes, slot)`` enqueues block
        steps on the current stream; ``merge``: the joint task groups as
        single launches (the merged issue with exchanges; measured slower
        there).  ``phys`` (per-GPU placement of whole super-blocks) is
        updated after both halves of a round arrived.  Returns host seconds
        spent issuing/blocking on exchanges."""
        import time

        if self.cuda:  # everything enqueued on the caller's stream so far (metric
            # reset, initial norms) happens before any task or exchange
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(self.At.device))
            if self.timing and self._t0 is None:
                self._t0 = torch.cuda.Event(enable_timing=True)
                self._t0.record(torch.cuda.current_stream(self.At.device))
            for s in self.streams + ([self.comm_stream] if self.comm_stream else []):
                s.wait_event(ready)
        last = {}       # (slot, half) -> [events of tasks since last exchange]
        pending = {}    # (slot, half) -> arrival event / works, not yet waited for
        t_comm = 0.0
        halves_done = {}
        index = {id(it): i for i, it in enumerate(plan.items)}
        groups = self._groups.get((id(plan), merge))
        if groups is None:
            groups = issue_groups(plan.items, merge)
            self._groups[(id(plan), merge)] = groups
        for it in groups:
            if isinstance(it, Send):
                tc = time.perf_counter()
                self._send(it, last, pending)
                halves_done[it.round] = halves_done.get(it.round, 0) + 1
                if halves_done[it.round] == self.parts:
                    self._update_phys(it.round, phys)
                t_comm += time.perf_counter() - tc
                continue
            tasks = it if isinstance(it, tuple) else (it,)
            if not self.cuda:
                for t in tasks:
                    for hv in t.halves:
                        self._consume(hv, pending)
                    run_steps(self._pairs(index[id(t)], t), t.modes, t.stream)
                continue
            pairs = [self._pairs(index[id(t)], t) for t in tasks]
            starts = []
            for t in tasks:  # dependencies, on each task's own stream
                s = self.streams[t.stream]
                with torch.cuda.stream(s):
                    for hv in t.halves:
                        for ev in last.get(hv, ()):
                            s.wait_event(ev)
                        self._consume(hv, pending)
                    if self.timing:
                        st = self._event()
                        st.record(s)
                        starts.append(st)
            if len(tasks) == 2 and merge and list(tasks[0].modes) == list(tasks[1].modes) \
                    and pairs[0].shape == pairs[1].shape:
                # both tasks as ONE launch per step on the first task's stream,
                # after the second task's dependencies too (merged issue)
                a, b = tasks
                sa, sb = self.streams[a.stream], self.streams[b.stream]
                joined = self._event()
                joined.record(sb)
                sa.wait_event(joined)
                with torch.cuda.stream(sa):
                    run_steps(torch.cat(pairs, dim=1).contiguous(), a.modes, a.stream)
                done = self._event()
                done.record(sa)
                sb.wait_event(done)
            else:  # one task, or a group that cannot merge: each task on its
                # own stream (as run_merged falls back)
                for q, t in enumerate(tasks):
                    with torch.cuda.stream(self.streams[t.stream]):
                        run_steps(pairs[q], t.modes, t.stream)
            for q, t in enumerate(tasks):
                ev = self._event()
                ev.record(self.streams[t.stream])
                if self.timing:
                    self._busy.append((starts[q], ev))
                for hv in t.halves:
                    last.setdefault(hv, []).append(ev)
        if self.cuda:
            main = torch.cuda.current_stream(self.At.device)
            for s in self.streams + ([self.comm_stream] if self.comm_stream else []):
                main.wait_stream(s)
        return t_comm

    def _send(self, it: Send, last, pending):
        comm, tour = self.comm, self.tour
        g = comm.rank
        r, x, hh = it.round, it.slot, it.half
        dst, src = int(tour.send_to[r, g]), int(tour.recv_from[r, g])
        out_b, in_b = self.layout.loc[x][hh], self.layout.spare[hh]
        so, si = self._buf(out_b), self._buf(in_b)
        sends = [(self.At[so], dst), (self.D[so], dst)]
        recvs = [(self.At[si], src), (self.D[si], src)]
        if self.Vt is not None:
            sends.append((self.Vt[so], dst))
            recvs.append((self.Vt[si], src))
        self.bytes_sent += sum(t.numel() * t.element_size() for t, _ in sends)
        self.exchanges += 1
        if not comm.distributed:
            raise RuntimeError("exchange on a single rank")
        # from here on (host program order) the half lives in the received buffer
        self.layout.loc[x][hh], self.layout.spare[hh] = in_b, out_b
        phases = [(sends, recvs)]
        if self.spread:
            phases = self._spread_phases(r, [t for t, _ in sends], [t for t, _ in recvs])
        if not self.cuda:
            for ps, pr in phases:
                comm.sendrecv(ps, pr)
            last.pop((x, hh), None)
            return
        cs = self.comm_stream
        for ev in last.pop((x, hh), ()):
            cs.wait_event(ev)
        if not self.stream_ordered:
            # gloo on device tensors (one-GPU rehearsal of the multi-rank
            # path) does not order its copies after other streams: make the
            # data ready on the host side first.  RCCL needs none of this.
            cs.synchronize()
            with torch.cuda.stream(cs):
                if len(phases) > 1:
                    # relayed: both phases complete here -- the relay buffers
                    # are reused by the next exchange, which this host-driven
                    # path would otherwise start while forwards still read them
                    for ps, pr in phases:
                        for w in comm.isendrecv(ps, pr):
                            w.wait()
                        torch.cuda.synchronize(self.At.device)
                    pending[(x, hh)] = []
                else:
                    pending[(x, hh)] = comm.isendrecv(sends, recvs)
            return
        # Stream-ordered (RCCL): the comm stream issues the grouped send/recv
        # after the producers' events, then waits (device-side) for both
        # directions; consumers wait on ONE arrival event -- no host sync.
        # The receive buffer's last readers were waited for by the exchange
        # that freed it, earlier on this same stream.
        with torch.cuda.stream(cs):
            t_issue = None
            if self.timing:
                t_issue = torch.cuda.Event(enable_timing=True)
                t_issue.record(cs)
            for ps, pr in phases:  # phase 2 is stream-ordered after phase 1
                for w in comm.isendrecv(ps, pr):
                    w.wait()
            arrived = self._event()
            arrived.record(cs)
        if self.timing:
            self._spans.append((t_issue, arrived))
        pending[(x, hh)] = arrived

    def _spread_phases(self, r: int, outs: list, ins: list) -> list:
        """[(sends, recvs)] of the two relayed phases of round r's exchange
        (parallel/spread.py) on flat views of the outgoing / incoming half
        buffers; the norms (tiny) go directly."""
        comm = self.comm
        P = comm.world
        flat_out = [t.reshape(-1) for t in outs]
        flat_in = [t.reshape(-1) for t in ins]
        sizes = [t.numel() for t in flat_out]
        flags = [t.dim() == 2 for t in outs]  # At / Vt spread, D direct
        key = (r, tuple(sizes))
        ops = self._spread_ops.get(key)
        if ops is None:
            ops = spread_ops(comm.rank, self.tour.send_to[r], sizes, flags)
            self._spread_ops[key] = ops

        def relay(mi):
            buf = self._relay.get(mi)
            if buf is None:
                buf = torch.empty(P, relay_chunk(sizes[mi], P), dtype=flat_out[mi].dtype,
                                  device=flat_out[mi].device)
                self._relay[mi] = buf
            return buf

        def tensor(op):
            mi, (a, b), peer, where = op
            if where == "out":
                return flat_out[mi][a:b], peer
            if where == "in":
                return flat_in[mi][a:b], peer
            return relay(mi)[where[1], :b - a], peer

        p1 = ([tensor(o) for o in ops.p1_send], [tensor(o) for o in ops.p1_recv])
        p2 = ([tensor(o) for o in ops.p2_send], [tensor(o) for o in ops.p2_recv])
        self.bytes_relayed += sum(t.numel() * t.element_size() for t, _ in p2[0])
        return [p1, p2]

    def _consume(self, hv, pending):
        got = pending.pop(hv, None)
        if got is None:
            return
        if self.stream_ordered:
            s = torch.cuda.current_stream(self.At.device)
            if self.timing:
                ready = torch.cuda.Event(enable_timing=True)
                ready.record(s)
                self._waits.append((ready, got))
            s.wait_event(got)
        else:
            for w in got:
                w.wait()  # gloo: blocks the host until both directions are done
            if self.cuda:
                torch.cuda.synchronize(self.At.device)

    def canonicalize(self):
        """Move every half back to buffer 2 slot + half (enqueued on the
        current stream, which :meth:`run` made wait for every other stream)."""
        for src, dst in self.layout.moves_to_canonical():
            for t in (self.At, self.Vt, self.D):
                if t is not None:
                    t[self._buf(dst)].copy_(t[self._buf(src)])

    def comm_summary(self) -> dict:
        """Exchange counts and bytes of every sweep run so far; with timing
        on also the exchange times (synchronises).  The timing fields are
        absent when timing is off."""
        out = {"exchanges": int(self.exchanges), "bytes_sent": int(self.bytes_sent),
               "exchange": self.exchange, "bytes_relayed": int(self.bytes_relayed),
               "timing": bool(self.timing and self._t0 is not None)}
        if self.exchange_choice is not None:
            out["exchange_choice"] = self.exchange_choice
        elif self.exchange == "spread":
            out["exchange_choice"] = "spread: model-based default (parallel/spread.py)"
        if not out["timing"]:
            return out
        torch.cuda.synchronize(self.At.device)
        t0 = self._t0
        out["comm_ms"] = round(sum(a.elapsed_time(b) for a, b in self._spans), 3)
        waits = [(t0.elapsed_time(r), t0.elapsed_time(a)) for r, a in self._waits]
        busy = [(t0.elapsed_time(a), t0.elapsed_time(b)) for a, b in self._busy]
        out["exposed_comm_ms"] = round(exposed_time(waits, busy), 3)
        # the round-2 figure (sum over consumers of arrival - consumer ready),
        # which double-counts shared arrivals and waits under other compute
        out["consumer_wait_sum_ms"] = round(sum(max(0.0, b - a) for a, b in waits), 3)
        return out

    def _update_phys(self, r: int, phys):
        tour, P = self.tour, self.comm.world
        old = [[phys[h][0], phys[h][1]] for h in range(P)]
        for h in range(P):
            src_h = int(tour.recv_from[r, h])
            phys[h][int(tour.xslot[r, h])] = old[src_h][int(tour.xslot[r, src_h])]
