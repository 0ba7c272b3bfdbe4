"""Half-block pipelined sweep plan (parallel/pipeline.py): coverage and
exchange structure on CPU."""
import os
from pathlib import Path

import pytest

import svdj
pipeline = svdj.parallel.pipeline
schedule = svdj.parallel.schedule


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("k", [2, 4, 6])
def test_every_block_pair_meets_once(P, k):
    tour = schedule.tournament(P)
    plans = [pipeline.sweep_plan(P, k, tour.xslot[:, g]) for g in range(P)]
    pipeline.check_plan_coverage(plans, tour)


def test_sends_follow_last_use():
    """Half 0 of the next outgoing slot is sent after its last user in the
    round, and before anything of the next round touches it."""
    P, k = 4, 4
    tour = schedule.tournament(P)
    plan = pipeline.sweep_plan(P, k, tour.xslot[:, 0])
    items = plan.items
    for i, it in enumerate(items):
        if not isinstance(it, pipeline.Send):
            continue
        hv = (it.slot, it.half)
        prev = [j for j in range(i) if isinstance(items[j], pipeline.Task)
                and hv in items[j].halves and f"r{it.round - 1}." in items[j].name]
        later = [j for j in range(i + 1, len(items)) if isinstance(items[j], pipeline.Task)
                 and hv in items[j].halves]
        assert prev, it
        assert all(f"r{it.round}." in items[j].name or items[j].name.startswith("r" + str(it.round + 1))
                   or int(items[j].name[1:].split(".")[0]) > it.round - 1 for j in later[:1])


def test_odd_k_rejected():
    with pytest.raises(ValueError):
        pipeline.sweep_plan(2, 3, schedule.tournament(2).xslot[:, 0])


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("k", [2, 4, 6])
def test_joint_groups_keep_coverage(P, k):
    """Joint issue (the merged one-GPU launches) pairs independent tasks of
    different streams;
    the regrouped order (Sends moved after a pair) still meets every pair
    once and never moves a Send past a task that touches its half."""
    tour = schedule.tournament(P)
    plans = [pipeline.sweep_plan(P, k, tour.xslot[:, g]) for g in range(P)]
    regrouped = []
    for pl in plans:
        groups = pipeline.issue_groups(pl.items, True)
        pos = {id(x): i for i, x in enumerate(pl.items)}
        flat = []
        for g in groups:
            if isinstance(g, tuple):
                a, b = g
                assert a.stream != b.stream and not set(a.halves) & set(b.halves)
                for x in pl.items[pos[id(a)] + 1:pos[id(b)]]:  # Sends moved after the pair
                    assert isinstance(x, pipeline.Send) and (x.slot, x.half) not in b.halves
                flat += [a, b]
            else:
                flat.append(g)
        assert sorted(map(id, flat)) == sorted(map(id, pl.items))
        npairs = sum(isinstance(g, tuple) for g in groups)
        assert npairs >= (2 * P - 1) + 1 - (1 if P > 1 else 0)
        new = pipeline.SweepPlan(pl.P, pl.k)
        new.items = flat
        regrouped.append(new)
    pipeline.check_plan_coverage(regrouped, tour)
    assert pipeline.issue_groups(plans[0].items, False) == plans[0].items


def _native_plan(P, g):
    import ctypes
    import importlib
    import numpy as np
    b = importlib.import_module("svd-jacobi-mpi-cuda_amd._build")
    try:
        b.build_dist()
    except (FileNotFoundError, RuntimeError) as e:  # no hipcc / rccl in this environment
        pytest.skip(f"native distributed library not buildable here: {e}")
    lib = ctypes.CDLL(str(b.DIST_LIB))
    out = np.zeros((4096, 7), dtype=np.int32)
    n = lib.svdj_dist_plan(P, g, out.ctypes.data_as(ctypes.c_void_p), out.shape[0])
    assert n > 0
    return out[:n].tolist()


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
def test_native_plan_matches_python(P):
    """csrc/dist/svdj_dist.cpp builds the same sweep and issue order as the
    Python executor (sweep_plan + issue_groups) on every rank."""
    tour = schedule.tournament(P)

    def hv(x):
        return [s * 2 + h for s, h in x.halves]

    for g in range(P):
        groups = pipeline.issue_groups(pipeline.sweep_plan(P, 4, tour.xslot[:, g]).items, True)
        want = []
        for it in groups:
            if isinstance(it, pipeline.Send):
                want.append([2, it.round, it.slot, it.half, -1, -1, -1])
            elif isinstance(it, tuple):
                a, b_ = it
                want.append([1, a.stream, *hv(a), b_.stream, *hv(b_)])
            else:
                want.append([0, it.stream, *hv(it), -1, -1, -1])
        assert _native_plan(P, g) == want


def test_native_block_rule_matches_python():
    """bin/svdj_dist_main picks the block width with svdj_dist_choose_block,
    the Python solvers with models.block.choose_block: same rule."""
    import ctypes
    import importlib
    import torch
    b = importlib.import_module("svd-jacobi-mpi-cuda_amd._build")
    try:
        b.build_dist()
    except (FileNotFoundError, RuntimeError) as e:
        pytest.skip(f"native distributed library not buildable here: {e}")
    lib = ctypes.CDLL(str(b.DIST_LIB))
    choose = svdj.models.block.choose_block
    for dt, code in ((torch.float32, 0), (torch.float64, 1)):
        for world in (1, 2, 4, 8):
            for m, n in ((512, 512), (2048, 2048), (4096, 4096), (5000, 5000), (6144, 6144),
                         (8192, 8192), (12288, 12288), (16384, 16384), (32768, 8192),
                         (65536, 65536), (20000, 20000)):
                assert lib.svdj_dist_choose_block(code, world, m, n) == choose(dt, n // world, m), \
                    (dt, world, m, n)


def test_dist_lib_resolves_to_shared_object():
    """ops._native.dist_lib() must load libsvdj_dist.so -- never the
    bin/svdj_dist_main launcher that build_dist() also produces (round-2
    GPU-suite failure: 'cannot dynamically load executable')."""
    import importlib
    b = importlib.import_module("svd-jacobi-mpi-cuda_amd._build")
    nat = importlib.import_module("svd-jacobi-mpi-cuda_amd.ops._native")
    try:
        built = b.build_dist()
    except (FileNotFoundError, RuntimeError) as e:
        pytest.skip(f"native distributed library not buildable here: {e}")
    assert built == b.DIST_LIB and built.suffix == ".so"
    assert b.DIST_DRIVER_BIN.exists() and b.DIST_DRIVER_BIN != built
    path = nat.dist_lib_path()
    want = Path(os.environ["SVDJ_DIST_LIB"]) if os.environ.get("SVDJ_DIST_LIB") else b.DIST_LIB
    assert path == want and path.name == "libsvdj_dist.so"  # (the ASan run overrides)
    lib = nat.dist_lib()  # the exact loader bench.py --engine native uses
    assert hasattr(lib, "svdj_dist_solve") and hasattr(lib, "svdj_dist_comm_init")


def test_chain_count_validated():
    """Only the blocking (1) and pipelined two-chain (2) executors exist: any
    other value is rejected when the config is built, not mid-solve."""
    for bad in (0, 3, 4):
        with pytest.raises(ValueError):
            svdj.SolverConfig(chains=bad)
    with pytest.raises(ValueError):
        pipeline.sweep_plan(2, 4, schedule.tournament(2).xslot[:, 0], chains=4)


def test_half_layout_receive_in_place_and_canonicalize():
    """Exchanges receive into the spare of their half index and swap; after
    any exchange sequence the canonicalising moves bring every (slot, half)
    back to buffer 2 slot + half, never overwriting live data."""
    import random
    rnd = random.Random(3)
    for trial in range(200):
        lay = pipeline.HalfLayout(spares=True)
        content = {b: None for b in range(6)}  # buffer -> (slot, half) data tag
        for s in range(2):
            for h in range(2):
                content[lay.loc[s][h]] = (s, h, 0)
        gen = {(s, h): 0 for s in range(2) for h in range(2)}
        for _ in range(rnd.randrange(0, 12)):
            x, h = rnd.randrange(2), rnd.randrange(2)
            out_b, in_b = lay.loc[x][h], lay.spare[h]
            assert {lay.loc[0][h], lay.loc[1][h], lay.spare[h]} == {h, 2 + h, 4 + h}
            gen[(x, h)] += 1
            content[in_b] = (x, h, gen[(x, h)])   # the received replacement
            lay.loc[x][h], lay.spare[h] = in_b, out_b
        want = {(s, h): content[lay.loc[s][h]] for s in range(2) for h in range(2)}
        for src, dst in lay.moves_to_canonical():
            content[dst] = content[src]
        assert lay.canonical()
        for s in range(2):
            for h in range(2):
                assert content[2 * s + h] == want[(s, h)]


def test_exposed_time_counts_each_moment_once():
    """exposed_time: a wait counts only while no task runs on any stream, and
    overlapping waits (two consumers of one arrival) count once."""
    ex = pipeline.exposed_time
    assert ex([(0, 10)], []) == 10
    assert ex([(0, 10), (2, 10)], []) == 10            # two consumers, one arrival
    assert ex([(0, 10)], [(0, 4), (6, 8)]) == 4        # other stream busy 6 of 10
    assert ex([(0, 10)], [(-5, 20)]) == 0              # fully hidden
    assert ex([(0, 3), (5, 8)], [(2, 6)]) == 4
    assert ex([], [(0, 1)]) == 0


def test_native_inner_order_rule_matches_python():
    """inner_order="auto": the native drivers (svdj_choose_inner_order in
    libsvdj_hip) pick the cross-step EVD by the same rule as
    models.block.choose_inner_order."""
    import torch
    choose = svdj.models.block.choose_inner_order
    lib = svdj.ops.hip_lib()
    code = {1: "bipartite", 2: "cross"}
    for dt, dcode in ((torch.float32, 0), (torch.float64, 1)):
        for W in (32, 64):
            for pairs in (1, 4, 8, 16, 17, 32, 64, 128, 256):
                assert code[lib.svdj_choose_inner_order(dcode, W, pairs)] == choose(W, pairs, dt), \
                    (dt, W, pairs)


def test_native_mma_rule_matches_python():
    """mma="auto": the native drivers and engine (svdj_choose_mma in
    libsvdj_hip) pick the apply's matrix-core mode by the same rule as
    models.block.choose_mma / SolverConfig.resolved_mma."""
    import torch
    choose = svdj.models.block.choose_mma
    lib = svdj.ops.hip_lib()
    code = {0: "native", 1: "bf16x6"}
    for dt, dcode in ((torch.float32, 0), (torch.float64, 1)):
        for W in (32, 64):
            assert code[lib.svdj_choose_mma(dcode, W)] == choose(dt, W), (dt, W)
    cfg = svdj.SolverConfig()
    A = torch.zeros(4, 4, dtype=torch.float32)
    assert cfg.resolved_mma(A, 64) == "bf16x6" and cfg.resolved_mma(A, 32) == "native"
    assert cfg.resolved_mma(A.double(), 64) == "native"
    assert svdj.SolverConfig(mma="native").resolved_mma(A, 64) == "native"


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("k", [4, 8, 12])
def test_quad_plan_meets_every_pair_once(P, k):
    """Quad order (two cross steps fused per quad): the same coverage, and
    every mode-4/5 step pair holds quads in the kernels' orientation."""
    tour = schedule.tournament(P)
    plans = [pipeline.sweep_plan(P, k, tour.xslot[:, g], quad=True) for g in range(P)]
    pipeline.check_plan_coverage(plans, tour)
    for it in plans[0].items:
        if isinstance(it, pipeline.Task):
            schedule.check_quad_steps(it.pairs, it.modes)
            assert 4 in it.modes


def test_quad_plan_needs_multiple_of_4():
    with pytest.raises(ValueError):
        pipeline.sweep_plan(1, 6, schedule.tournament(1).xslot[:, 0], quad=True)


def test_dist_id_file_handshake(tmp_path, monkeypatch):
    """Host part of the native engine's RCCL bootstrap (svdj_dist_id_file,
    ADVICE r4): a rank accepts only a FRESH id file carrying ITS job token --
    SVDJ_JOB_TOKEN, or torchrun's run id joined with the restart count, so an
    elastic restart (or a reused --rdzv-id after a crash) never picks up the
    dead attempt's id."""
    import ctypes
    import os
    import time

    from svdj.ops import _native as nat

    lib = nat.dist_lib()
    path = str(tmp_path / "job.id").encode()
    blob = bytes(range(128))  # sizeof(ncclUniqueId)

    def publish():
        b = ctypes.create_string_buffer(blob, 128)
        assert lib.svdj_dist_id_file(0, path, 5.0, b, 128) == 0

    def read(timeout=5.0):
        b = ctypes.create_string_buffer(128)
        rc = lib.svdj_dist_id_file(1, path, timeout, b, 128)
        return rc, b.raw

    monkeypatch.delenv("TORCHELASTIC_RUN_ID", raising=False)
    monkeypatch.setenv("SVDJ_JOB_TOKEN", "job-a")
    publish()
    assert read() == (0, blob)
    monkeypatch.setenv("SVDJ_JOB_TOKEN", "job-b")  # another job's file: refused
    assert read(timeout=0.3)[0] == -2
    # torchrun: same run id, another restart attempt -> refused; same attempt -> read
    monkeypatch.delenv("SVDJ_JOB_TOKEN")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "rdzv-1")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    publish()
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    assert read(timeout=0.3)[0] == -2
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    assert read() == (0, blob)
    # a leftover older than the window is refused even with the right token
    old = time.time() - 3600
    os.utime(path.decode(), (old, old))
    assert read(timeout=0.3)[0] == -2
    assert lib.svdj_dist_id_file(1, path, 0.3, ctypes.create_string_buffer(64), 64) == -2  # size
    # freshness counts from the reading process's start, not from
    # its call -- a tokenless peer that arrives late (slow GPU init) still
    # accepts the id its rank 0 published after the launch.  Published 29 s
    # before this process started: inside the 30 s window of the launch, but
    # older than 30 s before this call (the test process has run > 1 s).
    monkeypatch.delenv("TORCHELASTIC_RUN_ID")
    monkeypatch.delenv("TORCHELASTIC_RESTART_COUNT")
    publish()
    import psutil
    t_start = psutil.Process().create_time()
    assert time.time() - t_start > 1.0
    os.utime(path.decode(), (t_start - 29, t_start - 29))
    assert read(timeout=0.5) == (0, blob)
    os.utime(path.decode(), (t_start - 40, t_start - 40))  # before the window: a leftover
    assert read(timeout=0.3)[0] == -2


@pytest.mark.parametrize("k,quad", [(8, False), (8, True), (16, True), (128, True)])
def test_native_merged_lists_match_python(k, quad):
    """One GPU: the native engine's merged launches (svdj_dist_merged_lists)
    carry the pair lists and step modes of PipelineExecutor.run_merged --
    the two parallel tasks of each issue group side by side, step by step --
    in plain and in quad order (k = 128: the 16384^2 headline's plan)."""
    import ctypes

    import numpy as np

    from svdj.ops import _native as nat

    lib = nat.dist_lib()
    plan = pipeline.sweep_plan(1, k, schedule.tournament(1).xslot[:, 0], quad=quad)
    want_pairs, want_modes, want_meta = [], [], []
    for it in pipeline.issue_groups(plan.items, True):
        if not isinstance(it, tuple):
            continue
        a, b_ = it
        assert list(a.modes) == list(b_.modes) and a.pairs.shape == b_.pairs.shape
        want_meta += [sum(p.size for p in want_pairs), a.pairs.shape[0], 2 * a.pairs.shape[1]]
        want_pairs.append(np.concatenate([a.pairs, b_.pairs], axis=1).ravel())
        want_modes += list(a.modes)
    assert len(want_meta) == 9  # rr0 + rr1, T00 + T11, T01 + T10
    i32p = ctypes.POINTER(ctypes.c_int32)
    pairs = np.zeros(4 * k * k, np.int32)
    modes = np.zeros(4 * k, np.int32)
    meta = np.zeros(9, np.int32)
    n = lib.svdj_dist_merged_lists(k, int(quad), 0, pairs.ctypes.data_as(i32p), pairs.size,
                                   modes.ctypes.data_as(i32p), modes.size, meta.ctypes.data_as(i32p))
    want = np.concatenate(want_pairs)
    assert n == want.size
    assert np.array_equal(pairs[:n], want)
    assert modes[:len(want_modes)].tolist() == want_modes
    assert meta.tolist() == want_meta


def test_native_issue_rules_match_python(monkeypatch):
    """Quad steps and the merged one-GPU issue are decided by the same rules in
    libsvdj_dist (svdj_dist_issue_rules) and the Python engine
    (models.block.resolve_quad, parallel.distributed.choose_merged)."""
    import ctypes

    import torch

    from svdj.models.block import resolve_quad
    from svdj.ops import _native as nat
    from svdj.parallel.distributed import choose_merged

    import itertools

    lib = nat.dist_lib()
    q, mg = ctypes.c_int32(), ctypes.c_int32()
    cases = itertools.product(
        (1, 2, 8), ((torch.float32, 0), (torch.float64, 1)), (32, 64),
        (("native", 0), ("bf16x6", 1), ("bf16x3", 2)),
        ((8, 16384), (16, 8192), (16, 16384), (30, 32768), (32, 4096), (32, 16384), (62, 8192),
         (64, 8192), (128, 16384), (256, 65536)),
        (("auto", 0), ("on", 1), ("off", 2)))
    cases = list(cases)
    # the A/B override (SVDJ_DEBUG merge=0/1) acts on one GPU only, in both engines
    for dbg in (None, "merge=0", "merge=1"):
        if dbg is None:
            monkeypatch.delenv("SVDJ_DEBUG", raising=False)
        else:
            monkeypatch.setenv("SVDJ_DEBUG", dbg)
        for world, (dt, code), W, (mma, mcode), (k, m_pad), (mode, mc) in cases:
            where = (dbg, world, dt, W, mma, k, mode)
            rc = lib.svdj_dist_issue_rules(world, code, W, mcode, k, m_pad, mc,
                                           ctypes.byref(q), ctypes.byref(mg))
            try:
                want_q = resolve_quad(mode, dt, W, mma, k, world, m_pad)
            except ValueError:
                assert rc < 0, where
                continue
            assert rc == 0, where
            want_m = choose_merged(world, k, want_q)
            assert (bool(q.value), bool(mg.value)) == (want_q, want_m), where
            if world > 1:
                assert not want_m, where

def test_native_geometry_matches_python_and_pads_for_quad_steps():
    """svdj_dist_geometry and DistributedBlockJacobi.geometry agree on every
    shape; a column count that would land on k % 4 == 2 where the quad rule
    holds is padded to the next k % 4 == 0 (4097 columns on one GPU: 68 -> 72
    blocks, so quad steps run), but not for fp64 (no quad steps) nor where
    the rule would not take quad steps anyway (fewer than 12 pairs per step);
    multiples of the quad granule are never padded."""
    import ctypes
    import itertools
    import types

    import torch

    from svdj.ops import _native as nat
    from svdj.parallel import DistributedBlockJacobi

    lib = nat.dist_lib()
    out = [ctypes.c_int32() for _ in range(4)]

    def native(P, m, n, W, code):
        assert lib.svdj_dist_geometry(P, m, n, W, code, *[ctypes.byref(o) for o in out]) == 0
        return tuple(o.value for o in out)

    def python(P, m, n, W, dt):
        s = DistributedBlockJacobi(svdj.SolverConfig(block=W), types.SimpleNamespace(world=P))
        g = s.geometry(m, n, dt)
        return g["B"], g["ncols"], g["m_pad"], g["n_v"]

    dts = ((torch.float32, 0), (torch.float64, 1), (torch.float32, 2))
    for P, n, W, (dt, code) in itertools.product((1, 2, 4, 8), (100, 2300, 4097, 4352, 8200, 16400,
                                                                 16384, 33000), (32, 64), dts):
        for m in (n, 2 * n, 17000):
            if m < n:
                continue
            assert native(P, m, n, W, code) == python(P, m, n, W, dt), (P, m, n, W, code)
    assert native(1, 4500, 4097, 64, 0)[0] // 64 == 36   # padded: quad steps
    assert native(1, 4500, 4097, 64, 1)[0] // 64 == 34   # fp64: not padded
    assert native(1, 16400, 16400, 64, 0)[0] // 64 == 132
    assert native(1, 4096, 4096, 64, 0)[0] // 64 == 32   # exact granule: unchanged
    assert native(8, 16384, 16384, 64, 0)[0] // 64 == 16
    assert native(2, 8200, 8200, 64, 0)[0] // 64 == 36   # 17 -> 18 pairs per step: quad
    assert native(8, 16400, 16400, 64, 0)[0] // 64 == 18  # 9 pairs: no quad, no padding


def test_quad_and_merge_rules_pin_the_measured_choices():
    """The measured decisions (profiles/r5_quad2): 16384^2 fp32 W = 64 runs
    quad steps on 1, 2 and 4 GPUs (64 / 32 / 16 pairs per chain step, 16384
    rows) but not on 8 (8 pairs); 8192^2 on one GPU does (32 pairs);
    4096^2 on one GPU does too, merged (16 pairs: round 6, profiles/r6_issue);
    from 32 pairs the one-GPU solve keeps the two chains apart (round 6,
    profiles/r6_merge: with the shared-GPU apply grid they beat merging);
    since the quad apply leaves the concurrent chain CUs (round 6,
    profiles/r6_grid) quad steps win from 12 pairs per step on columns of any
    length (8192^2 on two GPUs, 12288^2 on four), not yet at 8 pairs
    (16384^2 on 8 GPUs, 8192^2 on 4: ties or within 5 %)."""
    import torch

    from svdj.models.block import resolve_quad
    from svdj.parallel.distributed import choose_merged

    def plan(n, P, m=None):
        m_pad = m or n
        k = n // (2 * P) // 64  # W-blocks per super-block
        q = resolve_quad("auto", torch.float32, 64, "bf16x6", k, P, m_pad)
        return q, choose_merged(P, k, q)

    assert plan(16384, 1) == (True, False)
    assert plan(16384, 2) == (True, False)
    assert plan(16384, 4) == (True, False)
    assert plan(16384, 8) == (False, False)
    assert plan(4096, 1) == (True, True)
    assert plan(8192, 2) == (True, False)
    assert plan(12288, 4) == (True, False)
    assert plan(8192, 4) == (False, False)
    assert plan(8192, 1) == (True, False)
    assert plan(32768, 8) == (True, False)
    assert not resolve_quad("auto", torch.float64, 64, "native", 128, 1, 16384)
