"""Quad steps (csrc/hip/block.hip "quad step") and the kernel variants that
are selected by the pair count of a step, against the fp64 torch reference.

Reference: the per-pair host solve these steps replace, main.cu:685-766
(V accumulation main.cu:749-758); the Givens kernel main.cu:139-147.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _orth_blocks(nb, W, m, m_pad, seed):
    """nb internally orthogonal W-column blocks (cross steps start from such
    blocks), column norms graded 1..3 and scaled per block (equal norms in
    two blocks make the first bipartite rotations exact 45-degree ties whose
    direction is decided by rounding), as At (nb*W, m_pad) fp64."""
    g = torch.Generator().manual_seed(seed)
    A64 = torch.zeros(nb * W, m_pad, dtype=torch.float64)
    A64[:, :m] = torch.rand(nb * W, m, generator=g, dtype=torch.float64) - 0.3
    for b in range(nb):
        q, _ = torch.linalg.qr(A64[b * W:(b + 1) * W, :m].t())
        sc = torch.linspace(1, 3, W, dtype=torch.float64) * (1 + 0.37 * b / nb)
        A64[b * W:(b + 1) * W, :m] = (q * sc).t()
    return A64


def _quad_pairs(svdj, nb):
    """The two steps of the first super-step of quad_round_robin(nb)."""
    pr = svdj.parallel.schedule.quad_round_robin(nb)
    return torch.from_numpy(pr[1:3].copy())


def test_quad_step_matches_reference(svdj, cuda):
    """GPU quad step (GRAM_QUAD, two cross EVDs, Gram-space update, fp64 T,
    K = 256 split-bf16 apply) vs ops.reference.quad_step in fp64 on a small
    well-separated case: same rotation count and convergence value, A, V and D
    to fp32 level.  (With many pairs, fp32 rounding of the couplings moves
    near-degenerate rotation angles far more than rounding: those cases are
    compared against the GPU's own two cross steps below.)"""
    K, R = svdj.ops.kernels, svdj.ops.reference
    W, nb, m = 64, 8, 500
    n, m_pad = nb * W, 512
    A64 = _orth_blocks(nb, W, m, m_pad, seed=11)
    At = A64.float().to(cuda)
    Vt = torch.zeros(n, 256, dtype=torch.float32, device=cuda)
    g = torch.Generator().manual_seed(5)
    Vt[:, :] = (torch.rand(n, 256, generator=g) - 0.5).to(cuda)  # any rows: V is rotated likewise
    D = K.col_norms2(At, m_pad)
    pairs = _quad_pairs(svdj, nb)
    At64, Vt64, D64 = At.double().cpu(), Vt.double().cpu(), D.double().cpu()
    metric = K.new_metric(cuda)
    K.block_steps(At, Vt, D, m_pad, pairs.to(cuda), W, [4, 5], 1e-6, 1, metric, mma="bf16x6")
    mx_ref, nrot_ref = R.quad_step(At64, Vt64, D64, pairs[0], pairs[1], W, 1e-6, 1)
    mx, nrot = K.read_metric(metric)
    assert nrot == nrot_ref == nb
    assert math.isclose(mx, mx_ref, rel_tol=1e-3)
    rt = 2e-4
    torch.testing.assert_close(At.double().cpu()[:, :m], At64[:, :m], rtol=rt, atol=rt)
    torch.testing.assert_close(Vt.double().cpu(), Vt64, rtol=rt, atol=rt)
    torch.testing.assert_close(D.double().cpu(), D64, rtol=rt, atol=rt)


def _two_step_runs(svdj, cuda, nb, m, inner, modes_list, seed=3):
    K = svdj.ops.kernels
    W = 64
    m_pad = (m + 127) // 128 * 128
    A64 = _orth_blocks(nb, W, m, m_pad, seed=seed)
    pairs = _quad_pairs(svdj, nb).to(cuda)
    outs = []
    for modes in modes_list:
        At = A64.float().to(cuda)
        Vt = torch.zeros(nb * W, nb * W, dtype=torch.float32, device=cuda)
        K.set_identity(Vt, nb * W)
        D = K.col_norms2(At, m_pad)
        metric = K.new_metric(cuda)
        K.block_steps(At, Vt, D, m_pad, pairs, W, modes, 1e-6, inner, metric, mma="bf16x6")
        outs.append((At.double().cpu(), Vt.double().cpu(), D.double().cpu(), K.read_metric(metric)))
    return A64, outs


@pytest.mark.parametrize("nb,m,inner", [(16, 700, 1), (16, 700, 3), (128, 256, 1)])
def test_quad_step_equals_two_cross_steps(svdj, cuda, nb, m, inner):
    """A quad step is the two cross steps it fuses (mode 3, data Gram for the
    second) to fp32 rounding: the Gram-space couplings are exact.  nb = 128 is
    64 pairs (32 quads) per step, the 1-GPU geometry.  Also: V stays
    orthogonal and A = A0 V on the touched columns.

    The quad Gram runs on split-bf16 MFMAs (gram_quad_kernel, products exact
    to 2^-26), the cross steps' Gram on f32 MFMAs: both fp32-accurate, but
    rounded differently.  With one inner EVD sweep the results agree column
    by column; with three, the near-degenerate rotation angles the EVD
    converges on are ill-conditioned in the couplings (the test's blocks have
    graded, close norms; the D of a pair whose EVD stops before it converges
    moves with them), so the two are compared through what is invariant: the
    sum of the squared norms of every quad (the trace of its Gram), and the
    validity of each result (gram_quad_kernel's own accuracy:
    test_gram_quad_matches_fp64)."""
    A64, outs = _two_step_runs(svdj, cuda, nb, m, inner, ([4, 5], [3, 3]))
    (a1, v1, d1, (m1, r1)), (a2, v2, d2, (m2, r2)) = outs
    assert r1 == r2 == nb
    assert math.isclose(m1, m2, rel_tol=1e-3)
    if inner == 1:
        # (the cross steps' Gram row chunking sets their rounding: 5e-5 held
        # with 128-row chunks, 8.3e-5 was seen with 384-row chunks)
        tol = 2e-4
        torch.testing.assert_close(a1, a2, rtol=tol, atol=tol)
        torch.testing.assert_close(v1, v2, rtol=tol, atol=tol)
        torch.testing.assert_close(d1, d2, rtol=tol, atol=tol)
    else:
        torch.testing.assert_close(d1.view(-1, 4 * 64).sum(1), d2.view(-1, 4 * 64).sum(1),
                                   rtol=1e-6, atol=0)
    n = v1.shape[0]
    for a, v in ((a1, v1), (a2, v2)):
        assert float((v @ v.t() - torch.eye(n, dtype=torch.float64)).abs().max()) < 2e-6
        assert float((A64[:, :m].t() @ v.t() - a[:, :m].t()).abs().max()) < 2e-5


@pytest.mark.parametrize("parts,bound", [(3, 2e-6), (2, 6e-5)])
def test_gram_quad_matches_fp64(svdj, cuda, parts, bound):
    """gram_quad_kernel (one read of the quad's four blocks, the six cross
    Grams on split-bf16 MFMAs) against fp64 products: every entry within
    2e-6 of |a_i| |b_j| (fp32 level: the split products are exact to 2^-26
    and the accumulation is fp32), for 16 quads, several row chunks; the
    2-part form of the early sweeps within 6e-5 (~2^-16 per product, summed
    over 1000 rows: at most 2^-14, in practice far less)."""
    K = svdj.ops.kernels
    W, nb, m, m_pad = 64, 64, 1000, 1024
    g = torch.Generator().manual_seed(4)
    A64 = torch.zeros(nb * W, m_pad, dtype=torch.float64)
    A64[:, :m] = torch.rand(nb * W, m, generator=g, dtype=torch.float64) - 0.4
    A64 *= torch.logspace(-3, 3, nb * W, dtype=torch.float64)[:, None]  # graded column norms
    At = A64.float().to(cuda)
    pairs = torch.from_numpy(svdj.parallel.schedule.quad_round_robin(nb)[1].copy())
    sl = K.gram_quad(At, m_pad, pairs.to(cuda), W, 256, parts=parts)  # (3P, nchunk, W, W)
    P = pairs.shape[0]
    C = sl.double().sum(1).cpu()
    X = At.double().cpu()
    nrm = X.norm(dim=1)
    want = [tuple(pr) for pr in pairs.tolist()]  # slabs [0, P): the step's pairs
    for q in range(P // 2):
        (a, c_), (b, d) = pairs[2 * q].tolist(), pairs[2 * q + 1].tolist()
        want.extend([(a, d), (b, c_), (a, b), (c_, d)])
    for s_, (x, y) in enumerate(want):
        ref = X[x * W:(x + 1) * W] @ X[y * W:(y + 1) * W].t()
        scale = nrm[x * W:(x + 1) * W, None] * nrm[None, y * W:(y + 1) * W]
        err = float(((C[s_] - ref).abs() / scale).max())
        assert err < bound, (s_, x, y, err)


def test_quad_preconverged_skipped(svdj, cuda):
    """Quads whose couplings are all below tol leave A, V and D untouched
    (the apply skips them; T of a skipped quad is never used)."""
    K = svdj.ops.kernels
    W, nb, m, m_pad = 64, 8, 512, 512
    q, _ = torch.linalg.qr(torch.rand(m, nb * W, dtype=torch.float64))
    At = q.t().contiguous().float().to(cuda)   # all columns orthonormal
    Vt = torch.zeros(nb * W, nb * W, dtype=torch.float32, device=cuda)
    K.set_identity(Vt, nb * W)
    D = K.col_norms2(At, m_pad)
    a0, v0, d0 = At.clone(), Vt.clone(), D.clone()
    metric = K.new_metric(cuda)
    K.block_steps(At, Vt, D, m_pad, _quad_pairs(svdj, nb).to(cuda), W, [4, 5], 1e-3, 1, metric,
                  mma="bf16x6")
    assert K.read_metric(metric)[1] == 0
    assert torch.equal(At, a0) and torch.equal(Vt, v0) and torch.equal(D, d0)


@pytest.mark.parametrize("quad", ["on", "off"])
def test_svd_quad_end_to_end(svdj, cuda, quad):
    """Whole solve through the pipelined engine with quad steps on and off:
    both converge to the fp32 accuracy bounds of the block path."""
    from svdj.parallel import DistributedBlockJacobi
    A = svdj.utils.inputs.random_dense(1100, 1024, dtype=torch.float64, seed=8)
    cfg = svdj.SolverConfig(dtype=torch.float32, block=64, mma="bf16x6", quad=quad)
    res = DistributedBlockJacobi(cfg).solve(A.to(cuda))
    assert res.converged and res.info["quad"] == (quad == "on"), res.info
    rep = svdj.utils.metrics.verify(A.to(cuda), res.U, res.S, res.V, torch.linalg.svdvals(A))
    assert rep["residual_rel"] < 8e-6 and rep["sigma_max_abs_err_over_smax"] < 1e-6, rep
    assert rep["orth_u_fro"] < 1.5e-3 and rep["orth_v_fro"] < 2e-4, rep


def test_svd_api_runs_the_pipeline_engine(svdj, cuda):
    """The public entry point gets the headline engine:
    svdj.svd on a GPU runs the distributed plan at P = 1 -- with 32 pairs per
    chain step (8192^2: 128 blocks, 2 super-blocks of 64) quad steps on two
    chains (merged only from 16 to 31 pairs since round 6) -- and gives the
    same result as
    DistributedBlockJacobi on a world-1 communicator."""
    from svdj.parallel import Communicator, DistributedBlockJacobi
    n = 8192
    A = svdj.utils.inputs.random_dense(n, n, dtype=torch.float32, device=cuda, seed=12)
    res = svdj.svd(A)
    assert res.converged and res.info["engine"] == "pipeline", res.info
    assert res.info["quad"] and not res.info["merged_chains"] and res.info["block"] == 64, res.info
    ref = DistributedBlockJacobi(svdj.SolverConfig(), Communicator.local(cuda)).solve(A)
    assert ref.sweeps == res.sweeps and torch.equal(ref.S, res.S)
    rel = float((A @ res.V - res.U * res.S).norm() / A.norm())
    assert rel < 1e-5, rel
    steps = svdj.svd(A[:2048, :2048], extra={"engine": "steps"})
    assert steps.info["engine"] == "steps" and steps.converged


@pytest.mark.parametrize("m,n", [(4500, 4097), (4200, 6000)])
def test_svd_api_ragged_shapes(svdj, cuda, m, n):
    """svd() on shapes that are not multiples of the block: 4097 columns pad
    to whole 64-column blocks (zero columns ride along the quad steps and the
    merged issue) and a wide input runs transposed; fp64 svdvals as oracle."""
    A = svdj.utils.inputs.random_dense(m, n, dtype=torch.float32, device=cuda, seed=21)
    res = svdj.svd(A)
    assert res.converged and res.info["engine"] == "pipeline" and res.info["quad"], res.info
    k = min(m, n)
    assert res.S.shape == (k,) and res.U.shape == (m, k) and res.V.shape == (n, k)
    ref = torch.linalg.svdvals(A.double().cpu())
    got = torch.sort(res.S.double().cpu(), descending=True).values
    assert float((got - ref).abs().max() / ref[0]) < 1e-6
    # reconstruction (for the transposed solve A V - U S would measure the
    # orthogonality of the Jacobi side's U' = V, amplified by sigma ratios)
    rel = float((A - (res.U * res.S) @ res.V.T).norm() / A.norm())
    assert rel < 1e-5, rel
    eye = torch.eye(k, device=cuda)
    assert float((res.V.T @ res.V - eye).abs().max()) < 1e-4
    assert float((res.U.T @ res.U - eye).abs().max()) < 1e-4


def test_svd_quad_without_v_and_bf16(svdj, cuda):
    """Quad steps without V (jobv = NoVec: the apply's V tiles are skipped)
    give bitwise the singular values of the AllVec solve (V never feeds back
    into A); and the bf16 problem mode's 2-way split runs quad steps
    (apply_quad_ts_kernel<2>) to bf16-level accuracy."""
    from svdj.config import SVDOptions
    from svdj.parallel import DistributedBlockJacobi
    A = svdj.utils.inputs.random_dense(1100, 1024, dtype=torch.float64, seed=8).to(cuda)
    cfg = svdj.SolverConfig(dtype=torch.float32, block=64, mma="bf16x6", quad="on")
    full = DistributedBlockJacobi(cfg).solve(A)
    nov = DistributedBlockJacobi(cfg).solve(A, jobv=SVDOptions.NoVec)
    assert nov.info["quad"] and nov.V is None
    assert full.sweeps == nov.sweeps and torch.equal(full.S, nov.S)
    cfg16 = svdj.SolverConfig(dtype=torch.bfloat16, block=64, quad="on")
    r16 = DistributedBlockJacobi(cfg16).solve(A.to(torch.bfloat16))
    assert r16.converged and r16.info["quad"] and r16.info["mma"] == "bf16x3", r16.info
    ref = torch.linalg.svdvals(A.to(torch.bfloat16).double().cpu())
    got = torch.sort(r16.S.double().cpu(), descending=True).values
    assert float((got - ref).abs().max() / ref[0]) < 1e-4


# ---- pair-count-selected variants of the per-step kernels:
# qbuild_kernel<T, W, 16> from 64 pairs per step, the Gram geometry from 32
# pairs; the other kernel tests use 2 pairs.
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_block_step_many_pairs_matches_few_pairs(svdj, cuda, dtype):
    """One cross step with 64 pairs (qbuild_kernel<T, W, 16>, the 256-workgroup
    Gram geometry) equals the same pairs issued 2 per step (the R = 4 Q build
    and 512-workgroup geometry the 2-pair reference tests cover), and the fp64
    one equals the fp64 torch reference."""
    K, R = svdj.ops.kernels, svdj.ops.reference
    W, nb, m, m_pad = 64, 128, 256, 256
    n = nb * W
    A64 = _orth_blocks(nb, W, m, m_pad, seed=9)
    pairs = torch.from_numpy(svdj.parallel.schedule.round_robin(nb)[3:4].copy())
    assert pairs.shape[1] == 64
    tol = 1e-6 if dtype == torch.float32 else 1e-13
    outs = []
    for split in (False, True):
        At = A64.to(dtype).to(cuda)
        Vt = torch.zeros(n, 128, dtype=dtype, device=cuda)
        g = torch.Generator().manual_seed(1)
        Vt[:, :] = (torch.rand(n, 128, generator=g, dtype=torch.float64) - 0.5).to(dtype).to(cuda)
        D = K.col_norms2(At, m_pad)
        metric = K.new_metric(cuda)
        if split:  # 32 steps of 2 pairs: the same pairs, disjoint, in any order
            pp = pairs[0].view(32, 2, 2)
            K.block_steps(At, Vt, D, m_pad, pp.to(cuda), W, [0] * 32, tol, 1, metric,
                          inner_order="cross")
        else:
            K.block_steps(At, Vt, D, m_pad, pairs.to(cuda), W, [0], tol, 1, metric,
                          inner_order="cross")
        outs.append((At.double().cpu(), Vt.double().cpu(), D.double().cpu(), K.read_metric(metric)))
    (a1, v1, d1, (m1, r1)), (a2, v2, d2, (m2, r2)) = outs
    assert r1 == r2 == 64
    assert math.isclose(m1, m2, rel_tol=1e-5)
    # (fp32: the two issues may sum the Gram over different row chunks --
    # 1 vs 2 at m_pad = 256 -- so they agree to the couplings' rounding
    # amplified by the EVD, 5.8e-5 seen, not bit for bit)
    rt = 1e-4 if dtype == torch.float32 else 1e-11
    torch.testing.assert_close(a1, a2, rtol=rt, atol=rt)
    torch.testing.assert_close(v1, v2, rtol=rt, atol=rt)
    torch.testing.assert_close(d1, d2, rtol=rt, atol=rt)
    if dtype == torch.float64:
        At64, Vt64 = A64.clone(), outs[0][1] * 0
        g = torch.Generator().manual_seed(1)
        Vt64 = torch.rand(n, 128, generator=g, dtype=torch.float64) - 0.5
        D64 = (At64 ** 2).sum(1)
        R.block_step(At64, Vt64, D64, pairs[0], W, False, tol, 1, order="cross")
        torch.testing.assert_close(a1[:, :m], At64[:, :m], rtol=1e-11, atol=1e-11)
        torch.testing.assert_close(v1, Vt64, rtol=1e-11, atol=1e-11)
