"""CPU checks of the split-bf16 apply's arithmetic (csrc/hip/block.hip
apply_split_kernel): the 3-way round-to-nearest bf16 split is accurate to
2^-27, and the six order < 3 products of X (Q - I), added to X in fp32,
reproduce X Q to fp32 rounding.  The GPU kernel itself is checked against the
f32 MFMA apply in tests/test_gpu_kernels.py (test_bf16x6_matches_native)."""
import pytest
import torch


def split3(x: torch.Tensor):
    parts, r = [], x.float()
    for _ in range(3):
        p = r.to(torch.bfloat16).float()  # round to nearest even
        parts.append(p)
        r = r - p                          # exact in fp32
    return parts


def test_split_is_accurate_to_2_pow_27():
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(200000, generator=g, dtype=torch.float64) * 2 - 1).float()
    x = x * torch.pow(2.0, torch.randint(-20, 20, x.shape, generator=g)).float()
    p0, p1, p2 = split3(x)
    resid = (x.double() - (p0.double() + p1.double() + p2.double())).abs()
    assert float((resid / x.double().abs().clamp_min(1e-300)).max()) <= 2.0 ** -26


def test_delta_form_matches_fp32_product():
    g = torch.Generator().manual_seed(1)
    N, rows = 128, 512
    X = torch.rand(rows, N, generator=g, dtype=torch.float64).float()
    # a near-identity rotation (what late Jacobi sweeps apply) and a random one
    S = torch.randn(N, N, generator=g, dtype=torch.float64) * 1e-3
    for Q in (torch.linalg.matrix_exp(S - S.t()).float(),
              torch.linalg.qr(torch.randn(N, N, generator=g, dtype=torch.float64))[0].float()):
        D = Q - torch.eye(N)                 # exact: entries of Q - I near the diagonal are Sterbenz
        xs, qs = split3(X), split3(D)
        acc = torch.zeros(rows, N, dtype=torch.float64)
        for o in range(3):                   # products of order < 3, exact in fp64 here
            for a in range(o + 1):
                acc += xs[o - a].double() @ qs[a].double()
        Y = (X.double() + acc.float().double()).float()   # fp32 accumulator + fp32 add
        ref = X.double() @ Q.double()
        err = (Y.double() - ref).abs().max() / ref.abs().max()
        assert float(err) < 4 * 2.0 ** -24, float(err)


@pytest.mark.parametrize("inner", [1, 3])
def test_reference_quad_step_equals_two_cross_steps(inner):
    """ops.reference.quad_step (Gram-space couplings for the second step, T =
    T1 T2 applied once) equals the two cross steps it fuses, in fp64."""
    import torch
    import svdj
    R, S = svdj.ops.reference, svdj.parallel.schedule
    torch.manual_seed(0)
    W, nb, m = 16, 8, 300
    n = nb * W
    A = torch.rand(n, m, dtype=torch.float64)
    for b in range(nb):
        q, _ = torch.linalg.qr(A[b * W:(b + 1) * W].t())
        A[b * W:(b + 1) * W] = (q * torch.linspace(1, 3, W, dtype=torch.float64)).t()
    pr = torch.from_numpy(S.quad_round_robin(nb))
    At1, Vt1 = A.clone(), torch.eye(n, dtype=torch.float64)
    D1 = R.col_norms2(At1)
    At2, Vt2, D2 = At1.clone(), Vt1.clone(), D1.clone()
    m1a, r1a = R.block_step(At1, Vt1, D1, pr[1], W, False, 1e-12, inner, order="cross")
    m1b, r1b = R.block_step(At1, Vt1, D1, pr[2], W, False, 1e-12, inner, order="cross")
    m2, r2 = R.quad_step(At2, Vt2, D2, pr[1], pr[2], W, 1e-12, inner)
    assert r2 == r1a + r1b == nb
    assert abs(m2 - max(m1a, m1b)) < 1e-12
    for x, y in ((At1, At2), (Vt1, Vt2), (D1, D2)):
        assert float((x - y).abs().max()) < 1e-13
