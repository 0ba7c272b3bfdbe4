"""CPU checks of the split-bf16 apply's arithmetic (csrc/hip/block.hip
apply_split_kernel): the 3-way round-to-nearest bf16 split is accurate to
2^-27, and the six order < 3 products of X (Q - I), added to X in fp32,
reproduce X Q to fp32 rounding.  The GPU kernel itself is checked against the
f32 MFMA apply in tests/test_gpu_kernels.py (test_bf16x6_matches_native)."""
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
