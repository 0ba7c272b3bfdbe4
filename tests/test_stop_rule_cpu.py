"""Second-order sweep stop test (csrc/include/svdj_stop.h) on the CPU.

The rule ends the iteration after a sweep whose applied rotations were all
noise: (column rotations) x (largest coupling) x (largest effective sine)
<= tol / 2.  The reference has no stop test at all (one sweep,
reference main.cu:482; its convergence value is discarded, main.cu:710)."""
import pytest
import torch

from svdj.ops import kernels as K


def test_rule_table():
    tol = 1.5e-5
    c = K.sweep_converged
    assert c(0.0, 0.0, 0, 0, tol) == 1                       # nothing rotated
    assert c(1.01 * tol, 0.1, 2, 3, tol) == 2                # 3 noise rotations: 0.30 tol
    assert c(1.01 * tol, 0.2, 2, 3, tol) == 0                # 0.61 tol > tol / 2
    assert c(0.1, 1e-3, 40, 1000, tol) == 0                  # a real sweep
    assert c(0.1, 1e-12, 40, 1000, tol) == 2                 # large couplings, tiny angles
    assert c(1.01 * tol, 0.1, 2, 3, tol, stop_rule="no_rotation") == 0
    assert c(1.01 * tol, 0.1, 2, 3, tol, tol_mode="absolute") == 0  # reference parity mode
    assert c(1.01 * tol, 0.1, 2, 0, tol) == 0                # inconsistent counts: no shortcut


def _solve(A, rule):
    n = A.shape[1]
    At = A.t().contiguous().clone()
    Vt = torch.eye(n, dtype=A.dtype)
    D = K.col_norms2(At, n)
    tol = n ** 0.5 * torch.finfo(A.dtype).eps
    sw, hist = K.block_solve(At, Vt, D, n, 32, tol, 1, 60, inner_order="cross", stop_rule=rule)
    G = At.double() @ At.double().t()
    d = G.diagonal().sqrt()
    cmax = float((G / d[:, None] / d[None, :]).abs().fill_diagonal_(0).max())
    return sw, At, Vt, cmax / tol


@pytest.mark.parametrize("seed,saves", [(1, True), (3, False)])
def test_block_solve_second_order(seed, saves):
    """seed 1: the rule ends the solve one sweep earlier and the result is
    BITWISE the no-rotation solve's (the confirmation sweep it skips rotates
    nothing); seed 3: its last rotating sweep is not noise-level, the rule
    must not fire and both stop after the same sweep."""
    g = torch.Generator().manual_seed(seed)
    A = torch.rand(256, 256, dtype=torch.float32, generator=g)
    sw0, At0, Vt0, c0 = _solve(A, "no_rotation")
    sw1, At1, Vt1, c1 = _solve(A, "second_order")
    assert sw1 == (sw0 - 1 if saves else sw0)
    assert torch.equal(At0, At1) and torch.equal(Vt0, Vt1)
    assert c1 <= 1.5  # the rule's guarantee: couplings at most 1.5 tol at the end
