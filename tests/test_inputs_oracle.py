"""Reference input parity, CPU oracle accuracy and reference-behaviour checks."""
import math

import numpy as np
import pytest
import torch

import svdj


def _canonical_stream(seed, count):
    """Python twin of libstdc++ minstd_rand0 + generate_canonical<double,53>
    (SURVEY.md section 6.4): two draws per value, R = 2^31 - 2."""
    x = seed % 2147483647
    R = 2147483646.0
    out = []
    for _ in range(count):
        x = (16807 * x) % 2147483647
        g1 = x
        x = (16807 * x) % 2147483647
        g2 = x
        s = float(g1 - 1) + float(g2 - 1) * R
        v = s / (R * R)  # R*R rounded like libstdc++'s long double product -> double
        if v >= 1.0:
            v = math.nextafter(1.0, 0.0)
        out.append(v)
    return np.array(out)


def test_reference_rng_stream_bit_exact():
    native = svdj.utils.inputs.reference_uniform_stream(1000)
    twin = _canonical_stream(1000000, 1000)
    assert np.array_equal(native.view(np.uint64), twin.view(np.uint64))
    assert 0.0 <= native.min() and native.max() < 1.0


def test_reference_triu_layout():
    n = 6
    A = svdj.utils.inputs.reference_triu(n)
    stream = svdj.utils.inputs.reference_uniform_stream(n * (n + 1) // 2)
    it = iter(stream)
    for i in range(n):  # row by row, j >= i (reference main.cu:1559-1567)
        for j in range(i, n):
            assert A[i, j].item() == next(it)
    assert torch.count_nonzero(torch.tril(A, -1)) == 0


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-12), (torch.float32, 5e-5)])
@pytest.mark.parametrize("ordering", ["sameh", "round_robin"])
def test_oracle_matches_lapack(dtype, tol, ordering):
    A = svdj.utils.inputs.random_dense(96, 80, seed=11)
    res = svdj.svd(A, method="oracle", dtype=dtype, ordering=ordering)
    assert res.converged
    rep = svdj.utils.metrics.verify(A, res.U, res.S, res.V, torch.linalg.svdvals(A))
    assert rep["sigma_max_abs_err_over_smax"] < tol
    assert rep["residual_rel"] < tol
    assert rep["orth_v_fro"] < 50 * tol


def test_oracle_config1_512_fp64():
    """BASELINE config 1: 512x512 fp64 dense, single-process CPU sweep."""
    A = svdj.utils.inputs.reference_dense(512)
    res = svdj.svd(A, method="oracle", dtype=torch.float64)
    rep = svdj.utils.metrics.verify(A, res.U, res.S, res.V, torch.linalg.svdvals(A))
    assert res.converged and 8 <= res.sweeps <= 20, res.sweeps
    assert rep["sigma_max_rel_err"] < 1e-10 and rep["orth_u_fro"] < 1e-10, rep


def test_reference_single_sweep_residual_is_vacuous():
    """Reproduces SURVEY.md 6.3: the reference's 1-sweep, absolute-1e-16 run on
    its triangular input has a tiny ||A - U S V^T|| but U is far from
    orthogonal -- the reference's only check cannot detect non-convergence."""
    A = svdj.utils.inputs.reference_triu(128)
    res = svdj.svd(A, method="oracle", dtype=torch.float64, max_sweeps=1, tol_mode="absolute")
    rep = svdj.utils.metrics.verify(A, res.U, res.S, res.V, torch.linalg.svdvals(A))
    assert res.sweeps == 1
    assert rep["residual_rel"] < 1e-12
    assert rep["orth_u_fro"] > 1.0
    # the fixed solver (relative threshold, stopping test) converges
    good = svdj.svd(A, method="oracle", dtype=torch.float64)
    rep2 = svdj.utils.metrics.verify(A, good.U, good.S, good.V)
    assert good.converged and rep2["orth_v_fro"] < 1e-10


def test_cpu_verification_helpers_match_torch():
    import ctypes as C

    A = svdj.utils.inputs.random_dense(40, 30, seed=3)
    res = svdj.svd(A, method="oracle")
    lib = svdj.ops.cpu_lib()
    a = np.ascontiguousarray(A.t().numpy())
    u = np.ascontiguousarray(res.U.t().numpy())
    v = np.ascontiguousarray(res.V.t().numpy())
    s = np.ascontiguousarray(res.S.numpy())
    P = C.POINTER(C.c_double)
    r = lib.svdj_cpu_residual_f64(40, 30, 30, a.ctypes.data_as(P), 40, u.ctypes.data_as(P), 40,
                                  s.ctypes.data_as(P), v.ctypes.data_as(P), 30, 2)
    o = lib.svdj_cpu_orth_f64(40, 30, u.ctypes.data_as(P), 40, 2)
    rep = svdj.utils.metrics.verify(A, res.U, res.S, res.V)
    assert abs(r - rep["residual_fro"]) < 1e-12
    assert abs(o - rep["orth_u_fro"]) < 1e-12


def test_oracle_ordered_rotation_sorts_sigma():
    """Ordered (Erricos) rotation from reference lib/Utils.cu:57-80: converges to
    the same SVD and leaves sigma (nearly) sorted in column order."""
    A = svdj.utils.inputs.random_dense(120, 96, seed=13)
    res = svdj.svd(A, method="oracle", rotation="ordered", ordering="round_robin")
    rep = svdj.utils.metrics.verify(A, res.U, res.S, res.V, torch.linalg.svdvals(A))
    assert res.converged and rep["residual_rel"] < 1e-12 and rep["sigma_max_rel_err"] < 1e-10
    inversions = int((res.S[:-1] < res.S[1:]).sum())
    plain = svdj.svd(A, method="oracle", ordering="round_robin")
    inv_plain = int((plain.S[:-1] < plain.S[1:]).sum())
    assert inversions < inv_plain
