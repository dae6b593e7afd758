"""fp32 storage of X, Y (context option dtype = 1; C5's "fp32" configuration) on the GPU.

X and Y are held in HBM as fp32 (half the bytes per sweep); every product and statistic is
accumulated in fp64.  So the GPU fit on fp32-stored data must match the fp64 oracle run on the
same fp32-rounded data to the fp64 tolerances (loglik 1e-10 relative, loadings 1e-8 absolute):
the only fp32 effect is the rounding of the data itself, which these tests apply to the oracle's
input as well.
"""
import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu


def _ctx32():
    from ppls_amd import Context
    c = Context(0)
    c.set_option("dtype", 1)
    return c


def _round32(A):
    return np.asarray(A, dtype=np.float32).astype(np.float64)


def _theta(th):
    from ppls_amd import Theta
    return Theta(th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])


def _relerr(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


@pytest.mark.parametrize("p,q,r", [(37, 23, 3), (700, 41, 10), (130, 96, 1)])
def test_fp32_storage_em_matches_oracle_on_rounded_data(p, q, r):
    X, Y, th0 = make_problem(333, p, q, r, seed=40 + r)
    X32, Y32 = _round32(X), _round32(Y)
    with _ctx32() as c:
        c.set_data(X, Y)
        Xb, Yb = c.get_data()
        assert np.array_equal(Xb, X32) and np.array_equal(Yb, Y32)
        Xr, Yr = c.get_data_rows(5, 300)
        assert np.array_equal(Xr, X32[5:305]) and np.array_equal(Yr, Y32[5:305])
        sx, sy = c.ssq()
        assert np.isclose(sx, np.sum(X32 * X32), rtol=1e-13)
        est, ll, _, _ = c.em_run(_theta(th0), 6, -np.inf, 0, want_eout=False)
    ref = o.ppls_simult(X32, Y32, r, EMsteps=6, atol=-np.inf, theta0=th0)
    assert _relerr(ll, ref["loglik"]) < 1e-10
    assert np.abs(est.W - ref["estimates"]["W"]).max() < 1e-8
    assert _relerr([est.sigE, est.sigF, est.sigH], [ref["estimates"][k] for k in ("sigE", "sigF", "sigH")]) < 1e-8


def test_fp32_synthetic_equals_rounded_fp64_synthetic():
    from ppls_amd import Context, Theta
    rng = np.random.default_rng(3)
    W = np.linalg.qr(rng.standard_normal((45, 2)))[0]
    C = np.linalg.qr(rng.standard_normal((31, 2)))[0]
    truth = Theta(W, C, [1.2, 0.8], 0.5, 0.5, 0.1, [1.0, 0.9])
    with Context(0) as c64, _ctx32() as c32:
        c64.generate_synthetic(5000, 45, 31, truth, seed=77)
        c32.generate_synthetic(5000, 45, 31, truth, seed=77)
        X64, Y64 = c64.get_data()
        X32, Y32 = c32.get_data()
    assert np.array_equal(X32, _round32(X64)) and np.array_equal(Y32, _round32(Y64))


def test_fp32_sequential_init_matches_oracle():
    X, Y, _ = make_problem(260, 28, 19, 2, seed=44)
    X32, Y32 = _round32(X), _round32(Y)
    inits = [o.initial_guess(28, 19, "equal")] * 2
    with _ctx32() as c:
        c.set_data(X, Y)
        f = c.ppls(2, 20, 1e-4, inits)
    ref = o.ppls(X32, Y32, 2, 20, 1e-4, inits)
    assert np.abs(f["W"] - ref["W"]).max() < 1e-8
    assert _relerr(f["Other_output"]["Loglikelihoods"], ref["Other_output"]["Loglikelihoods"]) < 1e-10


@pytest.mark.parametrize("dtype,p,q", [(1, 4100, 300), (1, 700, 41), (0, 2600, 9)])
def test_row_padding_is_invisible(dtype, p, q):
    """Panel-path rows are padded to 128 B / 4 KB (ldpad, ppls_capi.cpp ld_of); the padding
    columns are zero, so a fit on padded rows equals the 16-B-row fit (the E-step and one EM step
    bitwise; over several iterations to rounding, since the grid partition of the ||X||^2 and
    reduction kernels follows the row stride), and get_data returns the unpadded matrices.
    (4100 fp32 = 16,400 B -> 4-KB padding; 700 fp32 -> 128 B; 2600 fp64 = 20,800 B -> 4 KB.)"""
    from ppls_amd import Context
    r = 3
    X, Y, th0 = make_problem(700, p, q, r, seed=p + q)
    out = []
    for pad in (0, 1):
        with Context(0) as c:
            c.set_option("dtype", dtype)
            c.set_option("ldpad", pad)
            c.set_data(X, Y)
            Xb, Yb = c.get_data()
            mu = c.estep(_theta(th0)).mu_T
            one, _ = c.em_step(_theta(th0))
            est, ll, _, _ = c.em_run(_theta(th0), 3, -np.inf, 0, want_eout=False)
            out.append((Xb, Yb, mu, one, est, ll))
    (X0, Y0, m0, o0, e0, l0), (X1, Y1, m1, o1, e1, l1) = out
    assert X1.shape == (700, p) and Y1.shape == (700, q)
    assert np.array_equal(X0, X1) and np.array_equal(Y0, Y1)
    assert np.array_equal(m0, m1)
    assert np.array_equal(o0.W, o1.W) and np.array_equal(o0.C, o1.C)
    assert _relerr(l1, l0) < 1e-14
    assert np.abs(e0.W - e1.W).max() < 1e-14 and np.abs(e0.C - e1.C).max() < 1e-14



@pytest.mark.parametrize("dtype,n,p,q,r,grid", [(1, 2000, 1500, 90, 10, 0), (1, 700, 65, 33, 3, 3),
                                                 (0, 900, 2300, 17, 9, 0), (1, 5000, 31, 2, 2, 2)])
def test_dots_wave_pair_equals_single_wave(dtype, n, p, q, r, grid):
    """Panel dots on small shards split each row tile's columns over a wave pair (KS = 2 in
    ppls_panel_mfmadots_kernel; option dots_pair = 0 forces one wave per tile).  Both forms sum the same
    products in a different grouping: mu within 1e-13 of each other and of the oracle's E-step;
    `grid` > 0 shrinks the dots grid so workgroups loop (the pair's LDS combine sits inside that
    loop behind workgroup barriers); one column tile per matrix (p = 31, q = 2) leaves the pair's
    first wave without columns."""
    from ppls_amd import Context
    X, Y, th0 = make_problem(n, p, q, r, seed=n + p)
    if dtype:
        X, Y = _round32(X), _round32(Y)
    mus = []
    for pair in (-1, 0):
        with Context(0) as c:
            c.set_option("dtype", dtype)
            if grid:
                c.set_option("grid", grid)
            c.set_option("dots_pair", pair)
            c.set_data(X, Y)
            assert "panel" in c.sweep_kernel(r)
            assert ("wave pair" in c.sweep_kernel(r)) == (pair == -1)
            e = c.estep(_theta(th0))
            mus.append((e.mu_T, e.mu_U))
    ref = o.expect_m(X, Y, *(th0[k] for k in ("W", "C", "B", "sigE", "sigF", "sigH", "sigT")))
    scale = max(np.abs(ref["mu_T"]).max(), np.abs(ref["mu_U"]).max())
    for (mt, mu) in mus:
        assert np.abs(mt - ref["mu_T"]).max() < 1e-12 * scale
        assert np.abs(mu - ref["mu_U"]).max() < 1e-12 * scale
    assert np.abs(mus[0][0] - mus[1][0]).max() < 1e-13 * scale
    assert np.abs(mus[0][1] - mus[1][1]).max() < 1e-13 * scale

