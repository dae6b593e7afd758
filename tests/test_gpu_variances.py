"""GPU parity of variances.PPLS_simult (EM_W_multi.R:830-860) and of its MFMA Gram X'X against the
oracle (oracle.ppls_oracle.variances_ppls_simult, a literal restatement).

Tolerances (fp64): the Gram 1e-13 relative (and exactly symmetric); W 1e-10 absolute; SSt_exp,
SSt_star 1e-11 relative; varMatrix and seLoad 1e-8 relative (the inverse of the observed information:
the hand-written blocked Cholesky + inverse of ppls_linalg.hip by default, rocSOLVER potrf/potri with
option var_chol = 2, LU getrf/getri with var_chol = 0 or when the matrix is not positive definite, vs
LAPACK gesv -- all backward stable, they differ by ~cond * eps).
"""
import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from ppls_amd import Context
    c = Context(0)
    yield c
    c.close()


def _rel(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


@pytest.mark.parametrize("n,p,nsplit", [(1000, 300, 1), (997, 257, 3), (64, 128, 0), (3001, 40, 7), (5, 129, 1)])
def test_gram_mfma_matches_numpy(ctx, n, p, nsplit):
    rng = np.random.default_rng(n + p)
    X = rng.standard_normal((n, p))
    ctx.set_data(X, rng.standard_normal((n, 3)))
    G, ms = ctx.gram(0, nsplit)
    ref = X.T @ X
    assert _rel(G, ref) < 1e-13
    assert np.array_equal(G, G.T)
    Gy, _ = ctx.gram(1, 0)
    Yd, _ = ctx.get_data()
    assert Gy.shape == (3, 3)


def test_gram_fp32_storage(ctx):
    rng = np.random.default_rng(5)
    X = rng.standard_normal((2000, 203))
    ctx.set_option("dtype", 1)
    try:
        ctx.set_data(X, rng.standard_normal((2000, 9)))
        G, _ = ctx.gram(0, 0)
    finally:
        ctx.set_option("dtype", 0)
    X32 = X.astype(np.float32).astype(np.float64)   # fp32 storage, fp64 products
    assert _rel(G, X32.T @ X32) < 1e-13


@pytest.mark.parametrize("chol", [1, 2, 0], ids=["chol", "chol_rocsolver", "lu"])
@pytest.mark.parametrize("from_s", [False, True], ids=["gram", "from_S"])
@pytest.mark.parametrize("xy", ["X", "Y"])
def test_variances_matches_oracle(ctx, xy, from_s, chol):
    """from_S: the cross-product form has formed S = [X Y]'[X Y] for this data, and the variances
    take its X'X / Y'Y block instead of a Gram of their own (q = 29: the Y block starts mid-tile)."""
    import ppls_amd
    X, Y, th0 = make_problem(700, 37, 29, 3, seed=61)
    fit = o.ppls_simult(X, Y, 3, EMsteps=20, atol=-np.inf, theta0=th0)
    D = X if xy == "X" else Y
    ref = o.variances_ppls_simult(fit, D, xy)
    ctx.set_option("var_chol", chol)
    ctx.set_data(X, Y)
    if from_s:
        ctx.xprod_prepare()
        assert ctx.xprod_info(3)["ready"]
    try:
        got = ppls_amd.variances_PPLS_simult(fit, None, xy, ctx=ctx)
    finally:
        ctx.set_option("var_chol", 1)
    assert np.abs(got["W"] - ref["W"]).max() < 1e-10
    for i in range(3):
        g, r = got["components"][i], ref["components"][i]
        assert _rel(g["B_exp"], r["B_exp"]) < 1e-13
        assert _rel(g["SSt_exp"], r["SSt_exp"]) < 1e-11
        assert _rel(g["SSt_star"], r["SSt_star"]) < 1e-11
        assert _rel(got["varMatrix"][i], ref["varMatrix"][i]) < 1e-8
    assert _rel(got["seLoad"], ref["seLoad"]) < 1e-8
    # data passed explicitly (a temporary context holds it) gives the same result
    got2 = ppls_amd.variances_PPLS_simult(fit, D, xy, full=False)
    assert _rel(got2["seLoad"], ref["seLoad"]) < 1e-8
    with pytest.raises(ValueError):
        ppls_amd.variances_PPLS_simult(fit, D)          # XorY left at its default c("X", "Y")


@pytest.mark.parametrize("xy", ["X", "Y"])
def test_variances_multi_block(ctx, xy):
    """p = 150, q = 131: the hand-written inverse's 64 x 64 blocks, a partial last block; equal to
    the oracle and to rocSOLVER's potrf/potri (var_chol = 2)."""
    import ppls_amd
    X, Y, th0 = make_problem(1500, 150, 131, 4, seed=67)
    fit = o.ppls_simult(X, Y, 4, EMsteps=15, atol=-np.inf, theta0=th0)
    D = X if xy == "X" else Y
    ref = o.variances_ppls_simult(fit, D, xy)
    ctx.set_data(X, Y)
    got = {}
    for chol in (1, 2):
        ctx.set_option("var_chol", chol)
        try:
            got[chol] = ppls_amd.variances_PPLS_simult(fit, None, xy, ctx=ctx)
        finally:
            ctx.set_option("var_chol", 1)
    for i in range(4):
        assert _rel(got[1]["varMatrix"][i], ref["varMatrix"][i]) < 1e-8
        assert _rel(got[1]["varMatrix"][i], got[2]["varMatrix"][i]) < 1e-9
        assert np.array_equal(got[1]["varMatrix"][i], got[1]["varMatrix"][i].T)
    assert _rel(got[1]["seLoad"], ref["seLoad"]) < 1e-8
