"""Numerics of the device M-step's orth() (EM_W_multi.R:732-733) on ill-conditioned X'mu_T.

The device computes the polar factor U V' of S = X'mu_T by Cholesky-QR2 + Jacobi and falls back to
Householder QR + Jacobi when S is too ill-conditioned for Cholesky-QR2.  Here S is
made EXACT on both sides: X = [I_p; 0] so that the device's X'mu_T is mu_T[:p] bit for bit, and S is
given singular values down to sigma_max / kappa.  Checks against numpy's SVD polar factor (the
oracle's orth, functions.R:256): W'W = I to 1e-13 whatever kappa; W'S symmetric positive definite
(the polar property); |W - W_ref| <= 1e-13 + 64 eps kappa (two backward-stable polar factors differ
by O(eps kappa), the factor's own condition number).
"""
import numpy as np
import pytest

from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu

EPS = np.finfo(np.float64).eps


def _with_condition(rng, p, r, kappa):
    U = np.linalg.qr(rng.standard_normal((p, r)))[0]
    V = np.linalg.qr(rng.standard_normal((r, r)))[0]
    s = np.geomspace(1.0, 1.0 / kappa, r) * 3.7
    return (U * s) @ V.T


@pytest.fixture(scope="module")
def ctx():
    from ppls_amd import Context
    c = Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("kappa", [1e2, 1e6, 1e10, 1e13])
@pytest.mark.parametrize("p,q,r", [(400, 300, 5), (900, 120, 10), (64, 40, 2)])
@pytest.mark.parametrize("typ", ["SVD", "QR"])
def test_orth_ill_conditioned(ctx, kappa, p, q, r, typ):
    from ppls_amd import Expect
    rng = np.random.default_rng(int(np.log10(kappa)) * 100 + p + r)
    n = max(p, q) + 7
    X = np.zeros((n, p))
    X[:p, :p] = np.eye(p)
    Y = np.zeros((n, q))
    Y[:q, :q] = np.eye(q)
    SX = _with_condition(rng, p, r, kappa)
    SY = _with_condition(rng, q, r, min(kappa, 1e4))
    ctx.set_data(X, Y)
    fit = Expect(r, n, want_mu=True)
    fit.mu_T[:p] = SX
    fit.mu_U[:q] = SY
    fit.Ctt[:] = 1.0 + np.arange(r)
    fit.Cuu[:] = 1.0
    fit.Cut[:] = 0.5
    fit.Chh[:] = np.eye(r) * 0.1
    fit.Cee, fit.Cff = 0.3, 0.2
    th = ctx.mstep(fit, 0 if typ == "SVD" else 1)
    for W, S, k in ((th.W, SX, kappa), (th.C, SY, min(kappa, 1e4))):
        assert np.abs(W.T @ W - np.eye(r)).max() < 1e-13
        ref = o.orth(S, typ)
        assert np.abs(W - ref).max() < 1e-13 + 64 * EPS * k
        H = W.T @ S
        if typ == "SVD":   # polar: W'S = V Sigma V' symmetric positive definite
            assert np.abs(H - H.T).max() < 1e-12 * np.abs(S).max()   # backward stable: eps ||S||
            assert np.linalg.eigvalsh((H + H.T) / 2).min() > 0
        else:              # QR: W'S upper triangular, first column along S[:, 0] (functions.R:257-259)
            assert np.abs(np.tril(H, -1)).max() < 1e-12 * np.abs(S).max()
            assert H[0, 0] > 0


@pytest.mark.parametrize("kappa", [1.0001, 3.0, 7.5, 9.0, 50.0])
@pytest.mark.parametrize("p,q,r", [(400, 300, 5), (5000, 120, 10), (2500, 64, 3)])
def test_orth_cholqr1_fast_path(ctx, kappa, p, q, r):
    """The finalize's Cholesky-QR1 fast path (option polar1, taken when ||R1||_F ||R1^-1||_F <= 2r; wide p runs it
    as a team) against numpy's SVD polar and against the Cholesky-QR2 path (polar1 = 0)."""
    from ppls_amd import Expect
    rng = np.random.default_rng(int(kappa * 10) + p + r)
    n = max(p, q) + 3
    X = np.zeros((n, p))
    X[:p, :p] = np.eye(p)
    Y = np.zeros((n, q))
    Y[:q, :q] = np.eye(q)
    SX = _with_condition(rng, p, r, kappa)
    SY = _with_condition(rng, q, r, kappa)
    ctx.set_data(X, Y)
    fit = Expect(r, n, want_mu=True)
    fit.mu_T[:p] = SX
    fit.mu_U[:q] = SY
    fit.Ctt[:] = 1.0 + np.arange(r)
    fit.Cuu[:] = 1.0
    fit.Cut[:] = 0.5
    fit.Chh[:] = np.eye(r) * 0.1
    fit.Cee, fit.Cff = 0.3, 0.2
    out = {}
    try:
        for fast in (1, 0):
            ctx.set_option("polar1", fast)
            out[fast] = ctx.mstep(fit, 0)
    finally:
        ctx.set_option("polar1", 1)
    for a, b, S in ((out[1].W, out[0].W, SX), (out[1].C, out[0].C, SY)):
        assert np.abs(a.T @ a - np.eye(r)).max() < 1e-13
        ref = o.orth(S, "SVD")
        assert np.abs(a - ref).max() < 1e-13
        assert np.abs(a - b).max() < 1e-13
