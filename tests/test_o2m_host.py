"""The 'o2m' starting values (EM_W_multi.R:126-131 inside PPLS's sequential loop :254-271; OmicsPLS::o2m
is not vendored -- oracle.ppls_oracle.o2m_1 restates its n = 1, nx = ny = 0 case, parity unpinned
against R): the product computes them from the joint Gram [X Y]'[X Y] with the earlier components'
deflation applied algebraically (ppls_amd.api.o2m_guess_from_gram); here, with a numpy Gram, they must
equal the oracle's values on the explicitly deflated data.  CPU only."""
import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as O
from ppls_amd.api import o2m_guess_from_gram


def _align(g, ref):
    """The singular pair's sign is LAPACK's: flip W and C together (B, the sigmas unchanged)."""
    if float(g["W"] @ ref["W"]) < 0:
        g = dict(g, W=-g["W"], C=-g["C"])
    return g


def _close(g, ref, tol):
    for k in ("W", "C"):
        assert np.abs(np.ravel(g[k]) - np.ravel(ref[k])).max() < tol, k
    for k in ("B", "sigE", "sigF", "sigH", "sigT"):
        assert abs(g[k] - ref[k]) <= tol * max(1.0, abs(ref[k])), (k, g[k], ref[k])


def test_o2m_1_is_the_first_singular_pair():
    X, Y, _ = make_problem(400, 30, 20, 2, seed=3)
    sim = O.o2m_1(X, Y)
    M = X.T @ Y
    s = float(sim["W"] @ M @ sim["C"])
    assert np.allclose(M @ sim["C"], s * sim["W"], atol=1e-10 * s)
    assert np.allclose(M.T @ sim["W"], s * sim["C"], atol=1e-10 * s)
    assert s >= np.linalg.svd(M, compute_uv=False)[0] * (1 - 1e-12)
    assert np.isclose(sim["B_T"], np.linalg.lstsq(sim["Tt"][:, None], sim["U"], rcond=None)[0][0])


@pytest.mark.parametrize("k", [0, 1, 2])
def test_o2m_from_gram_equals_oracle_on_deflated_data(k):
    n, p, q = 600, 25, 18
    X, Y, _ = make_problem(n, p, q, 3, seed=11 + k)
    rng = np.random.default_rng(k)
    # earlier components: unit vectors, deliberately not orthogonal (the deflation is sequential, :270-271)
    Wp = rng.standard_normal((p, k))
    Cp = rng.standard_normal((q, k))
    Wp /= np.linalg.norm(Wp, axis=0) if k else 1.0
    Cp /= np.linalg.norm(Cp, axis=0) if k else 1.0
    Xc, Yc = X.copy(), Y.copy()
    for j in range(k):
        Xc = Xc - np.outer(Xc @ Wp[:, j], Wp[:, j])
        Yc = Yc - np.outer(Yc @ Cp[:, j], Cp[:, j])
    ref = O.initial_guess_o2m(Xc, Yc)
    D = np.hstack([X, Y])
    g = o2m_guess_from_gram(D.T @ D, n, p, q, Wp if k else None, Cp if k else None)
    _close(_align(g, ref), ref, 1e-9)


def test_oracle_ppls_with_o2m_starting_values_runs():
    X, Y, _ = make_problem(300, 12, 9, 2, seed=5)
    fit = O.ppls(X, Y, 2, 30, 1e-6, ["o2m", "o2m"])
    assert fit["W"].shape == (12, 2) and np.all(np.isfinite(fit["B"]))
    assert abs(float(fit["W"][:, 0] @ fit["W"][:, 1])) < 1e-8   # the second fit lives on the deflated X
