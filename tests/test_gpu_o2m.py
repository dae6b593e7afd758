"""initialGuess = "o2m" (EM_W_multi.R:126-131 in PPLSi, :520-525 in meta_PPLSi; OmicsPLS::o2m not
vendored -- restated in oracle.ppls_oracle.o2m_1, parity unpinned against R): the product's starting
values come from the device's joint Gram with the earlier components' deflation applied
algebraically (api.o2m_guess_from_gram), the oracle's from the explicitly deflated data; the fits
from them agree to rounding (loadings 1e-8 absolute, B and sigmas 1e-8 relative, log-likelihoods
1e-10 relative, step counts exact).  A singular pair's sign is LAPACK's: the loadings are compared
after flipping W and C together when they point the other way."""
import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[0, 1], ids=["stream", "xprod"])
def ctx(request):
    from ppls_amd import Context
    c = Context(0)
    c.set_option("xprod", request.param)
    yield c
    c.close()


def _relerr(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def _aligned(W, C, Wr):
    W, C = np.array(W, dtype=float, ndmin=2).reshape(len(W), -1), np.array(C, dtype=float).reshape(len(C), -1)
    s = np.sign(np.sum(W * np.asarray(Wr).reshape(W.shape), axis=0))
    return W * s, C * s


@pytest.mark.parametrize("n,p,q,a", [(500, 30, 20, 3), (2000, 120, 45, 2)])
def test_ppls_o2m_matches_oracle(ctx, n, p, q, a):
    from ppls_amd import PPLS
    X, Y, _ = make_problem(n, p, q, a, seed=n + p)
    f = PPLS(X, Y, a, 40, 1e-6, "o2m", ctx=ctx)
    ref = o.ppls(X, Y, a, 40, 1e-6, ["o2m"] * a)
    W, C = _aligned(f["W"], f["C"], ref["W"])
    assert W.shape == ref["W"].shape
    assert np.abs(W - ref["W"]).max() < 1e-8 and np.abs(C - ref["C"]).max() < 1e-8
    assert _relerr(f["B"], ref["B"]) < 1e-8 and _relerr(f["sig"], ref["sig"]) < 1e-8
    oo = f["Other_output"]
    assert list(oo["Number_steps"]) == list(ref["Other_output"]["Number_steps"])
    assert _relerr(oo["Loglikelihoods"], ref["Other_output"]["Loglikelihoods"]) < 1e-10
    assert np.allclose(f["W"].T @ f["W"], np.eye(a), atol=1e-10)


def test_pplsi_o2m_starts_at_the_oracle_values(ctx):
    """PPLSi: the first log-likelihood of the trace is that of the o2m starting values (:149)."""
    from ppls_amd import PPLSi
    X, Y, _ = make_problem(800, 50, 35, 1, seed=9)
    one = PPLSi(X, Y, 25, 1e-8, "o2m", ctx=ctx)
    th = o.initial_guess_o2m(X, Y)
    r1 = o.pplsi(X, Y, 25, 1e-8, th)
    assert _relerr(one["logvalue"], r1["logvalue"]) < 1e-10
    W, C = _aligned(one["W"], one["C"], r1["W"])
    assert np.abs(W.ravel() - r1["W"]).max() < 1e-8 and one["Number_steps"] == r1["Number_steps"]


def test_meta_pplsi_o2m_matches_oracle(ctx):
    import ppls_amd
    X, Y, _ = make_problem(300, 26, 14, 1, seed=12)
    Ipopu = np.repeat([0, 1, 2], [80, 120, 100])
    m = ppls_amd.meta_PPLSi(X, Y, Ipopu, EMsteps=20, atol=-np.inf, initialGuess="o2m", ctx=ctx)
    ref = o.meta_pplsi(X, Y, [80, 120, 100], 20, -np.inf, o.initial_guess_o2m(X, Y))
    W, C = _aligned(m["W"], m["C"], ref["W"])
    assert np.abs(W.ravel() - np.ravel(ref["W"])).max() < 1e-8
    assert np.abs(C.ravel() - np.ravel(ref["C"])).max() < 1e-8
    assert _relerr(m["logvalue"], ref["logvalue"]) < 1e-10
