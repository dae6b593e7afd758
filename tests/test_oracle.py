"""The CPU oracle pinned against the reference's own known-answer checks (no GPU)."""
import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as o


@pytest.mark.parametrize("r", [1, 2, 3])
def test_closed_form_inverse_rank_one_inverse_R(r):
    # Package/rank_one_inverse.R:59: closed-form Sigma^-1 == solve(sseXY_W())
    X, Y, th = make_problem(50, 12, 9, r, seed=r)
    cf = o.coefficients(th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])
    W, C = th["W"], th["C"]
    S = o.sse_xy_w(W, C, th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])
    closed = o.blockm(-W @ np.diag(cf["c1"]) @ W.T + np.eye(12) / th["sigE"] ** 2,
                      -W @ np.diag(cf["c2"]) @ C.T,
                      -C @ np.diag(cf["c3"]) @ C.T + np.eye(9) / th["sigF"] ** 2)
    inv = np.linalg.inv(S)
    assert np.abs(closed - inv).max() / np.abs(inv).max() < 1e-13


@pytest.mark.parametrize("r", [1, 3])
def test_loglik_trace_identity_benchmark_R(r):
    # Package/Benchmark.R:36-45: tr(S Sigma^-1) == the closed-form quadratic of loglC_fast;
    # full check: loglC_fast == the dense Gaussian log-likelihood
    X, Y, th = make_problem(80, 10, 8, r, seed=10 + r)
    ll = o.logl_w(X, Y, th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])
    S = o.sse_xy_w(th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])
    XY = np.hstack([X, Y])
    _, ld = np.linalg.slogdet(S)
    dense = -0.5 * 80 * 18 * np.log(2 * np.pi) - 0.5 * 80 * ld - 0.5 * np.sum((XY @ np.linalg.inv(S)) * XY)
    assert abs(ll - dense) / abs(dense) < 1e-13


@pytest.mark.parametrize("r", [1, 2, 4])
def test_closed_form_estep_matches_dense_debug_branch(r):
    # Expect_M closed form (:668-714) vs Expect_M(debug=TRUE) (:643-667)
    X, Y, th = make_problem(60, 14, 11, r, seed=20 + r)
    args = (X, Y, th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])
    a, b = o.expect_m(*args), o.expect_m_dense(*args)
    for k in a:
        scale = max(np.abs(b[k]).max(), 1e-300)
        assert np.abs(a[k] - b[k]).max() / scale < 1e-12, k


def test_em_monotone_and_recovers_truth():
    X, Y, th = make_problem(400, 30, 25, 2, seed=3)
    res = o.ppls_simult(X, Y, 2, EMsteps=40, atol=-np.inf, theta0=th)
    assert np.all(np.diff(res["loglik"]) > -1e-9)
    assert not res["warning_negative"]


def test_sweep_statistics_identities():
    # the build's one-pass sufficient statistics reproduce Expect_M's moments
    X, Y, th = make_problem(70, 13, 7, 3, seed=5)
    cf = o.mu_coefficients(th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])
    st = o.sweep_stats(X, Y, th["W"], th["C"], cf)
    e = o.expect_m(X, Y, th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])
    assert np.allclose(st["mu_T"], e["mu_T"], rtol=1e-12, atol=1e-12)
    assert np.allclose(st["mu_U"], e["mu_U"], rtol=1e-12, atol=1e-12)
    m = o.maximiz_m(e, X, Y)
    assert np.allclose(o.orth(st["SX"]), m["W"], atol=1e-12)


def test_golden_fixtures_reproduce():
    import json, os
    here = os.path.join(os.path.dirname(__file__), "golden")
    for name in sorted(os.listdir(here)):
        if not name.endswith(".npz"):
            continue
        g = np.load(os.path.join(here, name))
        meta = json.loads(str(g["meta"]))
        th0 = dict(W=g["W0"], C=g["C0"], B=np.diag(g["B0"]), sigE=float(g["sig0"][0]),
                   sigF=float(g["sig0"][1]), sigH=float(g["sig0"][2]), sigT=np.diag(g["T0"]))
        res = o.ppls_simult(g["X"], g["Y"], meta["r"], EMsteps=meta["EMsteps"], atol=meta["atol"],
                            theta0=th0, type=meta["type"])
        assert np.allclose(res["loglik"], g["loglik"], rtol=1e-12, atol=0), name
        assert np.allclose(res["estimates"]["W"], g["W"], atol=1e-10), name
