"""The CPU oracle pinned against the reference's own known-answer checks (no GPU)."""
import os

import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as o

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


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
        if not name.endswith(".npz") or name.startswith(("seq_", "meta_", "rcheck_")):
            continue
        g = np.load(os.path.join(here, name))
        meta = json.loads(str(g["meta"]))
        th0 = dict(W=g["W0"], C=g["C0"], B=np.diag(g["B0"]), sigE=float(g["sig0"][0]),
                   sigF=float(g["sig0"][1]), sigH=float(g["sig0"][2]), sigT=np.diag(g["T0"]))
        res = o.ppls_simult(g["X"], g["Y"], meta["r"], EMsteps=meta["EMsteps"], atol=meta["atol"],
                            theta0=th0, type=meta["type"])
        assert np.allclose(res["loglik"], g["loglik"], rtol=1e-12, atol=0), name
        assert np.allclose(res["estimates"]["W"], g["W"], atol=1e-10), name


# ----------------------------------------------------------------------------- sequential initialiser

def test_emstepc_fast_equals_expect_m_rank1():
    """EMstepC_fast (loglC.cpp:340-397) and the closed-form Expect_M (EM_W_multi.R:668-716) are two
    independent statements of the same rank-1 E-step: they must agree (abs() masks inactive)."""
    X, Y, _ = make_problem(180, 12, 9, 1, seed=21)
    rng = np.random.default_rng(2)
    w = rng.standard_normal(12); w /= np.linalg.norm(w)
    c = rng.standard_normal(9); c /= np.linalg.norm(c)
    B, sE, sF, sH, sT = 0.8, 0.7, 0.6, 0.4, 1.1
    f = o.emstep_w(X, Y, w, c, B, sE, sF, sH, sT)
    e = o.expect_m(X, Y, w[:, None], c[:, None], np.array([[B]]), sE, sF, sH, np.array([[sT]]))
    for k in ("Ctt", "Cuu", "Cut", "Cee", "Cff", "Chh"):
        assert np.isclose(f[k], np.ravel(e[k])[0], rtol=1e-12, atol=0), k
    assert np.allclose(f["mu_T"], e["mu_T"][:, 0], rtol=1e-12, atol=1e-12)
    m = o.maximiz_m(e, X, Y)
    assert np.allclose(f["W"], m["W"][:, 0], atol=1e-13)    # orth(v) of a vector = v / ||v||


def test_implicit_deflation_equals_explicit():
    """The device path never forms Xc = X (I - w1 w1'): its sweep uses the weight P w on X and
    projects X' mu_T.  Check that algebra against the explicit deflation of EM_W_multi.R:270-271."""
    X, Y, _ = make_problem(160, 14, 11, 2, seed=22)
    f1 = o.pplsi(X, Y, 20, 1e-4, o.initial_guess(14, 11, "equal"))
    w1, c1 = f1["W"], f1["C"]
    Xc = X - np.outer(X @ w1, w1)
    Yc = Y - np.outer(Y @ c1, c1)
    th = o.initial_guess(14, 11, "random", np.random.default_rng(5))
    ref = o.emstep_w(Xc, Yc, th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])
    Pw = th["W"] - w1 * (w1 @ th["W"])
    Pc = th["C"] - c1 * (c1 @ th["C"])
    assert np.allclose(Xc @ th["W"], X @ Pw, atol=1e-12)
    # X'mu_T projected == Xc'mu_T ; ||Xc||^2 == ||X||^2 - ||Xc w1||^2
    mu = ref["mu_T"]
    SX = X.T @ mu
    assert np.allclose(SX - w1 * (w1 @ SX), Xc.T @ mu, atol=1e-10)
    assert np.isclose(o.ssq(Xc), o.ssq(X) - np.sum((X @ w1) ** 2), rtol=1e-12)


def test_ppls_loadings_orthonormal_and_golden_reproduced():
    import json
    for name in ("seq_equal_n200_p30_q25_a3", "seq_random_n240_p36_q20_a2", "seq_equal_atol_n150_p16_q12_a2"):
        g = np.load(os.path.join(GOLDEN, name + ".npz"))
        meta = json.loads(str(g["meta"]))
        a = meta["a"]
        inits = [dict(W=g["init_W"][:, k], C=g["init_C"][:, k], B=g["init_s"][k, 0], sigE=g["init_s"][k, 1],
                      sigF=g["init_s"][k, 2], sigH=g["init_s"][k, 3], sigT=g["init_s"][k, 4]) for k in range(a)]
        f = o.ppls(g["X"], g["Y"], a, meta["EMsteps"], meta["atol"], inits)
        assert np.array_equal(f["W"], g["W"]) and np.array_equal(f["sig"], g["sig"])
        assert list(f["Other_output"]["Number_steps"]) == list(g["number_steps"])
        assert np.allclose(f["W"].T @ f["W"], np.eye(a), atol=1e-12)
        assert np.allclose(f["C"].T @ f["C"], np.eye(a), atol=1e-12)
        for lv in f["Other_output"]["logvalue"]:
            assert np.all(np.diff(lv) > -1e-8 * np.abs(lv[:-1]))      # EM monotone


# ----------------------------------------------------------------------------- meta_* (multi-population)

def _meta_fixture(name):
    import json
    g = np.load(os.path.join(GOLDEN, name))
    return g, json.loads(str(g["meta"]))


def _meta_init(g):
    s = g["init_s"]
    return dict(W=g["init_W"], C=g["init_C"], B=s[0], sigE=s[1], sigF=s[2], sigH=s[3], sigT=s[4])


def test_meta_single_population_equals_pplsi():
    # with one population meta_EMstep's orth(sum) is EMstepC_fast's Cxt.normalized() and the stop rule is
    # PPLSi's: the two independent reference code paths must agree
    X, Y, _ = make_problem(150, 14, 11, 1, seed=31)
    init = o.initial_guess(14, 11, "equal")
    a = o.pplsi(X, Y, 40, 1e-5, init)
    m = o.meta_pplsi(X, Y, [150], 40, 1e-5, init)
    assert m["logvalue"].shape[0] - 1 == a["Number_steps"]
    assert np.abs(m["logvalue"][:, 0] - a["logvalue"]).max() / abs(a["logvalue"][-1]) < 1e-13
    assert np.abs(m["W"] - a["W"]).max() < 1e-12 and np.abs(m["C"] - a["C"]).max() < 1e-12
    p0 = m["params"][0]
    assert np.allclose([p0["B_T"], p0["sigX"], p0["sigY"], p0["sigH"], p0["sigT"]],
                       [a["B"], *a["sig"]], rtol=1e-12, atol=0)


def test_meta_estep_matches_closed_form_expect_m_rank1():
    # meta_Estep (loglC.cpp:399-448) vs the independent closed-form Expect_M at r = 1 (EM_W_multi.R:668-716)
    X, Y, th = make_problem(90, 12, 10, 1, seed=32)
    B, sE, sF, sH, sT = th["B"][0, 0], th["sigE"], th["sigF"], th["sigH"], th["sigT"][0, 0]
    cf = o.coefficients(np.array([B]), sE, sF, sH, np.array([sT]))
    e = o.meta_estep(th["W"][:, 0], th["C"][:, 0], B, X, Y, sE, sF, sH, sT, cf["c1"][0], cf["c2"][0], cf["c3"][0])
    E = o.expect_m(X, Y, th["W"], th["C"], th["B"], sE, sF, sH, th["sigT"])
    assert np.abs(e["mu_T"] - E["mu_T"][:, 0]).max() < 1e-12
    assert abs(e["Ctt"] - E["Ctt"][0, 0]) < 1e-12 and abs(e["Cut"] - E["Cut"][0, 0]) < 1e-12
    assert abs(e["Cee"] - E["Cee"][0, 0]) < 1e-12 and abs(e["Chh"] - E["Chh"][0, 0]) < 1e-12
    assert np.abs(e["Cxt"] - X.T @ E["mu_T"][:, 0] / 90).max() < 1e-12


@pytest.mark.parametrize("name", ["meta_equal_k2_p30_q20.npz", "meta_random_k3_p24_q18.npz"])
def test_meta_golden_reproduces(name):
    g, meta = _meta_fixture(name)
    f = o.meta_pplsi(g["X"], g["Y"], meta["sizes"], meta["EMsteps"], meta["atol"], _meta_init(g))
    assert f["logvalue"].shape[0] - 1 == meta["steps"]
    assert np.array_equal(f["logvalue"], g["logvalue"]) and np.array_equal(f["W"], g["W"])
    # the EM never decreases the summed log-likelihood after the first step (row 0 is rep(full, K))
    assert np.all(np.diff(g["logvalue"][1:].sum(1)) > -1e-9)


def test_variances_restatement_equals_literal_nxn_form():
    # variances.PPLS_simult (EM_W_multi.R:846) forms t(X) %*% diag(c(Ctt), N) %*% X with an N x N
    # diagonal; the oracle (and the device) use Ctt * X'X -- the same matrix
    X, Y, th0 = make_problem(60, 7, 5, 2, seed=51)
    fit = o.ppls_simult(X, Y, 2, EMsteps=5, atol=-np.inf, theta0=th0)
    v = o.variances_ppls_simult(fit, X, "X")
    N = X.shape[0]
    E, sE = fit["Expectations"], fit["estimates"]["sigE"]
    for i in range(2):
        Ctt = N * E["Ctt"][i, i]
        mu = E["mu_T"][:, i]
        w = v["W"][:, [i]]
        Vt = Ctt - mu @ mu
        Cxt = (X.T @ mu)[:, None]
        lit = (X.T @ np.diag(np.full(N, Ctt)) @ X - Cxt * (Ctt + 2 * Vt) @ w.T - w * (Ctt + 2 * Vt) @ Cxt.T
               + w * (Ctt ** 2 + 4 * (mu @ mu) * Vt + 2 * Vt * Vt) @ w.T) / sE ** 4 / N
        assert np.abs(lit - v["components"][i]["SSt_exp"]).max() < 1e-12 * np.abs(lit).max()
        # -solve(B_exp - SSt_exp) is a symmetric matrix; its diagonal gives seLoad
        V = v["varMatrix"][i]
        assert np.abs(V - V.T).max() < 1e-10 * np.abs(V).max()
        assert np.allclose(v["seLoad"][:, i] ** 2, np.diag(V), rtol=1e-12)


def test_pplsi_constraints_hold_and_free_fit_is_unchanged():
    # fconstraint (EM_W_multi.R:85-92): fixed values persist through every EM step (:165-169);
    # no constraints (all NULL) is the plain PPLSi
    X, Y, _ = make_problem(120, 9, 7, 1, seed=58)
    init = o.initial_guess(9, 7, "equal")
    free = o.pplsi(X, Y, 30, 1e-6, init)
    same = o.pplsi(X, Y, 30, 1e-6, init, o.fconstraint())
    assert np.array_equal(free["logvalue"], same["logvalue"])
    cfix = np.ones(7) / np.sqrt(7.0)
    fixed = o.pplsi(X, Y, 30, 1e-6, init, o.fconstraint(dict(sigH=0.25, C=cfix)))
    assert fixed["sig"][2] == 0.25 and np.array_equal(fixed["C"], cfix)
