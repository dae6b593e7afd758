"""GPU parity of the sequential initialiser PPLS(X, Y, a, EMsteps, atol, initialGuess)
(EM_W_multi.R:229-279, PPLSi :116-180, EMstepC_fast loglC.cpp:340-397) against the oracle's
explicit-deflation restatement and the golden fixtures tests/golden/seq_*.npz.

Tolerances (fp64): log-likelihoods 1e-10 relative; loadings 1e-8 absolute (unit vectors);
B, sigmas 1e-8 relative; step counts exact (the early-stop case stops on increments far from
atol).  The device path deflates implicitly (weights P w, projected X'mu_T), so agreement is to
rounding, not bitwise.
"""
import json
import os
import warnings

import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
SEQ = sorted(f for f in os.listdir(GOLD) if f.startswith("seq_") and f.endswith(".npz"))


@pytest.fixture(scope="module", params=[0, 1], ids=["stream", "xprod"])
def ctx(request):
    """Every test on both statistics paths: streaming sweeps, and the cross-products S (option xprod)."""
    from ppls_amd import Context
    c = Context(0)
    c.set_option("xprod", request.param)
    yield c
    c.close()


def _relerr(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def _inits(g, a):
    return [dict(W=g["init_W"][:, k], C=g["init_C"][:, k], B=g["init_s"][k, 0], sigE=g["init_s"][k, 1],
                 sigF=g["init_s"][k, 2], sigH=g["init_s"][k, 3], sigT=g["init_s"][k, 4]) for k in range(a)]


@pytest.mark.parametrize("name", SEQ)
def test_ppls_matches_golden(ctx, name):
    g = np.load(os.path.join(GOLD, name))
    meta = json.loads(str(g["meta"]))
    a = meta["a"]
    ctx.set_data(g["X"], g["Y"])
    f = ctx.ppls(a, meta["EMsteps"], meta["atol"], _inits(g, a))
    oo = f["Other_output"]
    assert list(oo["Number_steps"]) == list(g["number_steps"])
    assert np.abs(f["W"] - g["W"]).max() < 1e-8
    assert np.abs(f["C"] - g["C"]).max() < 1e-8
    assert _relerr(f["B"], g["B"]) < 1e-8
    assert _relerr(f["sig"], g["sig"]) < 1e-8
    assert _relerr(oo["Loglikelihoods"], g["loglikelihoods"]) < 1e-10
    for k in range(a):
        ref = g["logvalue"][k, :g["number_steps"][k] + 1]
        assert _relerr(oo["logvalue"][k], ref) < 1e-10
    assert np.abs(oo["Last_increment"] - g["last_increment"]).max() < 1e-6 * np.abs(g["loglikelihoods"]).max()


@pytest.mark.parametrize("name", SEQ[:2])
def test_simult_from_device_init_matches_golden(ctx, name):
    """PPLS_simult seeded by the device PPLS fit (:764-770) == the oracle chain."""
    from ppls_amd import PPLS_simult
    g = np.load(os.path.join(GOLD, name))
    meta = json.loads(str(g["meta"]))
    a = meta["a"]
    ctx.set_data(g["X"], g["Y"])
    f = ctx.ppls(a, meta["EMsteps"], meta["atol"], _inits(g, a))
    init = dict(W=f["W"], C=f["C"], B=np.diag(f["B"]), sigE=f["sig"][a - 1, 0], sigF=f["sig"][a - 1, 1],
                sigH=f["sig"][a - 1, 2], sigT=np.diag(f["sig"][:, 3]))
    res = PPLS_simult(None, None, a, EMsteps=10, atol=1e-4, init=init, ctx=ctx)
    assert len(res["loglik"]) == len(g["simult_loglik"])
    assert _relerr(res["loglik"], g["simult_loglik"]) < 1e-9
    assert np.abs(res["estimates"]["W"] - g["simult_W"]).max() < 1e-7


def test_ppls_r_mirror_random_and_default_simult(ctx):
    """R-mirror PPLS(..., 'random') with a seeded generator == ctx.ppls on the same draws; the
    default PPLS_simult (device f0, :762) runs and its likelihood is monotone."""
    from ppls_amd import PPLS, PPLS_simult, PPLSi, initial_guess
    X, Y, _ = make_problem(300, 22, 17, 3, seed=31)
    f = PPLS(X, Y, 3, 20, 1e-4, "random", rng=np.random.default_rng(7), ctx=ctx)
    rng = np.random.default_rng(7)
    inits = [initial_guess(22, 17, "random", rng) for _ in range(3)]
    ref = o.ppls(X, Y, 3, 20, 1e-4, inits)
    assert f["class"] == "PPLS"
    assert np.abs(f["W"] - ref["W"]).max() < 1e-8
    assert _relerr(f["sig"], ref["sig"]) < 1e-8
    one = PPLSi(X, Y, 20, 1e-4, "equal", ctx=ctx)
    r1 = o.pplsi(X, Y, 20, 1e-4, o.initial_guess(22, 17, "equal"))
    assert np.abs(one["W"] - r1["W"]).max() < 1e-8 and one["Number_steps"] == r1["Number_steps"]
    res = PPLS_simult(X, Y, 3, EMsteps=15, atol=-np.inf, seed=3, ctx=ctx)
    assert np.all(np.diff(res["loglik"]) > -1e-9 * np.abs(res["loglik"][:-1]))


def test_ppls_collapse_stops_like_reference(ctx):
    """A start with sigE below 100 eps makes PPLSi return NA (:152-154); PPLS keeps the
    components before it (:258-263)."""
    from ppls_amd import PPLS
    X, Y, _ = make_problem(200, 15, 12, 2, seed=32)
    good = o.initial_guess(15, 12, "equal")
    bad = dict(good, sigE=1e-15)
    ref = o.ppls(X, Y, 2, 20, 1e-4, [good, bad])
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        f = PPLS(X, Y, 2, 20, 1e-4, customGuess=[good, bad], ctx=ctx)
    assert f["W"].shape == ref["W"].shape == (15, 1)
    assert np.abs(f["W"] - ref["W"]).max() < 1e-8
    assert any("rank" in str(x.message) for x in w)


def test_ppls_multi_component_shapes_and_orthogonality(ctx):
    X, Y, _ = make_problem(400, 40, 30, 5, seed=33)
    ctx.set_data(X, Y)
    from ppls_amd import initial_guess
    f = ctx.ppls(5, 20, 1e-4, [initial_guess(40, 30, "equal")] * 5)
    ref = o.ppls(X, Y, 5, 20, 1e-4, [o.initial_guess(40, 30, "equal")] * 5)
    assert np.allclose(f["W"].T @ f["W"], np.eye(5), atol=1e-12)
    assert np.abs(f["W"] - ref["W"]).max() < 1e-8
    assert _relerr(f["Other_output"]["Loglikelihoods"], ref["Other_output"]["Loglikelihoods"]) < 1e-10


def test_scores_and_to_o2m_match_oracle(ctx):
    """scores.PPLS (:411-420) through the one-pass device kernel and PPLS_simult_to_o2m
    (PPLS_to_o2m.R:82-140) on a device fit, against the oracle restatements."""
    from ppls_amd import PPLS_simult, PPLS_simult_to_o2m, scores_PPLS
    X, Y, th0 = make_problem(350, 26, 21, 3, seed=51)
    fit = PPLS_simult(X, Y, 3, EMsteps=8, atol=-np.inf, init=th0, ctx=ctx)
    sc = scores_PPLS(fit, X, Y, ctx=ctx)
    ref = o.scores_ppls(fit["estimates"]["W"], fit["estimates"]["C"], X, Y)
    assert sc.shape == (700, 3) and np.abs(sc - ref).max() < 1e-11 * np.abs(ref).max()
    one = scores_PPLS(fit, None, None, subset=2, ctx=ctx)
    assert np.allclose(one, o.scores_ppls(fit["estimates"]["W"], fit["estimates"]["C"], X, Y, subset=2),
                       rtol=1e-12, atol=1e-12)
    m = PPLS_simult_to_o2m(None, None, fit, ctx=ctx)
    r = o.ppls_simult_to_o2m(X, Y, fit)
    for key in ("R2Xcorr", "R2Ycorr", "R2Yhat"):
        assert np.isclose(m[key], r[key], rtol=1e-13), key
    assert np.allclose(m["H_UT"], r["H_UT"], atol=1e-12)
    assert np.isclose(m["flags"]["ssqX"], r["ssqX"], rtol=1e-12)


def test_ppls_to_o2m_matches_oracle(ctx):
    """PPLS_to_o2m (PPLS_to_o2m.R:28-80) on a device sequential fit: scores from one device pass,
    R2 terms as r x r traces, against the literal n x p restatement."""
    from ppls_amd import PPLS, PPLS_to_o2m
    X, Y, _ = make_problem(330, 24, 19, 2, seed=53)
    f = PPLS(X, Y, 2, EMsteps=30, atol=1e-6, initialGuess="equal", ctx=ctx)
    m = PPLS_to_o2m(None, None, f, ctx=ctx)
    r = o.ppls_to_o2m(X, Y, f)
    for key in ("R2Xcorr", "R2Ycorr", "R2Xhat", "R2Yhat"):
        assert np.isclose(m[key], r[key], rtol=1e-12), key
    assert np.allclose(m["Tt"], r["Tt"], rtol=1e-12, atol=1e-12)
    assert np.allclose(m["H_UT"], r["H_UT"], rtol=1e-12, atol=1e-12)
    assert np.allclose(m["B_U"], r["B_U"], rtol=1e-14)


def test_scores_fp32_storage(ctx):
    from ppls_amd import Context
    X, Y, th0 = make_problem(300, 33, 17, 2, seed=52)
    with Context(0) as c32:
        c32.set_option("dtype", 1)
        c32.set_data(X, Y)
        T, U = c32.scores(th0["W"], th0["C"])
    X32 = X.astype(np.float32).astype(np.float64)
    Y32 = Y.astype(np.float32).astype(np.float64)
    assert np.allclose(T, X32 @ th0["W"], rtol=1e-12, atol=1e-12)
    assert np.allclose(U, Y32 @ th0["C"], rtol=1e-12, atol=1e-12)


def test_ppls_constraints_and_critfunc_match_oracle(ctx):
    """PPLS / PPLSi with fconstraint (EM_W_multi.R:85-92, :141-145, :165-169) and critfunc = abs:
    component 1 fixes B and sigT, component 2 fixes W (not orthogonal to w_1), so the deflation and the
    Loglikelihoods take the non-orthogonal route; the rest is estimated."""
    import ppls_amd
    X, Y, _ = make_problem(260, 21, 17, 2, seed=57)
    p, q = 21, 17
    inits = [o.initial_guess(p, q, "equal") for _ in range(2)]
    wfix = np.linspace(1.0, 2.0, p)
    wfix /= np.linalg.norm(wfix)                         # a unit vector not orthogonal to w_1
    cons = [ppls_amd.fconstraint(dict(B=0.8, sigT=1.3)), ppls_amd.fconstraint(dict(W=wfix))]
    ctx.set_data(X, Y)
    f = ppls_amd.PPLS(None, None, 2, 25, 1e-6, customGuess=inits, critfunc=abs, constraints=cons, ctx=ctx)
    ref = o.ppls(X, Y, 2, 25, 1e-6, inits, constraints=cons, critfunc=abs)
    oo, ro = f["Other_output"], ref["Other_output"]
    assert list(oo["Number_steps"]) == list(ro["Number_steps"])
    assert f["B"][0] == 0.8 and f["sig"][0, 3] == 1.3
    assert np.array_equal(f["W"][:, 1], wfix)
    assert np.abs(f["W"] - ref["W"]).max() < 1e-8 and np.abs(f["C"] - ref["C"]).max() < 1e-8
    assert _relerr(f["sig"], ref["sig"]) < 1e-8
    for k in range(2):
        assert _relerr(oo["logvalue"][k], ro["logvalue"][k]) < 1e-10
    assert _relerr(oo["Loglikelihoods"], ro["Loglikelihoods"]) < 1e-10
    one = ppls_amd.PPLSi(None, None, 25, 1e-6, customGuess=inits[0], constraints=cons[0], ctx=ctx)
    assert one["B"] == 0.8 and one["sig"][3] == 1.3
    with pytest.raises(ValueError):
        ppls_amd.PPLS(None, None, 2, 5, 1e-4, constraints=cons[:1], ctx=ctx)   # one list per component
