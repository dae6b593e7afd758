"""GPU parity of the team single-pass sweep (ppls_team.hip; set_option("sweep", 4), the default for
wide data) against the CPU oracle and against the two-pass panel sweep (sweep = 3).

Tolerances (fp64 arithmetic): log-likelihood 1e-10 relative, W/C 1e-8 absolute, variances 1e-8
relative, Expectations mu 1e-9 relative; team vs panel (the same sums in another order) 1e-11.
fp32 storage is compared with the oracle on the fp32-rounded data (the only fp32 effect).
"""
import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def _fit(X, Y, th0, r, steps, sweep, dtype=0, want_mu=False):
    from ppls_amd import Context, Theta
    with Context(0) as c:
        c.set_option("dtype", dtype)
        c.set_option("sweep", sweep)
        c.set_data(X, Y)
        info = c.sweep_info(r)
        est, ll, eout, _ = c.em_run(Theta(**th0), steps, -np.inf, 0, want_eout=want_mu, want_mu=want_mu)
    return info, est, ll, eout


@pytest.mark.parametrize("dtype,r", [(0, 3), (1, 3), (0, 10), (1, 10), (1, 1)])
def test_team_sweep_matches_oracle(dtype, r):
    # wide enough for a team plan (several workgroups per team), rows not a multiple of anything
    n, p, q = 5003, 2900, 310
    X, Y, th0 = make_problem(n, p, q, r, seed=70 + r + 10 * dtype)
    info, est, ll, eout = _fit(X, Y, th0, r, 6, 4, dtype, want_mu=True)
    assert info["variant"] == "team", info
    if dtype:
        X = X.astype(np.float32).astype(np.float64)
        Y = Y.astype(np.float32).astype(np.float64)
    ref = o.ppls_simult(X, Y, r, EMsteps=6, atol=-np.inf, theta0=th0)
    assert _rel(ll, ref["loglik"]) < 1e-10
    assert np.abs(est.W - ref["estimates"]["W"]).max() < 1e-8
    assert np.abs(est.C - ref["estimates"]["C"]).max() < 1e-8
    assert _rel([est.sigE, est.sigF, est.sigH], [ref["estimates"][k] for k in ("sigE", "sigF", "sigH")]) < 1e-8
    assert _rel(eout.mu_T, ref["Expectations"]["mu_T"]) < 1e-9
    assert _rel(eout.mu_U, ref["Expectations"]["mu_U"]) < 1e-9


def test_team_equals_panel_sweep():
    n, p, q, r = 4100, 3100, 130, 5
    X, Y, th0 = make_problem(n, p, q, r, seed=81)
    it, et, lt, _ = _fit(X, Y, th0, r, 5, 4, 1)
    ip, ep, lp, _ = _fit(X, Y, th0, r, 5, 3, 1)
    assert it["variant"] == "team" and ip["variant"] == "panel"
    assert _rel(lt, lp) < 1e-11
    assert np.abs(et.W - ep.W).max() < 1e-10


def test_team_repeatable_and_small_n_falls_back():
    n, p, q, r = 3000, 2600, 200, 2
    X, Y, th0 = make_problem(n, p, q, r, seed=82)
    _, e1, l1, _ = _fit(X, Y, th0, r, 4, 4, 0)
    _, e2, l2, _ = _fit(X, Y, th0, r, 4, 4, 0)
    assert np.array_equal(l1, l2) and np.array_equal(e1.W, e2.W)   # fixed-order sums: bitwise
    Xs, Ys = X[:50], Y[:50]                                          # too few rows for a team
    info, est, ll, _ = _fit(Xs, Ys, th0, r, 3, 4, 0)
    assert info["variant"] == "panel"
    ref = o.ppls_simult(Xs, Ys, r, EMsteps=3, atol=-np.inf, theta0=th0)
    assert _rel(ll, ref["loglik"]) < 1e-10


def test_team_initialiser_and_meta():
    """The r = 1 paths (sequential PPLS, meta_* row segments) run the team sweep (sweep = 4, opt-in)
    on wide data."""
    import ppls_amd
    from ppls_amd import Context
    X, Y, _ = make_problem(4000, 2700, 140, 1, seed=83)
    init = o.initial_guess(2700, 140, "equal")
    with Context(0) as c:
        c.set_option("sweep", 4)
        c.set_data(X, Y)
        assert c.sweep_info(1)["variant"] == "team"
        f = c.ppls(1, 10, 1e-6, [init])
        m = ppls_amd.meta_PPLSi(None, None, np.repeat([0, 1], [2500, 1500]), EMsteps=8, atol=-np.inf,
                                customGuess=init, ctx=c)
    ref = o.ppls(X, Y, 1, 10, 1e-6, [init])
    assert _rel(f["Other_output"]["logvalue"][0], ref["Other_output"]["logvalue"][0]) < 1e-10
    assert np.abs(f["W"] - ref["W"]).max() < 1e-8
    mref = o.meta_pplsi(X, Y, [2500, 1500], 8, -np.inf, init)
    assert _rel(m["logvalue"], mref["logvalue"]) < 1e-10
