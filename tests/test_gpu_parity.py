"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the golden fixtures.

Tolerances (fp64 throughout): log-likelihood 1e-10 relative; loadings W, C 1e-8 absolute on
unit-norm columns (BASELINE.json: "loadings within 1e-8 rel-err"); variances / B / sigT 1e-8
relative; moments 1e-9 relative.
"""
import json
import os

import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
# sweep-kernel variants (context options): split ownership (default; auto = 2 rows per step,
# occupancy grid), split 1 row/step pipelined / unpipelined, the same with non-temporal loads,
# panel (wide p) with 32 and (option dots_rows, auto below 32768 rows = 32) 64 rows per dots wave;
# the panel accumulation over few long row chunks (acc_chunks)
SWEEPS = [dict(), dict(rows_per_step=1, pipe=1), dict(rows_per_step=1, pipe=0), dict(nt=1),
          dict(sweep=3), dict(sweep=3, dots_rows=64), dict(sweep=3, dots_rows=64, dots_pair=0, nt=1),
          dict(sweep=3, acc_chunks=1), dict(sweep=3, acc_chunks=3, nt=1)]
SWEEP_IDS = ["split", "split_rp1", "split_rp1_nopipe", "split_nt", "panel", "panel_rows64", "panel_nt_single",
             "panel_chunks1", "panel_chunks3_nt"]
DEFAULTS = dict(sweep=0, grid=0, rows_per_step=0, pipe=1, nt=-1, dots_rows=0, dots_pair=-1, acc_chunks=0)


@pytest.fixture(scope="module")
def ctx():
    from ppls_amd import Context
    c = Context(0)
    yield c
    c.close()


@pytest.fixture(autouse=True)
def _reset_options(ctx):
    for k, v in DEFAULTS.items():
        ctx.set_option(k, v)
    yield


def _apply(ctx, opts):
    for k, v in opts.items():
        ctx.set_option(k, v)


def _theta(th):
    from ppls_amd import Theta
    return Theta(th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])


def _relerr(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def _golden():
    return sorted(f for f in os.listdir(GOLD) if f.endswith(".npz") and not f.startswith(("seq_", "meta_", "rcheck_")))


@pytest.mark.parametrize("sweep", SWEEPS, ids=SWEEP_IDS)
@pytest.mark.parametrize("name", _golden())
def test_em_run_matches_golden(ctx, name, sweep):
    g = np.load(os.path.join(GOLD, name))
    meta = json.loads(str(g["meta"]))
    _apply(ctx, sweep)
    ctx.set_data(g["X"], g["Y"])
    th0 = dict(W=g["W0"], C=g["C0"], B=np.diag(g["B0"]), sigE=g["sig0"][0], sigF=g["sig0"][1],
               sigH=g["sig0"][2], sigT=np.diag(g["T0"]))
    typ = 0 if meta["type"] == "SVD" else 1
    est, ll, eout, neg = ctx.em_run(_theta(th0), meta["EMsteps"], meta["atol"], typ)
    assert len(ll) == meta["steps_done"]
    assert _relerr(ll, g["loglik"]) < 1e-10
    assert np.abs(est.W - g["W"]).max() < 1e-8
    assert np.abs(est.C - g["C"]).max() < 1e-8
    assert _relerr(est.B, g["B"]) < 1e-8
    assert _relerr(est.sigT, g["T"]) < 1e-8
    assert _relerr([est.sigE, est.sigF, est.sigH], g["sig"]) < 1e-8
    assert _relerr(eout.mu_T, g["mu_T"]) < 1e-8
    assert _relerr(eout.mu_U, g["mu_U"]) < 1e-8
    assert _relerr(eout.Ctt, g["Ctt"]) < 1e-8
    assert _relerr(eout.Cut, g["Cut"]) < 1e-8
    assert _relerr(eout.Chh, g["Chh"]) < 1e-8
    assert abs(eout.Cee - g["Cee"]) / g["Cee"] < 1e-8
    assert abs(eout.Cff - g["Cff"]) / g["Cff"] < 1e-8
    assert not neg


@pytest.mark.parametrize("sweep", SWEEPS, ids=SWEEP_IDS)
@pytest.mark.parametrize("n,p,q,r", [(200, 50, 50, 2), (97, 33, 7, 1), (301, 64, 31, 5), (50, 9, 12, 8),
                                     (3, 5, 4, 2), (1, 6, 3, 1), (700, 1025, 3, 2), (400, 3, 1500, 3),
                                     (150, 17, 14, 10), (90, 24, 20, 16), (120, 2600, 9, 3)])
def test_estep_mstep_loglik_vs_oracle(ctx, sweep, n, p, q, r):
    X, Y, th0 = make_problem(n, p, q, r, seed=n + p + q + r)
    _apply(ctx, sweep)
    ctx.set_data(X, Y)
    th = _theta(th0)
    e = ctx.estep(th)
    ref = o.expect_m(X, Y, th0["W"], th0["C"], th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    assert _relerr(e.mu_T, ref["mu_T"]) < 1e-11
    assert _relerr(e.mu_U, ref["mu_U"]) < 1e-11
    assert _relerr(e.Ctt, np.diag(ref["Ctt"])) < 1e-10
    assert _relerr(e.Cuu, np.diag(ref["Cuu"])) < 1e-10
    assert _relerr(e.Cut, np.diag(ref["Cut"])) < 1e-10
    assert abs(e.Cee - ref["Cee"][0, 0]) / ref["Cee"][0, 0] < 1e-10
    assert abs(e.Cff - ref["Cff"][0, 0]) / ref["Cff"][0, 0] < 1e-10
    assert _relerr(e.Chh, ref["Chh"]) < 1e-9
    if n >= r:
        nx, _ = ctx.em_step(th)
        m = o.maximiz_m(ref, X, Y)
        assert np.abs(nx.W - m["W"]).max() < 1e-10
        assert np.abs(nx.C - m["C"]).max() < 1e-10
        assert _relerr(nx.B, np.diag(m["B"])) < 1e-10
        assert _relerr(nx.sigT, np.diag(m["sigT"])) < 1e-10
        assert _relerr([nx.sigE, nx.sigF, nx.sigH], [m["sigE"], m["sigF"], m["sigH"]]) < 1e-10
        # Maximiz_M from an explicit fit (the accumulate pass with mu given)
        mm = ctx.mstep(e)
        assert np.abs(mm.W - m["W"]).max() < 1e-10
        assert np.abs(mm.C - m["C"]).max() < 1e-10
    ll = ctx.loglik(th)
    ref_ll = o.logl_w(X, Y, th0["W"], th0["C"], th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    assert abs(ll - ref_ll) / abs(ref_ll) < 1e-11


def test_fewer_columns_than_components_is_an_argument_error(ctx):
    from ppls_amd import PplsError
    X, Y, th0 = make_problem(50, 4, 6, 2, seed=1)
    ctx.set_data(X[:, :1], Y)
    with pytest.raises(PplsError, match="must be >= number of components"):
        ctx.estep(_theta(dict(th0, W=th0["W"][:1])))


def test_loglC_fast_dropin(ctx):
    from ppls_amd import loglC_fast
    X, Y, th0 = make_problem(123, 20, 15, 3, seed=77)
    cf = o.logl_coefficients(th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    args = (th0["W"], th0["C"], X, Y, th0["sigE"], th0["sigF"], cf["sig2T"], cf["c1"], cf["c2"], cf["c3"], cf["Kc"])
    ref = o.loglc_fast(*args)
    got = loglC_fast(*args, ctx=ctx)
    assert abs(got - ref) / abs(ref) < 1e-12
    # zero-copy form on resident data
    got2 = ctx.loglC_fast(th0["W"], th0["C"], None, None, *args[4:])
    assert abs(got2 - ref) / abs(ref) < 1e-12


def test_colmajor_and_rowmajor_uploads_agree(ctx):
    X, Y, th0 = make_problem(150, 21, 19, 2, seed=5)
    ctx.set_option("sweep", 0)
    ctx.set_data(np.asfortranarray(X), np.asfortranarray(Y))
    a = ctx.estep(_theta(th0))
    Xb, Yb = ctx.get_data()
    assert np.array_equal(Xb, X) and np.array_equal(Yb, Y)
    Xr, Yr = ctx.get_data_rows(17, 100)
    assert Xr.flags.c_contiguous and np.array_equal(Xr, X[17:117]) and np.array_equal(Yr, Y[17:117])
    ctx.set_data(np.ascontiguousarray(X), np.ascontiguousarray(Y))
    b = ctx.estep(_theta(th0))
    assert np.array_equal(a.mu_T, b.mu_T) and a.Cee == b.Cee


@pytest.mark.parametrize("grid", [1, 7, 256, 1000])
def test_grid_invariance(ctx, grid):
    X, Y, th0 = make_problem(2000, 130, 90, 3, seed=11)
    ctx.set_option("sweep", 0)
    ctx.set_data(X, Y)
    ctx.set_option("grid", 0)
    a = ctx.estep(_theta(th0))
    ctx.set_option("grid", grid)
    b = ctx.estep(_theta(th0))
    ctx.set_option("grid", 0)
    assert _relerr(b.Ctt, a.Ctt) < 1e-12 and _relerr(b.Chh, a.Chh) < 1e-11
    assert np.array_equal(a.mu_T, b.mu_T)


def test_split_panel_agree_midsize(ctx):
    from ppls_amd import Theta
    p, q, r = 600, 500, 3
    rng = np.random.default_rng(1)
    W = np.linalg.qr(rng.standard_normal((p, r)))[0]
    C = np.linalg.qr(rng.standard_normal((q, r)))[0]
    truth = Theta(W, C, np.exp(np.log(1.5) - 0.3 * np.arange(r)), 0.5, 0.5, 0.1, np.exp(-0.1 * np.arange(r)))
    ctx.generate_synthetic(30000, p, q, truth, seed=20261015)
    th0 = _theta(dict(W=np.linalg.qr(rng.standard_normal((p, r)))[0], C=np.linalg.qr(rng.standard_normal((q, r)))[0],
                      B=np.eye(r), sigE=1.0, sigF=1.0, sigH=1.0, sigT=np.eye(r)))
    out = {}
    for sw in (0, 3):
        ctx.set_option("sweep", sw)
        out[sw] = ctx.em_run(th0, 6, -np.inf, 0)
    ctx.set_option("sweep", 0)
    (e1, l1, x1, _), (e3, l3, _, _) = out[0], out[3]
    assert _relerr(l3, l1) < 1e-12
    assert np.abs(e1.W - e3.W).max() < 1e-10
    assert np.all(np.diff(l1) > 0)
    # against the oracle on the same (copied back) data
    X, Y = ctx.get_data()
    ref = o.ppls_simult(X, Y, r, EMsteps=6, atol=-np.inf, theta0=th0.as_dict())
    assert _relerr(l1, ref["loglik"]) < 1e-10
    assert np.abs(e1.W - ref["estimates"]["W"]).max() < 1e-8
    assert np.abs(e1.C - ref["estimates"]["C"]).max() < 1e-8
    ctx.set_option("sweep", 0)


def test_synthetic_generator_properties(ctx):
    from ppls_amd import Context, Theta
    p, q, r, n = 40, 30, 2, 5000
    rng = np.random.default_rng(2)
    W = np.linalg.qr(rng.standard_normal((p, r)))[0]
    C = np.linalg.qr(rng.standard_normal((q, r)))[0]
    truth = Theta(W, C, [1.5, 1.1], 0.5, 0.5, 0.1, [1.0, 0.9])
    ctx.generate_synthetic(n, p, q, truth, seed=7)
    X, Y = ctx.get_data()
    ctx.generate_synthetic(n, p, q, truth, seed=7)
    X2, _ = ctx.get_data()
    assert np.array_equal(X, X2)                                  # deterministic
    # shard invariance: rows [1000, 3000) generated as a shard are bit-identical
    ctx.generate_synthetic(n, p, q, truth, seed=7, row0=1000, n_local=2000)
    Xs, Ys = ctx.get_data()
    assert np.array_equal(Xs, X[1000:3000]) and np.array_equal(Ys, Y[1000:3000])
    # model moments: Cov(X) = W diag(t^2) W' + sigE^2 I
    S = X.T @ X / n
    ref = W @ np.diag([1.0, 0.81]) @ W.T + 0.25 * np.eye(p)
    assert np.abs(S - ref).max() < 0.12
    ssx, ssy = ctx.ssq()
    assert abs(ssx - np.sum(Xs * Xs)) / ssx < 1e-12


def test_monotone_em_c2_shape(ctx):
    """Size-independent properties at BASELINE config C2 (n=1e5, p=q=1000, r=3)."""
    from ppls_amd import Theta
    p = q = 1000
    r, n = 3, 100_000
    rng = np.random.default_rng(3)
    W = np.linalg.qr(rng.standard_normal((p, r)))[0]
    C = np.linalg.qr(rng.standard_normal((q, r)))[0]
    truth = Theta(W, C, np.exp(np.log(1.5) - 0.3 * np.arange(r)), 0.5, 0.5, 0.1, np.exp(-0.1 * np.arange(r)))
    ctx.set_option("sweep", 0)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    th0 = _theta(dict(W=np.linalg.qr(rng.standard_normal((p, r)))[0], C=np.linalg.qr(rng.standard_normal((q, r)))[0],
                      B=np.eye(r), sigE=1.0, sigF=1.0, sigH=1.0, sigT=np.eye(r)))
    est, ll, eout, neg = ctx.em_run(th0, 40, -np.inf, 0, want_mu=False)
    assert len(ll) == 40 and not neg and np.all(np.diff(ll) > 0)
    assert np.abs(est.W.T @ est.W - np.eye(r)).max() < 1e-12
    assert np.abs(est.C.T @ est.C - np.eye(r)).max() < 1e-12
    # EM approaches the true subspace (canonicalisation may permute/flip components)
    assert np.linalg.svd(est.W.T @ W, compute_uv=False).min() > 0.95
    assert abs(est.sigE - 0.5) < 0.02


def test_rccl_single_rank_communicator_path():
    """ppls_comm_init + the per-iteration ncclAllReduce on a 1-rank communicator (the 8-GPU path
    is run by the driver; here the RCCL calls themselves are exercised on the one GPU)."""
    from ppls_amd import Context
    X, Y, th0 = make_problem(400, 30, 26, 3, seed=8)
    a = Context(0)
    a.set_data(X, Y)
    ra = a.em_run(_theta(th0), 5, -np.inf, 0)
    a.close()
    b = Context(0)
    b.comm_init(1, 0, Context.comm_unique_id())
    b.set_data(X, Y)
    rb = b.em_run(_theta(th0), 5, -np.inf, 0)
    b.close()
    assert np.array_equal(ra[1], rb[1]) and np.array_equal(ra[0].W, rb[0].W)


@pytest.mark.parametrize("n,p,q,r,steps,atol", [(400, 60, 40, 3, 400, 1e-3), (300, 90, 30, 10, 300, 1e-2),
                                                (500, 40, 30, 2, 5, 1e-12), (250, 30, 20, 4, 50, 1e6)])
def test_device_stop_rule_matches_oracle(ctx, n, p, q, r, steps, atol):
    """The device-side stop rule (EM_W_multi.R:792, evaluated in the finalize, later kernels exit):
    same number of steps, trace, estimates and Eout as the oracle's host loop, for long EMsteps
    (stops after a few iterations), an atol never reached, and an atol reached at once (i = 2)."""
    X, Y, th0 = make_problem(n, p, q, r, seed=n + r)
    ctx.set_data(X, Y)
    est, ll, eout, neg = ctx.em_run(_theta(th0), steps, atol, 0)
    ref = o.ppls_simult(X, Y, r, EMsteps=steps, atol=atol, theta0=th0)
    e = ref["estimates"]
    assert len(ll) == len(ref["loglik"]), (len(ll), len(ref["loglik"]))
    assert _relerr(ll, ref["loglik"]) < 1e-10
    assert np.abs(est.W - e["W"]).max() < 1e-8 and np.abs(est.C - e["C"]).max() < 1e-8
    assert _relerr(est.B, np.diag(e["B"])) < 1e-8
    assert _relerr(eout.mu_T, ref["Expectations"]["mu_T"]) < 1e-8
    assert _relerr(eout.Ctt, np.diag(ref["Expectations"]["Ctt"])) < 1e-8
    # a following run on the same context is unaffected by the previous run's stop flag
    est2, ll2, _, _ = ctx.em_run(_theta(th0), 3, -np.inf, 0)
    ref3 = o.ppls_simult(X, Y, r, EMsteps=3, atol=-np.inf, theta0=th0)
    assert len(ll2) == 3 and _relerr(ll2, ref3["loglik"]) < 1e-10


@pytest.mark.parametrize("n,p,q,r", [(500, 60, 40, 3), (400, 3000, 200, 5), (300, 2100, 90, 10)])
def test_polar1_fast_path_em_agrees(ctx, n, p, q, r):
    """EM with the finalize's Cholesky-QR1 fast path (default) equals EM with Cholesky-QR2 only
    (polar1 = 0) and the oracle; wide p exercises polar teams."""
    X, Y, th0 = make_problem(n, p, q, r, seed=7 * n + r)
    ctx.set_data(X, Y)
    res = {}
    try:
        for fast in (1, 0):
            ctx.set_option("polar1", fast)
            res[fast] = ctx.em_run(_theta(th0), 12, -np.inf, 0)
    finally:
        ctx.set_option("polar1", 1)
    ref = o.ppls_simult(X, Y, r, EMsteps=12, atol=-np.inf, theta0=th0)
    for fast in (1, 0):
        est, ll = res[fast][0], res[fast][1]
        assert _relerr(ll, ref["loglik"]) < 1e-10
        assert np.abs(est.W - ref["estimates"]["W"]).max() < 1e-8
    a, b = res[1][0], res[0][0]
    assert _relerr(res[1][1], res[0][1]) < 1e-13
    assert np.abs(a.W - b.W).max() < 1e-11 and np.abs(a.C - b.C).max() < 1e-11


@pytest.mark.parametrize("team_rows", [256, 1000])
def test_polar_team_sizes_agree(ctx, team_rows):
    """The finalize's polar teams (option team_rows: rows of X'mu per member; default 2048) give
    the single-block result: p = 3000 as 12 or 3 members vs one block, EM fits vs the oracle."""
    n, p, q, r = 400, 3000, 2500, 4
    X, Y, th0 = make_problem(n, p, q, r, seed=11 + team_rows)
    ctx.set_data(X, Y)
    res = {}
    try:
        for tr in (team_rows, 1 << 20):
            ctx.set_option("team_rows", tr)
            res[tr] = ctx.em_run(_theta(th0), 8, -np.inf, 0)
    finally:
        ctx.set_option("team_rows", 0)
    ref = o.ppls_simult(X, Y, r, EMsteps=8, atol=-np.inf, theta0=th0)
    a, b = res[team_rows], res[1 << 20]
    assert _relerr(a[1], ref["loglik"]) < 1e-10 and np.abs(a[0].W - ref["estimates"]["W"]).max() < 1e-8
    assert _relerr(a[1], b[1]) < 1e-13
    assert np.abs(a[0].W - b[0].W).max() < 1e-11 and np.abs(a[0].C - b[0].C).max() < 1e-11


def test_eout_is_expect_m_of_the_uncanonicalised_theta(ctx):
    """PPLS_simult's `Expectations` (EM_W_multi.R:802) are Expect_M at the loop's LAST theta, before
    the final sign/order canonicalisation (:794-799).  A fit whose components swap order and stops by
    the rule (atol) after ~110 iterations: eout must equal the oracle's Expectations, which differ
    from Expect_M at the canonicalised estimates."""
    X, Y, th = make_problem(300, 20, 16, 2, seed=16)
    th0 = dict(th, W=th["W"][:, ::-1].copy(), C=th["C"][:, ::-1].copy(), B=np.diag([0.6, 1.3]),
               sigT=np.diag([0.5, 1.2]))
    ref = o.ppls_simult(X, Y, 2, EMsteps=400, atol=1e-2, theta0=th0)
    E, est_ref = ref["Expectations"], ref["estimates"]
    E_canon = o.expect_m(X, Y, est_ref["W"], est_ref["C"], est_ref["B"], est_ref["sigE"], est_ref["sigF"],
                         est_ref["sigH"], est_ref["sigT"])
    assert 3 <= len(ref["loglik"]) < 400                                # the stop rule fired
    assert np.abs(E["mu_T"] - E_canon["mu_T"]).max() > 1.0              # canonicalisation reordered
    ctx.set_data(X, Y)
    est, ll, eout, _ = ctx.em_run(_theta(th0), 400, 1e-2, 0)
    assert len(ll) == len(ref["loglik"])
    assert np.abs(est.W - est_ref["W"]).max() < 1e-8
    assert _relerr(est.B, np.diag(est_ref["B"])) < 1e-8
    for k in ("mu_T", "mu_U", "Chh"):
        assert _relerr(getattr(eout, k), E[k]) < 1e-8, k
    for k in ("Ctt", "Cuu", "Cut"):
        assert _relerr(getattr(eout, k), np.diag(E[k])) < 1e-8, k
    cee, cff = float(np.ravel(E["Cee"])[0]), float(np.ravel(E["Cff"])[0])
    assert abs(eout.Cee - cee) / cee < 1e-8 and abs(eout.Cff - cff) / cff < 1e-8


def test_team_finalize_with_early_stop(ctx):
    """A finite atol on a wide-p fit whose polar factor runs as a team of small members
    (team_rows 256: p = 3000 -> 12 workgroups): the stop flag written by the finalize's scalar block
    must not strand a late team member (the entry check ignores the flag of the current launch),
    so the run ends without PPLS_E_HIP and matches the oracle."""
    X, Y, th0 = make_problem(400, 3000, 300, 3, seed=5)
    ctx.set_data(X, Y)
    ctx.set_option("team_rows", 256)
    try:
        est, ll, eout, _ = ctx.em_run(_theta(th0), 500, 1.0, 0)
    finally:
        ctx.set_option("team_rows", 0)
    ref = o.ppls_simult(X, Y, 3, EMsteps=500, atol=1.0, theta0=th0)
    assert 3 <= len(ll) < 500 and len(ll) == len(ref["loglik"])
    assert _relerr(ll, ref["loglik"]) < 1e-10
    assert np.abs(est.W - ref["estimates"]["W"]).max() < 1e-8


def test_split_sweep_balanced_partition():
    """The split sweep's calibrated row partition (option balance, default on from 2048 rows per
    workgroup): boundaries cover every row once, per-XCD-class weights stay within +-10 %, and the
    fit equals the even split's to rounding (the row sums are only regrouped).  C3's column shape
    (one 512-thread workgroup per CU) on 600,000 generated rows."""
    from ppls_amd import Context, Theta
    n, p, q, r = 600_000, 2000, 2000, 5
    rng = np.random.default_rng(0)
    W = np.linalg.qr(rng.standard_normal((p, r)))[0]
    C = np.linalg.qr(rng.standard_normal((q, r)))[0]
    truth = Theta(W, C, np.linspace(1.5, 0.8, r), 0.5, 0.5, 0.1, np.linspace(1.0, 0.7, r))
    th0 = Theta(np.linalg.qr(rng.standard_normal((p, r)))[0], np.linalg.qr(rng.standard_normal((q, r)))[0],
                np.ones(r), 1.0, 1.0, 1.0, np.ones(r))
    out = {}
    for bal in (1, 0):
        with Context(0) as c:
            c.set_option("balance", bal)
            c.generate_synthetic(n, p, q, truth, seed=7)
            est, ll, _, _ = c.em_run(th0, 4, -np.inf, 0, want_eout=False)
            out[bal] = (est, ll, c.sweep_balance(), c.sweep_info(r)["grid"])
    w, b = out[1][2]
    grid = out[1][3]
    assert b is not None and len(b) == grid + 1 and b[0] == 0 and b[-1] == n
    assert np.all(np.diff(b) >= 0) and np.all((w >= 0.9) & (w <= 1.1))
    rows = np.diff(b).astype(float)
    for x in range(8):   # rows per workgroup follow the weight of its class
        assert np.abs(rows[x::8].mean() / rows.mean() - w[x] / w[np.arange(grid) % 8].mean()) < 0.02
    assert out[0][2][1] is None   # balance 0: the even split
    assert _relerr(out[1][1], out[0][1]) < 1e-13
    assert np.abs(out[1][0].W - out[0][0].W).max() < 1e-12


@pytest.mark.parametrize("sweep", [dict(), dict(sweep=3)], ids=["auto", "panel"])
@pytest.mark.parametrize("n,p,q,r", [(200, 3, 3, 3), (40, 2, 9, 2), (25, 300, 150, 3), (1, 5, 4, 1),
                                     (2, 6, 5, 2), (500, 1, 1, 1), (64, 257, 3, 3)],
                         ids=["r_eq_p_eq_q", "p_eq_r", "n_lt_p", "one_row", "two_rows", "p_q_1", "ragged"])
def test_edge_shapes_vs_oracle(ctx, sweep, n, p, q, r):
    """Edge shapes the reference accepts (ncol >= nr_comp, EM_W_multi.R:245): square loadings
    (r = p = q), r = p < q, fewer rows than columns, one and two rows, p = q = 1, ragged widths;
    5 EM iterations through em_run against the oracle.  (One- and two-row fits are ill-posed and
    amplify rounding, hence their looser loading tolerance.)"""
    X, Y, th0 = make_problem(n, p, q, r, seed=n + p)
    _apply(ctx, sweep)
    ctx.set_data(X, Y)
    est, ll, eout, _ = ctx.em_run(_theta(th0), 5, -np.inf, 0)
    ref = o.ppls_simult(X, Y, r, EMsteps=5, atol=-np.inf, theta0=th0)
    tol = 1e-8 if n >= 25 else 1e-6
    assert _relerr(ll, ref["loglik"]) < 1e-10
    assert np.abs(est.W - ref["estimates"]["W"]).max() < tol
    assert np.abs(est.C - ref["estimates"]["C"]).max() < tol
    assert _relerr([est.sigE, est.sigF, est.sigH], [ref["estimates"][k] for k in ("sigE", "sigF", "sigH")]) < tol
    assert _relerr(eout.mu_T, ref["Expectations"]["mu_T"]) < tol


def test_option_values_are_validated(ctx):
    """ppls_set_option rejects out-of-range values and unknown keys with PPLS_E_ARG (include/ppls.h),
    and the context keeps its previous setting."""
    from ppls_amd import PplsError
    bad = dict(dots_rows=48, dots_pair=2, acc_chunks=-1, var_chol=3, polar1_kappa=256, vorth=0)
    for k, v in bad.items():
        with pytest.raises(PplsError):
            ctx.set_option(k, v)
    with pytest.raises(PplsError, match="unknown option"):
        ctx.set_option("no_such_option", 1)
    ctx.set_option("acc_chunks", 65535)   # the largest accepted value
    ctx.set_option("acc_chunks", 0)
