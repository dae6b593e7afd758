"""GPU parity of the cross-product form of the EM iteration (option "xprod", ppls_xprod.hip).

With S = [X Y]'[X Y] formed once (MFMA Gram), an iteration's statistics X'mu_T, Y'mu_U and the
Gram of [Xw Yc] (EM_W_multi.R:689-712, :732-733; loglC.cpp:334-335) are read off S instead of the
rows.  The iterates are the reference's; only the order of the floating-point sums differs, so the
bars are the ones of tests/test_gpu_parity.py: log-likelihood 1e-10 relative, loadings 1e-8
absolute, variances 1e-8 relative, against the golden fixtures and against the streaming sweep.
"""
import json
import os

import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEFAULTS = dict(xprod=0, xprod_rw=0, xprod_fuse=1, polar1=1, dtype=0)


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
    for k, v in DEFAULTS.items():
        ctx.set_option(k, v)


def _theta(th):
    from ppls_amd import Theta
    return Theta(th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])


def _relerr(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def _golden():
    return sorted(f for f in os.listdir(GOLD) if f.endswith(".npz") and not f.startswith(("seq_", "meta_", "rcheck_")))


# (xprod_rw, xprod_fuse): rows of S per wave of the tile kernel (0 auto); the Gram formed by the
# finalize (fuse 1, default) or by its own kernel
KERNELS = [(0, 1), (0, 0), (1, 1), (2, 1), (4, 1), (8, 1)]


@pytest.mark.parametrize("rw,fuse", KERNELS, ids=[f"rw{w}f{f}" for w, f in KERNELS])
@pytest.mark.parametrize("name", _golden())
def test_xprod_em_run_matches_golden(ctx, name, rw, fuse):
    g = np.load(os.path.join(GOLD, name))
    meta = json.loads(str(g["meta"]))
    ctx.set_option("xprod", 1)
    ctx.set_option("xprod_rw", rw)
    ctx.set_option("xprod_fuse", fuse)
    ctx.set_data(g["X"], g["Y"])
    th0 = dict(W=g["W0"], C=g["C0"], B=np.diag(g["B0"]), sigE=g["sig0"][0], sigF=g["sig0"][1],
               sigH=g["sig0"][2], sigT=np.diag(g["T0"]))
    typ = 0 if meta["type"] == "SVD" else 1
    est, ll, eout, neg = ctx.em_run(_theta(th0), meta["EMsteps"], meta["atol"], typ)
    assert ctx.xprod_info(th0["W"].shape[1])["ready"]   # the run did read S
    assert len(ll) == meta["steps_done"]
    assert _relerr(ll, g["loglik"]) < 1e-10
    assert np.abs(est.W - g["W"]).max() < 1e-8
    assert np.abs(est.C - g["C"]).max() < 1e-8
    assert _relerr(est.B, g["B"]) < 1e-8
    assert _relerr(est.sigT, g["T"]) < 1e-8
    assert _relerr([est.sigE, est.sigF, est.sigH], g["sig"]) < 1e-8
    # Expectations (:802): mu from the streaming sweep of the final, un-canonicalised theta
    assert _relerr(eout.mu_T, g["mu_T"]) < 1e-8
    assert _relerr(eout.mu_U, g["mu_U"]) < 1e-8
    assert _relerr(eout.Ctt, g["Ctt"]) < 1e-8
    assert _relerr(eout.Cut, g["Cut"]) < 1e-8
    assert _relerr(eout.Chh, g["Chh"]) < 1e-8
    assert abs(eout.Cee - g["Cee"]) / g["Cee"] < 1e-8
    assert abs(eout.Cff - g["Cff"]) / g["Cff"] < 1e-8
    assert not neg


# odd widths (16-B seam between X and Y columns of S), r up to PPLS_RMAX, one-row data, wide p
@pytest.mark.parametrize("n,p,q,r", [(200, 50, 50, 2), (97, 33, 7, 1), (301, 64, 31, 5), (50, 9, 12, 8),
                                     (3, 5, 4, 2), (1, 6, 3, 1), (700, 1025, 3, 2), (400, 3, 1500, 3),
                                     (150, 17, 14, 10), (90, 24, 20, 16), (600, 2600, 9, 3)])
def test_xprod_equals_streaming(ctx, n, p, q, r):
    from ppls_amd import PplsError
    X, Y, th0 = make_problem(n, p, q, r, seed=7 * n + p + q + r)
    steps = 25
    ctx.set_data(X, Y)
    try:
        ref_est, ref_ll, ref_eout, _ = ctx.em_run(_theta(th0), steps, -np.inf, 0)
    except PplsError as e:   # a degenerate fit (one row): the cross-product path fails the same way
        ctx.set_option("xprod", 1)
        with pytest.raises(PplsError) as e2:
            ctx.em_run(_theta(th0), steps, -np.inf, 0)
        assert e2.value.code == e.code
        return
    ctx.set_option("xprod", 1)
    est, ll, eout, _ = ctx.em_run(_theta(th0), steps, -np.inf, 0)
    assert ctx.xprod_info(r)["ready"]
    assert len(ll) == len(ref_ll) == steps
    assert _relerr(ll, ref_ll) < 1e-10
    assert np.abs(est.W - ref_est.W).max() < 1e-8
    assert np.abs(est.C - ref_est.C).max() < 1e-8
    assert _relerr(est.B, ref_est.B) < 1e-8
    assert _relerr([est.sigE, est.sigF, est.sigH], [ref_est.sigE, ref_est.sigF, ref_est.sigH]) < 1e-8
    assert _relerr(eout.mu_T, ref_eout.mu_T) < 1e-9
    assert _relerr(eout.Chh, ref_eout.Chh) < 1e-9


@pytest.mark.parametrize("n,p,q,r", [(900, 300, 260, 5), (500, 1025, 131, 10), (400, 129, 127, 3), (300, 2, 700, 1),
                                     (600, 256, 256, 8)])
def test_xprod_rows_per_wave_agree(ctx, n, p, q, r):
    """The tile kernel's rows-per-wave forms (multi-tile shapes, tiles cut by the X/Y seam, r up
    to 10) give the same iterates: every form sums each row of M = S B in the same column order."""
    X, Y, th0 = make_problem(n, p, q, r, seed=p + q + r)
    ctx.set_option("xprod", 1)
    ctx.set_data(X, Y)
    out = {}
    for rw in (1, 2, 4) + ((8,) if r <= 8 else ()):
        ctx.set_option("xprod_rw", rw)
        assert ctx.xprod_info(r)["rows_per_wave"] == rw
        est, ll, _, _ = ctx.em_run(_theta(th0), 12, -np.inf, 0, want_eout=False)
        out[rw] = (est, ll)
    for rw in out:
        assert _relerr(out[rw][1], out[1][1]) < 1e-12
        assert np.abs(out[rw][0].W - out[1][0].W).max() < 1e-10
        assert np.abs(out[rw][0].C - out[1][0].C).max() < 1e-10


def test_xprod_matches_oracle_and_qr(ctx):
    X, Y, th0 = make_problem(500, 60, 45, 4, seed=11)
    ctx.set_option("xprod", 1)
    ctx.set_data(X, Y)
    for typ, tname in ((0, "SVD"), (1, "QR")):
        est, ll, _, _ = ctx.em_run(_theta(th0), 15, -np.inf, typ)
        ref = o.ppls_simult(X, Y, 4, EMsteps=15, atol=-np.inf, type=tname, theta0=th0)
        assert _relerr(ll, ref["loglik"]) < 1e-10
        assert np.abs(est.W - ref["estimates"]["W"]).max() < 1e-8
        assert np.abs(est.C - ref["estimates"]["C"]).max() < 1e-8


def test_xprod_stop_rule_and_em_iterate(ctx):
    """The device stop rule fires at the same iteration as on the streaming path, and the
    em_begin/em_iterate session (the bench's loop) reads S too."""
    X, Y, th0 = make_problem(800, 40, 30, 3, seed=5)
    ctx.set_data(X, Y)
    ref_est, ref_ll, _, _ = ctx.em_run(_theta(th0), 3000, 1e-2, 0)
    ctx.set_option("xprod", 1)
    est, ll, _, _ = ctx.em_run(_theta(th0), 3000, 1e-2, 0)
    assert len(ll) == len(ref_ll) < 3000
    assert _relerr(ll, ref_ll) < 1e-10
    assert np.abs(est.W - ref_est.W).max() < 1e-8
    ctx.em_begin(_theta(th0))
    ctx.em_iterate(12)
    th_i, ll_i = ctx.em_state()
    ctx.set_option("xprod", 0)
    ctx.em_begin(_theta(th0))
    ctx.em_iterate(12)
    th_s, ll_s = ctx.em_state()
    assert len(ll_i) == len(ll_s) == 11
    assert _relerr(ll_i, ll_s) < 1e-10
    assert np.abs(th_i.W - th_s.W).max() < 1e-8


def test_xprod_fp32_storage(ctx):
    """fp32 storage: S holds the exact fp64 products of the stored values, so the cross-product
    iterates equal the fp32 streaming sweep's (which computes in fp64 too) to rounding."""
    X, Y, th0 = make_problem(1500, 300, 40, 5, seed=3)
    ctx.set_option("dtype", 1)
    ctx.set_data(X, Y)
    ref_est, ref_ll, _, _ = ctx.em_run(_theta(th0), 20, -np.inf, 0)
    ctx.set_option("xprod", 1)
    est, ll, _, _ = ctx.em_run(_theta(th0), 20, -np.inf, 0)
    assert _relerr(ll, ref_ll) < 1e-10
    assert np.abs(est.W - ref_est.W).max() < 1e-8


def test_xprod_data_change_invalidates(ctx):
    X, Y, th0 = make_problem(300, 20, 15, 2, seed=1)
    X2, Y2, _ = make_problem(300, 20, 15, 2, seed=2)
    ctx.set_option("xprod", 1)
    ctx.set_data(X, Y)
    ctx.em_run(_theta(th0), 5, -np.inf, 0)
    assert ctx.xprod_info(2)["ready"]
    ctx.set_data(X2, Y2)
    assert not ctx.xprod_info(2)["ready"]
    est, ll, _, _ = ctx.em_run(_theta(th0), 5, -np.inf, 0)
    ref = o.ppls_simult(X2, Y2, 2, EMsteps=5, atol=-np.inf, theta0=th0)
    assert _relerr(ll, ref["loglik"]) < 1e-10


def test_xprod_auto_policy(ctx):
    """Auto (-1): a long run on tall data forms S; a short run on data with more columns than
    rows streams."""
    X, Y, th0 = make_problem(20000, 30, 20, 2, seed=9)
    ctx.set_option("xprod", -1)
    ctx.set_data(X, Y)
    ctx.em_run(_theta(th0), 200, -np.inf, 0)
    assert ctx.xprod_info(2)["ready"]
    X, Y, th0 = make_problem(64, 900, 700, 2, seed=9)
    ctx.set_data(X, Y)
    ctx.em_run(_theta(th0), 2, -np.inf, 0)
    assert not ctx.xprod_info(2)["ready"]


def test_xprod_prepare_and_info(ctx):
    from ppls_amd import PplsError
    X, Y, _ = make_problem(1000, 70, 33, 2, seed=4)
    ctx.set_data(X, Y)
    ms, tot = ctx.xprod_prepare()
    assert ms > 0 and tot >= ms
    g, ar, tot2 = ctx.xprod_setup_times()
    assert g == ms and ar == 0.0 and tot2 == tot   # one rank: no all-reduce of S
    info = ctx.xprod_info(2)
    P = 70 + 34   # ld of q = 33 fp64 columns: 34
    assert info["ready"] and info["bytes_per_pass"] == 8 * P * P
    assert ctx.xprod_prepare() == (0.0, 0.0)   # already formed
    ctx.xprod_release()
    assert not ctx.xprod_info(2)["ready"]
    ms2, _ = ctx.xprod_prepare()
    assert ms2 > 0 and ctx.xprod_info(2)["ready"]
    # the tile kernel timed alone (bench.py's xprod roofline) in the middle of a session leaves its
    # iterates as they were
    ctx.set_option("xprod", 1)
    th = _theta(make_problem(1000, 70, 33, 2, seed=4)[2])
    ctx.em_begin(th)
    ctx.em_iterate(3)
    assert ctx.xprod_tile_timing(20) > 0.0
    ctx.em_iterate(3)
    est_a, ll_a = ctx.em_state()
    ctx.em_begin(th)
    ctx.em_iterate(6)
    est_b, ll_b = ctx.em_state()
    assert len(ll_a) == 5 and np.array_equal(ll_a, ll_b) and np.array_equal(est_a.W, est_b.W)
    # xprod = 0 ends a session that reads S (no silent switch to streaming under it), and keeps an S
    # formed by xprod_prepare until xprod_release
    ctx.set_option("xprod", 0)
    with pytest.raises(PplsError, match="ppls_em_begin first"):
        ctx.em_iterate(1)
    assert ctx.xprod_info(2)["ready"]
    ctx.xprod_release()
    # an S the run formed itself goes back when xprod goes from non-zero to 0 -- not when 0 is restated
    ctx.set_option("xprod", 1)
    ctx.em_run(th, 3, -np.inf, 0)
    assert ctx.xprod_info(2)["ready"]
    ctx.set_option("xprod", 0)
    assert not ctx.xprod_info(2)["ready"]
    ctx.xprod_prepare()
    ctx.set_option("xprod", 0)
    assert ctx.xprod_info(2)["ready"]
    ctx.xprod_release()


@pytest.mark.parametrize("k,n,p,q,r,dtype", [(3, 3001, 300, 200, 4, 0), (4, 2000, 700, 90, 10, 1),
                                             (4, 3, 20, 12, 2, 0)],
                         ids=["k3", "fp32_k4_r10", "empty_shard"])
def test_xprod_k_contexts_sharded(k, n, p, q, r, dtype):
    """Row shards, each forming its own S, ONE host all-reduce of S, then no collective per
    iteration: every rank holds bit-identical estimates equal to the unsharded fit."""
    from ppls_amd import Context
    from test_gpu_multirank import _run_ranks
    X, Y, th0 = make_problem(n, p, q, r, seed=n + k)
    steps = 8

    def fit(c, Xs, Ys, n_total):
        c.set_option("dtype", dtype)
        c.set_option("xprod", 1)
        c.set_data(Xs, Ys, n_total=n_total)
        est, ll, eout, _ = c.em_run(_theta(th0), steps, -np.inf, 0)
        return est, ll, eout

    with Context(0) as c:
        ref = fit(c, X, Y, None)

    def work(rank, c):
        r0, nl = Context.shard_range(n, k, rank)
        return fit(c, X[r0:r0 + nl], Y[r0:r0 + nl], n)

    res = _run_ranks(k, work)
    for est, ll, eout in res:
        assert np.array_equal(est.W, res[0][0].W) and np.array_equal(est.C, res[0][0].C)
        assert np.array_equal(ll, res[0][1])
        assert np.array_equal(eout.Ctt, res[0][2].Ctt) and eout.Cee == res[0][2].Cee
    est, ll, eout = res[0]
    tol = 1e-11 if n >= 100 else 1e-9
    assert _relerr(ll, ref[1]) < tol
    assert np.abs(est.W - ref[0].W).max() < tol and np.abs(est.C - ref[0].C).max() < tol
    mu = np.vstack([e.mu_T.reshape(-1, r) for _, _, e in res])
    assert _relerr(mu, ref[2].mu_T) < tol


@pytest.mark.parametrize("rw", [1, 2, 4])
@pytest.mark.parametrize("n,p,q,r", [(200, 24, 18, 3), (300, 50, 50, 2), (400, 300, 131, 5), (350, 129, 258, 10),
                                     (150, 7, 5, 1)])
def test_xprod_stats_unit_parity(ctx, rw, n, p, q, r):
    """One statistics step from S against the host: X'mu_T, Y'mu_U (EM_W_multi.R:691-694,
    :732-733) and the Gram of [XW YC] for a given theta, every rows-per-wave form."""
    X, Y, th0 = make_problem(n, p, q, r, seed=3 * p + q + r)
    ctx.set_option("xprod_rw", rw)
    ctx.set_data(X, Y)
    th = _theta(th0)
    SX, SY, G = ctx.xprod_stats(th)
    cf = o.mu_coefficients(th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    a, b = X @ th0["W"], Y @ th0["C"]
    muT = a * cf["alpha"] + b * cf["beta"]
    muU = a * cf["gamma"] + b * cf["delta"]
    Z = np.hstack([a, b])
    assert _relerr(SX, X.T @ muT) < 1e-12
    assert _relerr(SY, Y.T @ muU) < 1e-12
    assert _relerr(G, Z.T @ Z) < 1e-12
    assert np.array_equal(G, G.T)


# the cross-product iteration through both entry points: em_run and an em_begin / em_iterate session
# in two calls, against each other and the streaming sweep (shapes with ragged ldx, r = 1 .. 10, fp32)
@pytest.mark.parametrize("n,p,q,r,dtype", [(900, 300, 260, 5, 0), (500, 1025, 131, 8, 0), (400, 129, 127, 3, 0),
                                           (300, 2, 700, 1, 0), (600, 256, 256, 8, 1), (2000, 33, 7, 2, 0),
                                           (700, 64, 31, 4, 1), (500, 700, 90, 10, 0), (300, 6200, 90, 9, 1)])
def test_xprod_session_equals_run_and_stream(ctx, n, p, q, r, dtype):
    X, Y, th0 = make_problem(n, p, q, r, seed=5 * n + p + r)
    ctx.set_option("dtype", dtype)
    ctx.set_data(X, Y)
    out = {}
    for xp in (0, 1):
        ctx.set_option("xprod", xp)
        out[xp] = ctx.em_run(_theta(th0), 30, -np.inf, 0)
        ctx.em_begin(_theta(th0))
        ctx.em_iterate(7)
        ctx.em_iterate(5)
        out[xp] = out[xp] + ctx.em_state()
    (e0, l0, x0, _, t0, s0), (e1, l1, x1, _, t1, s1) = out[0], out[1]
    assert len(l0) == len(l1) == 30
    assert _relerr(l1, l0) < 1e-12
    assert np.abs(e1.W - e0.W).max() < 1e-10 and np.abs(e1.C - e0.C).max() < 1e-10
    assert _relerr(e1.B, e0.B) < 1e-10 and _relerr(e1.sigT, e0.sigT) < 1e-10
    assert _relerr([e1.sigE, e1.sigF, e1.sigH], [e0.sigE, e0.sigF, e0.sigH]) < 1e-10
    assert _relerr(x1.mu_T, x0.mu_T) < 1e-10 and _relerr(x1.Chh, x0.Chh) < 1e-10
    assert len(s0) == len(s1) == 11 and _relerr(s1, s0) < 1e-12
    assert np.array_equal(s1, l1[:11])   # the session's trace is the run's first 11 entries
    assert np.abs(t1.W - t0.W).max() < 1e-10


def test_xprod_stop_rule_both_polar_paths(ctx):
    """The device stop rule on the cross-product path, with Cholesky-QR1 allowed (polar1 = 1) and
    refused (every finalize takes Cholesky-QR2): it fires at the same iteration as the oracle's."""
    X, Y, th0 = make_problem(800, 40, 30, 3, seed=5)
    ctx.set_option("xprod", 1)
    ctx.set_data(X, Y)
    res = {}
    for polar1 in (1, 0):
        ctx.set_option("polar1", polar1)
        res[polar1] = ctx.em_run(_theta(th0), 3000, 1e-2, 0)
    ref = o.ppls_simult(X, Y, 3, EMsteps=3000, atol=1e-2, theta0=th0)
    for key, (est, ll, _, _) in res.items():
        assert len(ll) == len(ref["loglik"]) < 3000, key
        assert _relerr(ll, ref["loglik"]) < 1e-10, key
        assert np.abs(est.W - ref["estimates"]["W"]).max() < 1e-8, key
