"""The cross-product form (option "xprod") at the sizes the auto policy selects it for, and its
ill-conditioned and sharded corners.

The auto policy (the R shim and the Python default context set it) reads S =
[X Y]'[X Y] instead of the rows for any fit past ~58 iterations at C3, so the statistics of
EM_W_multi.R:668-742 come from S in production.  Here:

* full C3 (n = 1e6, p = q = 2000, r = 5, fp64) and full C5 (n = 5e5, p = 1e4, q = 500, r = 10, fp32
  storage) -- cross-product fit against the streaming fit of the same data and theta0: log-likelihood
  1e-12 relative, loadings 1e-10, Expectations' mu rows 1e-10 (they only reorder sums);
* C4 (C3's data over 8 row shards, each rank forming S over its rows + ONE all-reduce of S): ranks
  bitwise identical, equal to the unsharded cross-product and streaming fits;
* the M-step's orth() on ill-conditioned X'mu_T (kappa 1e2 .. 1e13) computed from S;
* the Expectations tail needs no collective: only one rank asks for mu.
"""
import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu

EPS = np.finfo(np.float64).eps
SEED = 20261015


def _theta(th):
    from ppls_amd import Theta
    return Theta(th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])


def _relerr(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def _bench_model(p, q, r):
    """bench.py's truth and theta0."""
    import bench
    truth, th0 = bench.make_truth_and_theta0(p, q, r)
    return truth, th0


def _stream_vs_xprod(c, r, th0, steps, rows):
    c.set_option("xprod", 0)
    est_s, ll_s, eo_s, _ = c.em_run(th0, steps, -np.inf, 0)
    c.set_option("xprod", 1)
    est_x, ll_x, eo_x, _ = c.em_run(th0, steps, -np.inf, 0)
    assert c.xprod_info(r)["ready"]
    assert len(ll_x) == len(ll_s) == steps
    assert _relerr(ll_x, ll_s) < 1e-12
    assert np.abs(est_x.W - est_s.W).max() < 1e-10 and np.abs(est_x.C - est_s.C).max() < 1e-10
    assert _relerr(est_x.B, est_s.B) < 1e-10 and _relerr(est_x.sigT, est_s.sigT) < 1e-10
    assert _relerr([est_x.sigE, est_x.sigF, est_x.sigH], [est_s.sigE, est_s.sigF, est_s.sigH]) < 1e-10
    for f in ("mu_T", "mu_U"):   # Expectations (:802): this rank's rows, sampled
        a, b = getattr(eo_x, f), getattr(eo_s, f)
        assert a.shape == b.shape
        assert _relerr(a[rows], b[rows]) < 1e-10
    assert _relerr(eo_x.Ctt, eo_s.Ctt) < 1e-10 and _relerr(eo_x.Chh, eo_s.Chh) < 1e-10
    assert abs(eo_x.Cee - eo_s.Cee) / eo_s.Cee < 1e-10
    return est_x, ll_x


def test_xprod_full_c3():
    """C3 at full size: 32 GB resident, S = 128 MB, 4 EM iterations each way."""
    from ppls_amd import Context
    n, p, q, r = 1_000_000, 2000, 2000, 5
    truth, th0 = _bench_model(p, q, r)
    rows = np.random.default_rng(0).integers(0, n, 4096)
    with Context(0) as c:
        c.generate_synthetic(n, p, q, truth, seed=SEED)
        est, ll = _stream_vs_xprod(c, r, th0, 4, rows)
        assert np.all(np.diff(ll) > 0)
        assert np.abs(est.W.T @ est.W - np.eye(r)).max() < 1e-12


def test_xprod_full_c5():
    """C5 at full size: fp32 storage (21 GB), S = (10,240 + 512)^2 doubles = 925 MB, 3 iterations."""
    from ppls_amd import Context
    n, p, q, r = 500_000, 10_000, 500, 10
    truth, th0 = _bench_model(p, q, r)
    rows = np.random.default_rng(1).integers(0, n, 4096)
    with Context(0) as c:
        c.set_option("dtype", 1)
        c.generate_synthetic(n, p, q, truth, seed=SEED)
        assert c.sweep_info(r)["variant"] == "panel"
        est, ll = _stream_vs_xprod(c, r, th0, 3, rows)
        assert np.all(np.diff(ll) > 0)


def test_xprod_c4_eight_shards():
    """C4: C3's data over 8 row shards (8 contexts on GPU 0, the host reducer standing in for RCCL).
    Each rank forms S over its 125,000 rows, ONE all-reduce of S, then iterations without a
    collective: ranks bitwise identical, equal to the unsharded cross-product and streaming fits."""
    from ppls_amd import Context
    from test_gpu_multirank import _run_ranks
    k, n, p, q, r, steps = 8, 1_000_000, 2000, 2000, 5, 3
    truth, th0 = _bench_model(p, q, r)

    def fit(c, row0, n_local, xprod):
        c.set_option("xprod", xprod)
        c.generate_synthetic(n, p, q, truth, seed=SEED, row0=row0, n_local=n_local)
        est, ll, _, _ = c.em_run(th0, steps, -np.inf, 0, want_eout=False)
        return est, ll, c.xprod_info(r)["ready"], c.xprod_setup_times()

    with Context(0) as c:
        ref_s = fit(c, 0, n, 0)
        ref_x = fit(c, 0, n, 1)
    res = _run_ranks(k, lambda rank, c: fit(c, *Context.shard_range(n, k, rank), 1))
    for est, ll, ready, times in res:
        assert ready and times[1] > 0.0   # the all-reduce of S ran (and was timed)
        for a, b in ((est.W, res[0][0].W), (est.C, res[0][0].C), (est.B, res[0][0].B),
                     (est.sigT, res[0][0].sigT), (ll, res[0][1])):
            assert np.array_equal(a, b)
    est, ll = res[0][0], res[0][1]
    for ref in (ref_x, ref_s):
        assert _relerr(ll, ref[1]) < 1e-12
        assert np.abs(est.W - ref[0].W).max() < 1e-10 and np.abs(est.C - ref[0].C).max() < 1e-10
        assert _relerr(est.B, ref[0].B) < 1e-10


@pytest.mark.parametrize("kappa", [1e2, 1e6, 1e10, 1e13])
@pytest.mark.parametrize("typ", ["SVD", "QR"])
def test_xprod_orth_ill_conditioned(kappa, typ):
    """The M-step's orth(X'mu_T) (EM_W_multi.R:732, functions.R:252-260) with X'mu_T read off S and
    condition number kappa.  X = [I_p; 0] and Y on the complementary rows make X'X = I, X'Y = 0, so
    X'mu_T = W0 diag(alpha) exactly, with alpha_k ~ sigT_k^2 spread over kappa.  The first M-step's
    W1 from S must be orthonormal to 1e-13 and agree with numpy's polar / QR factor of the same
    matrix, and with the streaming sweep's W1, to 1e-13 + 64 eps kappa."""
    from ppls_amd import Context
    p, q, r = 300, 200, 5
    n = p + q + 7
    rng = np.random.default_rng(int(np.log10(kappa)) + (typ == "QR"))
    X = np.zeros((n, p))
    X[:p, :p] = np.eye(p)
    Y = np.zeros((n, q))
    Y[p:p + q, :q] = np.eye(q)
    W0 = np.linalg.qr(rng.standard_normal((p, r)))[0]
    C0 = np.linalg.qr(rng.standard_normal((q, r)))[0]
    t = np.geomspace(1.0, kappa ** -0.5, r)
    th0 = dict(W=W0, C=C0, B=np.eye(r), sigE=1.0, sigF=1.0, sigH=0.5, sigT=np.diag(t))
    cf = o.mu_coefficients(th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    SX = W0 * cf["alpha"]
    sv = np.linalg.svd(SX, compute_uv=False)
    assert 0.1 * kappa < sv[0] / sv[-1] < 10 * kappa
    tcode = 0 if typ == "SVD" else 1
    out = {}
    with Context(0) as c:
        c.set_data(X, Y)
        for xp in (0, 1):
            c.set_option("xprod", xp)
            c.em_begin(_theta(th0))
            c.em_iterate(1, tcode)
            out[xp], _ = c.em_state()   # theta_1, un-canonicalised (column k from component k)
    ref = o.orth(SX, typ)
    for W in (out[1].W, out[0].W):
        assert np.abs(W.T @ W - np.eye(r)).max() < 1e-13
        assert np.abs(W - ref).max() < 1e-13 + 64 * EPS * kappa
    assert np.abs(out[1].W - out[0].W).max() < 1e-13 + 64 * EPS * kappa


def test_xprod_eout_requested_by_one_rank():
    """ppls_em_run's Expectations tail on the cross-product path writes only the asking rank's mu
    rows (no collective): three sharded ranks, only rank 0 asks for mu -- the run must neither hang
    nor mis-sum, and rank 0's mu rows equal the unsharded fit's."""
    from ppls_amd import Context
    from test_gpu_multirank import _run_ranks
    k, n, p, q, r, steps = 3, 2001, 120, 90, 3, 6
    X, Y, th0 = make_problem(n, p, q, r, seed=41)

    def fit(c, Xs, Ys, n_total, want_mu):
        c.set_option("xprod", 1)
        c.set_data(Xs, Ys, n_total=n_total)
        return c.em_run(_theta(th0), steps, -np.inf, 0, want_eout=True, want_mu=want_mu)

    with Context(0) as c:
        ref = fit(c, X, Y, None, True)

    def work(rank, c):
        r0, nl = Context.shard_range(n, k, rank)
        return fit(c, X[r0:r0 + nl], Y[r0:r0 + nl], n, rank == 0)

    res = _run_ranks(k, work)
    for est, ll, eout, _ in res:
        assert np.array_equal(ll, res[0][1]) and np.array_equal(est.W, res[0][0].W)
        assert np.array_equal(eout.Ctt, res[0][2].Ctt)
    r0, nl = Context.shard_range(n, k, 0)
    assert _relerr(res[0][2].mu_T, ref[2].mu_T[r0:r0 + nl]) < 1e-11
    assert _relerr(res[0][2].mu_U, ref[2].mu_U[r0:r0 + nl]) < 1e-11
    assert _relerr(res[0][1], ref[1]) < 1e-11


def test_default_split_is_reproducible_across_contexts():
    """The split sweep's default row partition is the even split (option balance = 0), so two fresh
    contexts give bit-identical fits on a shape past the calibrated partition's threshold (>= 2048
    rows per workgroup: 600,000 rows on a 256-workgroup grid); balance = 1 changes only the last bits."""
    from ppls_amd import Context
    n, p, q, r = 600_000, 64, 48, 3
    truth, th0 = _bench_model(p, q, r)
    runs = []
    for bal in (0, 0, 1):
        with Context(0) as c:
            c.set_option("balance", bal)
            c.set_option("grid", 256)
            c.generate_synthetic(n, p, q, truth, seed=SEED)
            assert c.sweep_info(r)["variant"] == "split512"
            est, ll, _, _ = c.em_run(th0, 5, -np.inf, 0, want_eout=False)
            runs.append((est, ll, c.sweep_balance()[1]))
    assert runs[0][2] is None and runs[1][2] is None and runs[2][2] is not None
    assert np.array_equal(runs[0][1], runs[1][1]) and np.array_equal(runs[0][0].W, runs[1][0].W)
    assert _relerr(runs[2][1], runs[0][1]) < 1e-13
