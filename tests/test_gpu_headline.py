"""GPU parity at the benchmark shapes: the kernel instantiations behind BENCH's numbers.

* C3 (the headline, BASELINE configs[2]: n = 1e6, p = q = 2000, r = 5, fp64) runs the split sweep
  ``split<5,4,512,2,false,4,4>``.  At n = 20,000 rows of the same synthetic model the full fit is
  checked against the CPU oracle (EM_W_multi.R:758-807 restated in oracle/ppls_oracle.py) with the
  loads both non-temporal (what n = 1e6 uses) and default-policy.  At the full n = 1e6 the
  size-independent properties are checked: monotone log-likelihood, W'W = I, per-row E-step
  (mu_T, mu_U of sampled rows) against the oracle at the same theta, log-likelihood of the
  estimates equal to the trace's last entry.
* C5 (n = 5e5, p = 1e4, q = 500, r = 10, fp32 storage / fp64 arithmetic) runs the panel sweep.
  At n = 5,000 the fit equals the fp64 oracle on the fp32-rounded data; at the full n = 5e5 the
  same properties as for C3.

Tolerances (fp64 arithmetic, BASELINE.json): log-likelihood 1e-10 relative; W, C 1e-8 absolute on
unit-norm columns; B, sigT, sigmas 1e-8 relative; per-row mu 1e-11 relative; W'W = I to 1e-12.
"""
import numpy as np
import pytest

from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu

SEED = 20261015


def _polar(M):
    U, _, Vt = np.linalg.svd(M, full_matrices=False)
    return U @ Vt


def _truth_theta0(p, q, r):
    """bench.py's synthetic model: truth seeds 1/2, theta0 seeds 3/4."""
    from ppls_amd import Theta
    k = np.arange(r)
    truth = Theta(_polar(np.random.default_rng(1).standard_normal((p, r))),
                  _polar(np.random.default_rng(2).standard_normal((q, r))),
                  np.exp(np.log(1.5) - 0.3 * k), 0.5, 0.5, 0.1, np.exp(-0.1 * k))
    th0 = Theta(_polar(np.random.default_rng(3).standard_normal((p, r))),
                _polar(np.random.default_rng(4).standard_normal((q, r))), np.ones(r), 1.0, 1.0, 1.0, np.ones(r))
    return truth, th0


def _relerr(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


@pytest.fixture(scope="module")
def ctx():
    from ppls_amd import Context
    c = Context(0)
    yield c
    c.close()


def _check_vs_oracle(est, ll, X, Y, r, steps, th0):
    ref = o.ppls_simult(X, Y, r, EMsteps=steps, atol=-np.inf, theta0=th0.as_dict())
    e = ref["estimates"]
    assert _relerr(ll, ref["loglik"]) < 1e-10
    assert np.abs(est.W - e["W"]).max() < 1e-8
    assert np.abs(est.C - e["C"]).max() < 1e-8
    assert _relerr(est.B, np.diag(e["B"])) < 1e-8
    assert _relerr(est.sigT, np.diag(e["sigT"])) < 1e-8
    assert _relerr([est.sigE, est.sigF, est.sigH], [e["sigE"], e["sigF"], e["sigH"]]) < 1e-8


@pytest.mark.parametrize("nt", [1, 0], ids=["nt", "default_policy"])
def test_c3_kernel_parity_vs_oracle(ctx, nt):
    """The C3 split instantiation on n = 20,000 rows of the C3 model, 4 EM steps vs the oracle."""
    n, p, q, r, steps = 20_000, 2000, 2000, 5, 4
    truth, th0 = _truth_theta0(p, q, r)
    ctx.set_option("dtype", 0)
    ctx.set_option("nt", nt)
    try:
        ctx.generate_synthetic(n, p, q, truth, seed=SEED)
        assert ctx.sweep_info(r)["variant"] == "split512"
        kern = ctx.sweep_kernel(r)
        assert kern.startswith("split<5,4,512,2,false,4,4>"), kern
        assert kern.endswith(" nt") == bool(nt), kern
        est, ll, _, neg = ctx.em_run(th0, steps, -np.inf, 0, want_eout=False)
        X, Y = ctx.get_data()
    finally:
        ctx.set_option("nt", -1)
    assert not neg and np.all(np.diff(ll) > 0)
    _check_vs_oracle(est, ll, X, Y, r, steps, th0)


def _sample_rows_check(ctx, est, n, r, rows=2000):
    """Per-row E-step (mu_T, mu_U; EM_W_multi.R:691-694) of sampled rows vs the oracle at theta."""
    e = ctx.estep(est, want_mu=True)
    th = est.as_dict()
    for r0 in (0, n // 2, n - rows):
        Xs, Ys = ctx.get_data(r0, rows)
        cf = o.mu_coefficients(th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])
        a, b = Xs @ th["W"], Ys @ th["C"]
        mu_T = a * cf["alpha"] + b * cf["beta"]
        mu_U = a * cf["gamma"] + b * cf["delta"]
        assert _relerr(e.mu_T[r0:r0 + rows], mu_T) < 1e-11
        assert _relerr(e.mu_U[r0:r0 + rows], mu_U) < 1e-11
    return e


def test_c3_full_size_properties(ctx):
    """C3 at full size (n = 1e6, 32 GB fp64 resident): 5 EM iterations through the production path."""
    n, p, q, r, steps = 1_000_000, 2000, 2000, 5, 5
    truth, th0 = _truth_theta0(p, q, r)
    ctx.set_option("dtype", 0)
    ctx.generate_synthetic(n, p, q, truth, seed=SEED)
    assert ctx.sweep_kernel(r) == "split<5,4,512,2,false,4,4> nt"
    est, ll, _, neg = ctx.em_run(th0, steps, -np.inf, 0, want_eout=False)
    assert len(ll) == steps and not neg and np.all(np.diff(ll) > 0)
    assert np.abs(est.W.T @ est.W - np.eye(r)).max() < 1e-12
    assert np.abs(est.C.T @ est.C - np.eye(r)).max() < 1e-12
    # the log-likelihood of the (canonicalised) estimates is the trace's last entry (:791)
    assert abs(ctx.loglik(est) - ll[-1]) / abs(ll[-1]) < 1e-12
    _sample_rows_check(ctx, est, n, r)


@pytest.mark.parametrize("rows64", [0, 1], ids=["dots32", "dots64"])
def test_c5_kernel_parity_vs_oracle(ctx, rows64):
    """The C5 panel sweep (fp32 storage) on n = 5,000 rows of the C5 model vs the fp64 oracle on the
    fp32-rounded data (the data as stored); dots64 = the 64-rows-per-wave dots kernel the full-size
    C5 run uses (option dots_rows selects it below 32768 rows)."""
    n, p, q, r, steps = 5_000, 10_000, 500, 10, 3
    truth, th0 = _truth_theta0(p, q, r)
    ctx.set_option("dtype", 1)
    ctx.set_option("dots_rows", 64 if rows64 else 0)
    try:
        ctx.generate_synthetic(n, p, q, truth, seed=SEED)
        assert ctx.sweep_info(r)["variant"] == "panel"
        assert ctx.sweep_kernel(r).startswith("panel<float,10>")
        est, ll, _, neg = ctx.em_run(th0, steps, -np.inf, 0, want_eout=False)
        X, Y = ctx.get_data()
    finally:
        ctx.set_option("dtype", 0)
        ctx.set_option("dots_rows", 0)
    assert np.array_equal(X.astype(np.float32).astype(np.float64), X)   # widened fp32 values
    assert not neg and np.all(np.diff(ll) > 0)
    _check_vs_oracle(est, ll, X, Y, r, steps, th0)


def test_c5_full_size_properties(ctx):
    """C5 at full size (n = 5e5, p = 1e4, q = 500, r = 10; 21 GB fp32 resident), 4 EM iterations."""
    n, p, q, r, steps = 500_000, 10_000, 500, 10, 4
    truth, th0 = _truth_theta0(p, q, r)
    ctx.set_option("dtype", 1)
    try:
        ctx.generate_synthetic(n, p, q, truth, seed=SEED)
        est, ll, _, neg = ctx.em_run(th0, steps, -np.inf, 0, want_eout=False)
        assert len(ll) == steps and not neg and np.all(np.diff(ll) > 0)
        assert np.abs(est.W.T @ est.W - np.eye(r)).max() < 1e-12
        assert np.abs(est.C.T @ est.C - np.eye(r)).max() < 1e-12
        assert abs(ctx.loglik(est) - ll[-1]) / abs(ll[-1]) < 1e-12
        _sample_rows_check(ctx, est, n, r, rows=500)
    finally:
        ctx.set_option("dtype", 0)
        ctx.set_data(np.zeros((1, 2)), np.zeros((1, 2)))   # release the 21 GB
