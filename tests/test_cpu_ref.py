"""The C restatement oracle/cpu_ref.c (bench.py's CPU baseline) against the numpy oracle.

cpu_ref keeps the reference's pass structure (EM_W_multi.R:689-709, :732-733, loglC.cpp:318-338);
its per-thread partial sums are added in thread-index order, so a run is deterministic for a
fixed thread count.
"""
import numpy as np
import pytest

from conftest import make_problem
from oracle import cpu_ref
from oracle import ppls_oracle as o


@pytest.mark.parametrize("n,p,q,r", [(400, 37, 29, 3), (250, 60, 12, 5), (120, 9, 14, 1)])
def test_cpu_ref_matches_oracle(n, p, q, r):
    X, Y, th0 = make_problem(n, p, q, r, seed=n + r)
    steps = 6
    th, ll = cpu_ref.em_steps(X, Y, th0, steps, nthreads=3)
    ref = o.ppls_simult(X, Y, r, EMsteps=steps, atol=-np.inf, theta0=th0)
    assert np.abs(ll - ref["loglik"]).max() / np.abs(ref["loglik"]).max() < 1e-12
    W, C, B, T = o.canonicalize(th["W"], th["C"], th["B"], th["sigT"])
    assert np.abs(W - ref["estimates"]["W"]).max() < 1e-10
    assert np.abs(C - ref["estimates"]["C"]).max() < 1e-10
    assert abs(th["sigE"] - ref["estimates"]["sigE"]) < 1e-12


def test_cpu_ref_deterministic_per_thread_count():
    X, Y, th0 = make_problem(3000, 40, 30, 3, seed=9)
    a = cpu_ref.em_steps(X, Y, th0, 3, nthreads=4)
    b = cpu_ref.em_steps(X, Y, th0, 3, nthreads=4)
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[0]["W"], b[0]["W"])
    c = cpu_ref.em_steps(X, Y, th0, 3, nthreads=1)
    assert np.abs(c[1] - a[1]).max() / np.abs(a[1]).max() < 1e-13


@pytest.mark.parametrize("n,p,q,a", [(300, 24, 18, 3), (200, 40, 9, 2)])
def test_cpu_ref_whole_call_matches_oracle(n, p, q, a):
    """cpu_ref_ppls_simult -- the whole PPLS_simult(X, Y, a) call bench.py times on the host (the
    initialiser PPLS(X, Y, a, 20, 1e-4, 'random') from given draws, the EM loop with its stop rule,
    Eout) -- against the numpy oracle's PPLS (EM_W_multi.R:229-279) + PPLS_simult (:758-807)."""
    X, Y, _ = make_problem(n, p, q, a, seed=3 * n + a)
    rng = np.random.default_rng(a)
    inits = [o.initial_guess(p, q, "random", rng) for _ in range(a)]
    est, ll, cs, secs = cpu_ref.ppls_simult_call(X, Y, a, inits, nthreads=2)
    f0 = o.ppls(X, Y, a, 20, 1e-4, theta0s=inits)
    assert list(cs) == list(f0["Other_output"]["Number_steps"])
    ref = o.ppls_simult(X, Y, a, EMsteps=10, atol=1e-4, theta0=o.simult_theta0_from_ppls(f0))
    assert len(ll) == len(ref["loglik"])
    assert np.abs(ll - ref["loglik"]).max() / np.abs(ref["loglik"]).max() < 1e-11
    assert np.abs(est["W"] - ref["estimates"]["W"]).max() < 1e-8
    assert np.abs(est["C"] - ref["estimates"]["C"]).max() < 1e-8
    assert abs(est["sigE"] - ref["estimates"]["sigE"]) < 1e-9
    assert all(v >= 0 for v in secs.values())
