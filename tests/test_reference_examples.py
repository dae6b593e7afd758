"""Parity against the outputs the reference itself printed.

The reference's R CMD check run (Package/PPLS.Rcheck/PPLS-Ex.R:39-53) fits PPLS() four times on
`exX = scale(matrix(rnorm(100*10),100,10))`, `exY = scale(matrix(rnorm(100*12),100,12))` drawn
after `set.seed(1)`, and prints print.PPLS tables (PPLS-Ex_x64.Rout:54-83; x64 and i386 agree).
The snapshot's PPLS/PPLSi/EMstep_W R code equals today's (Package/PPLS/R/EM_W_multi.R:51-279),
and its loglC_fast differs only by the 2*pi constant, which cancels in log LR.

The inputs and the 'random' starting values are regenerated with R's default stream
(oracle/r_rng.py; fixture tests/golden/rcheck_ppls_ex.npz, tests/golden/make_rcheck.py).
Asserted: every printed `#steps` exactly, and every printed ratio / log LR to the printed 3
digits -- for the oracle (CPU) and for the device path (`ppls_ppls_ex`, -m gpu).
"""
import os

import numpy as np
import pytest

from oracle import ppls_oracle as o
from oracle.r_rng import ppls_example_data

G = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rcheck_ppls_ex.npz"))
P, Q = 10, 12


def _random_inits():
    return [dict(W=G["random_W"][:, k] / np.linalg.norm(G["random_W"][:, k]),
                 C=G["random_C"][:, k] / np.linalg.norm(G["random_C"][:, k]),
                 B=G["random_s"][k, 0], sigE=G["random_s"][k, 1], sigF=G["random_s"][k, 2],
                 sigH=G["random_s"][k, 3], sigT=G["random_s"][k, 4]) for k in range(3)]


def _custom():
    w, c = np.arange(1, 11.0), np.arange(1, 13.0)          # orth(1:10), orth(1:12)
    return dict(W=w / np.linalg.norm(w), C=c / np.linalg.norm(c), B=0.1, sigE=1.0, sigF=1.0,
                sigH=1.0, sigT=0.1)


EXAMPLES = {
    # name: (nr_comp, starting values, constraints, printed table)
    "equal": (3, lambda: [o.initial_guess(P, Q, "equal")] * 3, None, "table_equal"),
    "random": (3, _random_inits, None, "table_random"),
    "custom": (1, lambda: [_custom()], None, "table_custom"),
    "constrained": (2, lambda: [o.initial_guess(P, Q, "equal")] * 2,
                    [o.fconstraint(dict(B=1.0)), o.fconstraint(dict(sigT=1.0))], "table_constrained"),
}


def _assert_table(got, want):
    got, want = np.asarray(got), np.asarray(want)
    assert got.shape == want.shape
    assert np.array_equal(got[:, 5], want[:, 5]), f"#steps {got[:, 5]} != printed {want[:, 5]}"
    assert np.abs(got[:, :5] - want[:, :5]).max() < 1e-9, f"\n{got}\n!=\n{want}"
    assert np.abs(got[:, 6]).max() < 5e-4                   # printed "last incr" 0


def test_fixture_regenerates_from_r_stream():
    exX, exY, rng = ppls_example_data()
    assert np.array_equal(exX, G["exX"]) and np.array_equal(exY, G["exY"])
    for k in range(3):      # PPLSi's draws per component, EM_W_multi.R:133
        assert np.array_equal(rng.runif(P), G["random_W"][:, k])
        assert np.array_equal(rng.runif(Q), G["random_C"][:, k])
        b = rng.rchisq(1, 1)[0]
        siglat = rng.rchisq(2, 100) / 100
        sig = rng.rchisq(2, 10) / 100
        assert np.array_equal([b, sig[0], sig[1], siglat[0], siglat[1]], G["random_s"][k])


@pytest.mark.parametrize("name", list(EXAMPLES))
def test_oracle_reproduces_printed_example(name):
    a, inits, cons, table = EXAMPLES[name]
    fit = o.ppls(G["exX"], G["exY"], a, 10000, 1e-4, theta0s=inits(), constraints=cons)
    _assert_table(o.print_ppls(fit), G[table])


@pytest.mark.gpu
@pytest.mark.parametrize("xprod", [0, 1], ids=["stream", "xprod"])
@pytest.mark.parametrize("name", list(EXAMPLES))
def test_device_reproduces_printed_example(name, xprod):
    """Both statistics paths: one streaming sweep per EM step, or the cross-products S (the printed
    step counts are exact integers, so the reordered sums must not move a single stop decision)."""
    from ppls_amd import PPLS, Context, print_PPLS
    a, inits, cons, table = EXAMPLES[name]
    with Context(0) as ctx:
        ctx.set_option("xprod", xprod)
        if name == "random":
            # the R stream itself drives the API's 'random' initial guess
            exX, exY, rng = ppls_example_data()
            fit = PPLS(exX, exY, a, 10000, 1e-4, "random", rng=rng, ctx=ctx)
        elif name == "custom":
            fit = PPLS(G["exX"], G["exY"], a, 10000, 1e-4, "custom", customGuess=_custom(), ctx=ctx)
        else:
            fit = PPLS(G["exX"], G["exY"], a, 10000, 1e-4, "equal", constraints=cons, ctx=ctx)
    rows, _ = print_PPLS(fit)
    _assert_table(rows, G[table])
    ref = o.ppls(G["exX"], G["exY"], a, 10000, 1e-4, theta0s=inits(), constraints=cons)
    assert np.abs(np.abs(fit["W"]) - np.abs(ref["W"])).max() < 1e-8
    assert np.abs(fit["sig"] - ref["sig"]).max() / np.abs(ref["sig"]).max() < 1e-8


@pytest.mark.gpu
@pytest.mark.parametrize("xprod", [0, 1], ids=["stream", "xprod"])
def test_device_ppls_simult_default_init_from_r_stream(xprod):
    """PPLS_simult(exX, exY, a) with its default init PPLS(X, Y, a, 20, 1e-4, 'random') drawn from
    R's stream after set.seed(1) + the data draws (EM_W_multi.R:762-806) vs the oracle."""
    from ppls_amd import PPLS_simult, Context
    exX, exY, rng = ppls_example_data()
    exX2, exY2, rng2 = ppls_example_data()
    with Context(0) as ctx:
        ctx.set_option("xprod", xprod)
        out = PPLS_simult(exX, exY, 2, EMsteps=50, atol=1e-4, ctx=ctx, rng=rng)
    f0 = o.ppls(exX2, exY2, 2, 20, 1e-4, theta0s=[o.initial_guess(P, Q, "random", rng2) for _ in range(2)])
    ref = o.ppls_simult(exX2, exY2, 2, EMsteps=50, atol=1e-4, theta0=o.simult_theta0_from_ppls(f0))
    assert len(out["loglik"]) == len(ref["loglik"])
    assert np.abs(out["loglik"] - ref["loglik"]).max() / np.abs(ref["loglik"]).max() < 1e-10
    est, rest = out["estimates"], ref["estimates"]
    assert np.abs(est["W"] - rest["W"]).max() < 1e-8
    assert np.abs(est["C"] - rest["C"]).max() < 1e-8
