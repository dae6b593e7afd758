"""GPU parity of the multi-population fits meta_EMstep / meta_PPLSi (EM_W_multi.R:446-589,
meta_Estep / meta_Mstep src/loglC.cpp:399-474) against the oracle and the golden fixtures
tests/golden/meta_*.npz.

Tolerances (fp64): log-likelihoods 1e-10 relative; loadings 1e-8 absolute (unit vectors); per-
population B and sigmas 1e-8 relative; Cxt/Cyu 1e-9 relative; step counts exact.  Each population
is one r = 1 sweep over its row block, so agreement is to rounding, not bitwise.
"""
import json
import os

import numpy as np
import pytest

from conftest import make_problem
from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
META = sorted(f for f in os.listdir(GOLD) if f.startswith("meta_") and f.endswith(".npz"))


@pytest.fixture(scope="module")
def ctx():
    from ppls_amd import Context
    c = Context(0)
    yield c
    c.close()


def _relerr(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def _init(g):
    s = g["init_s"]
    return dict(W=g["init_W"], C=g["init_C"], B=s[0], sigE=s[1], sigF=s[2], sigH=s[3], sigT=s[4])


@pytest.mark.parametrize("name", META)
def test_meta_ppls_matches_golden(ctx, name):
    g = np.load(os.path.join(GOLD, name))
    meta = json.loads(str(g["meta"]))
    ctx.set_data(g["X"], g["Y"])
    W, C, P, lg = ctx.meta_ppls(meta["sizes"], meta["EMsteps"], meta["atol"], _init(g))
    assert lg.shape[0] - 1 == meta["steps"]
    assert _relerr(lg, g["logvalue"]) < 1e-10
    assert np.abs(W - g["W"]).max() < 1e-8 and np.abs(C - g["C"]).max() < 1e-8
    assert _relerr(P, g["params"]) < 1e-8


@pytest.mark.parametrize("name", META)
def test_meta_emstep_one_step_matches_golden(ctx, name):
    g = np.load(os.path.join(GOLD, name))
    meta = json.loads(str(g["meta"]))
    ctx.set_data(g["X"], g["Y"])
    s = g["init_s"]
    K = len(meta["sizes"])
    params = np.tile([s[0], s[1], s[2], s[3], s[4]], (K, 1))
    W, C, P, cxt, cyu = ctx.meta_emstep(g["init_W"], g["init_C"], meta["sizes"], params)
    assert np.abs(W - g["step1_W"]).max() < 1e-10 and np.abs(C - g["step1_C"]).max() < 1e-10
    assert _relerr(P, g["step1_params"]) < 1e-10
    assert _relerr(cxt, g["step1_Cxt"]) < 1e-9 and _relerr(cyu, g["step1_Cyu"]) < 1e-9


def test_meta_pplsi_api_levels_and_single_population(ctx):
    import ppls_amd
    X, Y, _ = make_problem(160, 13, 9, 1, seed=41)
    init = o.initial_guess(13, 9, "equal")
    # levels are sorted (as.factor) and only their counts matter (X[popui, ] by cumsum(table(.))):
    # labels "b" x 100 then "a" x 60 -> population "a" is rows 1..60
    Ipopu = np.array(["b"] * 100 + ["a"] * 60)
    f = ppls_amd.meta_PPLSi(X, Y, Ipopu, EMsteps=15, atol=-np.inf, customGuess=init, ctx=ctx)
    ref = o.meta_pplsi(X, Y, [60, 100], 15, -np.inf, init)
    assert _relerr(f["logvalue"], ref["logvalue"]) < 1e-10
    assert f["log"].shape == (15, 2)
    assert np.abs(f["W"] - ref["W"]).max() < 1e-8
    assert abs(f["params"][1]["sigT"] - ref["params"][1]["sigT"]) < 1e-8 * ref["params"][1]["sigT"]
    # one population == the device PPLSi (two independent reference code paths)
    m = ppls_amd.meta_PPLSi(X, Y, np.zeros(160), EMsteps=30, atol=1e-6, customGuess=init, ctx=ctx)
    a = ppls_amd.PPLSi(X, Y, EMsteps=30, atol=1e-6, customGuess=init, ctx=ctx)
    assert m["logvalue"].shape[0] - 1 == a["Number_steps"]
    assert _relerr(m["logvalue"][:, 0], a["logvalue"]) < 1e-12
    assert np.abs(m["W"] - a["W"]).max() < 1e-10


def test_meta_rejects_bad_populations(ctx):
    from ppls_amd import PplsError
    X, Y, _ = make_problem(50, 6, 5, 1, seed=42)
    ctx.set_data(X, Y)
    init = o.initial_guess(6, 5, "equal")
    with pytest.raises(PplsError):
        ctx.meta_ppls([30, 10], 5, 1e-4, init)       # sizes do not cover nrow(X)
    with pytest.raises(PplsError):
        ctx.meta_ppls([50, 0], 5, 1e-4, init)        # an empty level


@pytest.mark.parametrize("storage", ["f64", "f32", "wide"])
@pytest.mark.parametrize("sizes,atol", [([300, 250, 200, 250], 1e-6), ([997], -np.inf), ([3, 500, 2, 495], 1e-5),
                                        ([40] * 25, -np.inf)],
                         ids=["K4_stop", "K1", "tiny_pops", "K25"])
def test_meta_device_loop_equals_host_loop(ctx, sizes, atol, storage):
    """The device meta_PPLSi (the statistics of every population from one read of X, Y per EM step,
    the M-step, the log-likelihoods and the stop rule in one kernel; option meta_device = 1, the
    default) against the per-population host loop (meta_device = 0) and the oracle: the same steps,
    log-likelihoods to 1e-12, loadings and parameters to 1e-10 (the sums are regrouped).  storage:
    fp64 (the split sweep, one segmented launch), fp32 storage and fp64 wide p (the panel sweep, one
    launch per population) -- fp32 against the oracle on the fp32-rounded data."""
    n = int(sum(sizes))
    p, q = (4200, 29) if storage == "wide" else (37, 29)
    X, Y, _ = make_problem(n, p, q, 1, seed=n)
    if storage == "f32":
        X = X.astype(np.float32).astype(np.float64)
        Y = Y.astype(np.float32).astype(np.float64)
    init = o.initial_guess(p, q, "equal")
    ctx.set_option("dtype", 1 if storage == "f32" else 0)
    ctx.set_data(X, Y)
    res = {}
    for dev in (1, 0):
        ctx.set_option("meta_device", dev)
        res[dev] = ctx.meta_ppls(sizes, 40, atol, init)
        assert ctx.meta_info() == ("host" if not dev else "device_split" if storage == "f64" else "device_panel")
    ctx.set_option("meta_device", 1)
    ctx.set_option("dtype", 0)
    (W1, C1, P1, L1), (W0, C0, P0, L0) = res[1], res[0]
    assert L1.shape == L0.shape
    assert _relerr(L1, L0) < 1e-12
    assert np.abs(W1 - W0).max() < 1e-10 and np.abs(C1 - C0).max() < 1e-10
    assert _relerr(P1, P0) < 1e-10
    ref = o.meta_pplsi(X, Y, sizes, 40, atol, init)
    assert L1.shape[0] == ref["logvalue"].shape[0]
    assert _relerr(L1, ref["logvalue"]) < 1e-10
