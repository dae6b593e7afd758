"""Non-finite and degenerate input: the reference's failure behaviour, collectively.

The reference stops on such data: R's svd() inside orth() refuses X'mu_T with NaN/Inf entries
(EM_W_multi.R:732-733), and `if (NA < atol)` errors when a log-likelihood increment is NA
(PPLS_simult :792, PPLSi :173, meta_PPLSi :575) -- which is what an all-zero X or Y produces.  The
library's contract (include/ppls.h):

* a NaN/Inf element in X or Y -> ppls_set_data / ppls_generate_synthetic return PPLS_E_ARG on every
  rank (detected from the all-reduced sums of squares, so a rank whose shard is clean fails too
  and none waits alone in a collective), the data are dropped;
* an all-zero X or Y -> every fit entry point returns PPLS_E_ARG;
* a NaN increment under a finite atol stops the run with PPLS_E_NUMERIC, and no run returns
  PPLS_OK with a non-finite trace entry or estimate.

Every case runs in a child process under a timeout, so a hang (a rank left in a collective) fails
the test instead of stalling the suite; the 3-rank cases use the host reducer (k contexts on GPU 0,
one thread per rank).  Also here: a long cross-product run with the finalize's carried Jacobi V
re-orthonormalised every 8th iteration (the default) against every iteration.
"""
import json
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
if HERE not in sys.path:
    sys.path.insert(0, HERE)

E_ARG, E_NUMERIC, E_STATE = -1, -3, -4


def _problem(n=600, p=40, q=30, r=3, seed=5):
    from conftest import make_problem
    return make_problem(n, p, q, r, seed=seed)


def _theta(th):
    from ppls_amd import Theta
    return Theta(th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])


def _err(fn):
    """(code, message) of the PplsError fn raises, or (0, '') when it returns."""
    from ppls_amd import PplsError
    try:
        fn()
    except PplsError as e:
        return e.code, str(e)
    return 0, ""


def _fits(ctx, th0, r):
    """Every fit entry point on the context's data: {name: (code, message)}."""
    out = {}
    out["em_run"] = _err(lambda: ctx.em_run(_theta(th0), 10, 1e-4, 0))
    out["em_run_noatol"] = _err(lambda: ctx.em_run(_theta(th0), 10, -np.inf, 0))
    out["em_begin"] = _err(lambda: ctx.em_begin(_theta(th0)))
    p, q = th0["W"].shape[0], th0["C"].shape[0]
    init = [dict(W=np.ones(p) / np.sqrt(p), C=np.ones(q) / np.sqrt(q), B=1.0, sigE=1.0 / p, sigF=1.0 / q,
                 sigH=1.0, sigT=1.0) for _ in range(r)]
    out["ppls"] = _err(lambda: ctx.ppls(r, 20, 1e-4, init))
    return out


# ------------------------------------------------------------------ cases (run in a child process)

def case_nan_x(mode):
    """A NaN in one X element: set_data fails (PPLS_E_ARG, names X); the context then has no data;
    valid data afterwards fit normally."""
    from ppls_amd import Context
    X, Y, th0 = _problem()
    Xb = X.copy()
    Xb[17, 3] = np.nan
    res = {}
    with Context(0) as ctx:
        ctx.set_option("xprod", 1 if mode == "xprod" else 0)
        res["set_data"] = _err(lambda: ctx.set_data(Xb, Y))
        res["after"] = _err(lambda: ctx.em_run(_theta(th0), 5, -np.inf, 0, want_eout=False))
        ctx.set_data(X, Y)
        est, ll, _, _ = ctx.em_run(_theta(th0), 5, -np.inf, 0)
        res["recovered"] = bool(np.all(np.isfinite(ll)) and len(ll) == 5)
    return res


def case_inf_y(mode):
    """+Inf (and -Inf) in Y: set_data fails naming Y; the fp32 storage path too."""
    from ppls_amd import Context
    X, Y, _ = _problem()
    Yb = Y.copy()
    Yb[5, 2] = np.inf
    Yb[9, 0] = -np.inf
    res = {}
    with Context(0) as ctx:
        ctx.set_option("xprod", 1 if mode == "xprod" else 0)
        res["set_data"] = _err(lambda: ctx.set_data(X, Yb))
        ctx.set_option("dtype", 1)
        res["set_data_f32"] = _err(lambda: ctx.set_data(X, Yb))
        # a finite fp64 value beyond the fp32 range becomes Inf in fp32 storage
        Xo = X.copy()
        Xo[0, 0] = 1e39
        res["set_data_f32_overflow"] = _err(lambda: ctx.set_data(Xo, Y))
    return res


def case_zero_y(mode):
    """An all-zero Y: the data load (it is valid data), every fit refuses it with PPLS_E_ARG, and
    the R-level PPLS_simult (default 'random' initialiser, tried three times) raises."""
    from ppls_amd import Context, PPLS_simult
    X, Y, th0 = _problem()
    Z = np.zeros_like(Y)
    res = {}
    with Context(0) as ctx:
        ctx.set_option("xprod", 1 if mode == "xprod" else 0)
        res["set_data"] = _err(lambda: ctx.set_data(X, Z))
        res.update(_fits(ctx, th0, 3))
        res["PPLS_simult"] = _err(lambda: PPLS_simult(None, None, 3, ctx=ctx, seed=1))
        # and an all-zero X
        ctx.set_data(np.zeros_like(X), Y)
        res["em_run_zero_x"] = _err(lambda: ctx.em_run(_theta(th0), 10, 1e-4, 0))
    return res


def case_nan_increment(mode):
    """Finite data, but a theta0 whose coefficients overflow (sigE = 1e-170: 1 / sigE^2 = Inf): the
    log-likelihood is not finite, and the run must fail with PPLS_E_NUMERIC -- with the stop rule
    (NaN increment, :792) and without it (atol = -Inf: the final check) -- never PPLS_OK."""
    from ppls_amd import Context
    X, Y, th0 = _problem()
    bad = dict(th0, sigE=1e-170)
    res = {}
    with Context(0) as ctx:
        ctx.set_option("xprod", 1 if mode == "xprod" else 0)
        ctx.set_data(X, Y)
        res["em_run"] = _err(lambda: ctx.em_run(_theta(bad), 10, 1e-4, 0))
        res["em_run_noatol"] = _err(lambda: ctx.em_run(_theta(bad), 10, -np.inf, 0))
        # the context stays usable
        est, ll, _, _ = ctx.em_run(_theta(th0), 5, -np.inf, 0)
        res["recovered"] = bool(np.all(np.isfinite(ll)))
    return res


class _ThreadAllReduce:
    """Sum over k host threads in rank order (every rank gets the bitwise-same result)."""

    def __init__(self, k):
        self.bar = threading.Barrier(k, timeout=30)
        self.bufs = [None] * k

    def fn(self, rank):
        def reduce(buf):
            self.bufs[rank] = buf.copy()
            self.bar.wait()
            tot = self.bufs[0].copy()
            for b in self.bufs[1:]:
                tot += b
            self.bar.wait()
            buf[:] = tot
        return reduce


def case_ranks3(what, mode="stream"):
    """3 ranks (host reducer, k contexts on GPU 0): `what` = nan (only rank 2's shard holds a NaN),
    zero (an all-zero Y on every shard), incr (a theta0 whose log-likelihood is not finite).
    Every rank must return the same error, and return."""
    from ppls_amd import Context
    X, Y, th0 = _problem(n=901)
    if what == "nan":
        X = X.copy()
        X[850, 7] = np.nan    # rows [600, 901) are rank 2's
    if what == "zero":
        Y = np.zeros_like(Y)
    k = 3
    red = _ThreadAllReduce(k)
    out = [None] * k

    def body(rank):
        res = {}
        try:
            with Context(0) as c:
                c.set_option("xprod", 1 if mode == "xprod" else 0)
                c.set_reducer(red.fn(rank))
                r0, nl = Context.shard_range(X.shape[0], k, rank)
                res["set_data"] = _err(lambda: c.set_data(X[r0:r0 + nl], Y[r0:r0 + nl], n_total=X.shape[0]))
                if what != "nan":
                    th = dict(th0, sigE=1e-170) if what == "incr" else th0
                    res["em_run"] = _err(lambda: c.em_run(_theta(th), 10, 1e-4, 0, want_eout=False))
                    res["em_run_noatol"] = _err(lambda: c.em_run(_theta(th), 10, -np.inf, 0, want_eout=False))
        except BaseException as e:   # noqa: BLE001
            res["exception"] = repr(e)
            red.bar.abort()
        out[rank] = res

    ths = [threading.Thread(target=body, args=(i,)) for i in range(k)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=60)
    return {"ranks": out, "alive": [t.is_alive() for t in ths]}


CASES = {
    "nan_x_stream": lambda: case_nan_x("stream"),
    "nan_x_xprod": lambda: case_nan_x("xprod"),
    "inf_y_stream": lambda: case_inf_y("stream"),
    "inf_y_xprod": lambda: case_inf_y("xprod"),
    "zero_y_stream": lambda: case_zero_y("stream"),
    "zero_y_xprod": lambda: case_zero_y("xprod"),
    "nan_incr_stream": lambda: case_nan_increment("stream"),
    "nan_incr_xprod": lambda: case_nan_increment("xprod"),
    "ranks3_nan": lambda: case_ranks3("nan"),
    "ranks3_zero": lambda: case_ranks3("zero"),
    "ranks3_incr_stream": lambda: case_ranks3("incr", "stream"),
    "ranks3_incr_xprod": lambda: case_ranks3("incr", "xprod"),
}


def _run_case(name, timeout=90):
    proc = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), name], capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)
    assert proc.returncode == 0, (proc.returncode, proc.stdout[-2000:], proc.stderr[-4000:])
    line = [ln for ln in proc.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


# ------------------------------------------------------------------------------- the tests

@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["stream", "xprod"])
def test_nan_in_x_refused(mode):
    res = _run_case(f"nan_x_{mode}")
    code, msg = res["set_data"]
    assert code == E_ARG and "X contains NaN or Inf" in msg and "EM_W_multi.R:732-733" in msg, res
    assert res["after"][0] == E_STATE, res    # the data were dropped: "no data"
    assert res["recovered"], res


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["stream", "xprod"])
def test_inf_in_y_refused(mode):
    res = _run_case(f"inf_y_{mode}")
    for k in ("set_data", "set_data_f32"):
        code, msg = res[k]
        assert code == E_ARG and "Y contains NaN or Inf" in msg, (k, res)
    code, msg = res["set_data_f32_overflow"]
    assert code == E_ARG and "X contains NaN or Inf" in msg, res


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["stream", "xprod"])
def test_all_zero_y_refused_by_every_fit(mode):
    res = _run_case(f"zero_y_{mode}")
    assert res["set_data"] == [0, ""], res
    for k in ("em_run", "em_run_noatol", "em_begin", "ppls"):
        code, msg = res[k]
        assert code == E_ARG and "Y is all zero" in msg, (k, res)
    assert res["PPLS_simult"][0] == E_ARG, res
    code, msg = res["em_run_zero_x"]
    assert code == E_ARG and "X is all zero" in msg, res


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["stream", "xprod"])
def test_non_finite_loglik_never_ok(mode):
    res = _run_case(f"nan_incr_{mode}")
    for k in ("em_run", "em_run_noatol"):
        assert res[k][0] == E_NUMERIC, (k, res)
    assert res["recovered"], res


@pytest.mark.gpu
def test_nan_on_one_rank_fails_every_rank():
    res = _run_case("ranks3_nan")
    assert res["alive"] == [False] * 3, res
    for rk in res["ranks"]:
        assert "exception" not in rk, res
        code, msg = rk["set_data"]
        assert code == E_ARG and "X contains NaN or Inf" in msg, res


@pytest.mark.gpu
def test_all_zero_y_fails_every_rank():
    res = _run_case("ranks3_zero")
    assert res["alive"] == [False] * 3, res
    for rk in res["ranks"]:
        assert "exception" not in rk and rk["set_data"] == [0, ""], res
        for k in ("em_run", "em_run_noatol"):
            assert rk[k][0] == E_ARG and "Y is all zero" in rk[k][1], res


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["stream", "xprod"])
def test_non_finite_loglik_fails_every_rank(mode):
    res = _run_case(f"ranks3_incr_{mode}")
    assert res["alive"] == [False] * 3, res
    for rk in res["ranks"]:
        assert "exception" not in rk, res
        for k in ("em_run", "em_run_noatol"):
            assert rk[k][0] == E_NUMERIC, (k, res)
    # the same message on every rank (the same all-reduced statistics)
    assert len({tuple(rk["em_run"]) for rk in res["ranks"]}) == 1, res


@pytest.mark.gpu
def test_long_xprod_run_carried_v_stays_orthonormal():
    """the finalize re-orthonormalises its carried Jacobi V only every 8th
    iteration.  400 iterations of the cross-product path on data with latent scales spread over
    three decades (X'mu_T ill-conditioned; the CholQR2 branch): W'W = I and C'C = I to 1e-12, and
    the iterates equal those of re-orthonormalising every iteration (vorth = 1)."""
    from conftest import make_problem
    from ppls_amd import Context
    rng = np.random.default_rng(11)
    n, p, q, r = 4000, 120, 90, 4
    X, Y, th0 = make_problem(n, p, q, r, seed=3, sigE=0.02, sigF=0.03)
    scale = np.array([30.0, 1.0, 0.1, 0.03])
    # rescale the latent directions: project on the generating loadings' span and stretch
    Wt = np.linalg.qr(rng.standard_normal((p, r)))[0]
    X = X + (rng.standard_normal((n, r)) * scale) @ Wt.T
    runs = {}
    with Context(0) as ctx:
        ctx.set_data(X, Y)
        ctx.set_option("xprod", 1)
        for vo in (8, 1):
            ctx.set_option("vorth", vo)
            est, ll, _, _ = ctx.em_run(_theta(th0), 400, -np.inf, 0, want_eout=False)
            runs[vo] = (est, ll)
            assert len(ll) == 400 and np.all(np.isfinite(ll))
            for M in (est.W, est.C):
                assert np.abs(M.T @ M - np.eye(r)).max() < 1e-12, vo
        st = ctx.xprod_info(r)
        assert st["ready"]
    # the same iterates to the parity bars (log-likelihood 1e-10 relative, loadings 1e-8): the fit is
    # still creeping after 400 iterations (slow modes amplify last-bit differences), measured 1e-11
    (e8, l8), (e1, l1) = runs[8], runs[1]
    dl = np.abs(l8 - l1).max() / np.abs(l1).max()
    dw = max(np.abs(e8.W - e1.W).max(), np.abs(e8.C - e1.C).max())
    print(f"vorth 8 vs 1 over 400 iterations: loglik {dl:.2e} rel, loadings {dw:.2e} abs")
    assert dl < 1e-10 and dw < 1e-8


if __name__ == "__main__":
    name = sys.argv[1]
    print("RESULT " + json.dumps(CASES[name]()), flush=True)
