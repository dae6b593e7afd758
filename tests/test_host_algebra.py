"""libppls_amd.so loads, exports every include/*.h symbol, and its host-compiled finalize
(the same ppls_math.h code the device finalize runs) reproduces the oracle's EM step (no GPU)."""
import ctypes as ct
import os
import re

import numpy as np
import pytest

from conftest import ROOT, make_problem
from oracle import ppls_oracle as o


@pytest.fixture(scope="module")
def L():
    from ppls_amd import _lib
    return _lib.lib()


def test_every_declared_symbol_is_exported(L):
    import glob
    hdr = "".join(open(h).read() for h in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))
    names = set(re.findall(r"\b(ppls_[a-zA-Z0-9_]+)\s*\(", hdr))
    assert len(names) >= 20
    for n in sorted(names):
        assert hasattr(L, n), n
    from ppls_amd._lib import SIGNATURES
    assert names == set(SIGNATURES), names ^ set(SIGNATURES)


def test_version_and_errors(L):
    assert L.ppls_version() >= 100
    assert L.ppls_strerror(-3) == b"numerical failure"


def test_shard_range_partitions():
    from ppls_amd import Context
    for n, k in [(10, 3), (1_000_000, 8), (5, 8), (0, 2)]:
        rows = [Context.shard_range(n, k, r) for r in range(k)]
        assert rows[0][0] == 0 and sum(nl for _, nl in rows) == n
        for (a, na), (b, _) in zip(rows, rows[1:]):
            assert a + na == b


def _finalize(th, st, X, Y, typ=0):
    from ppls_amd._lib import Expect, Theta, dptr, lib
    p, q, r = th.W.shape[0], th.C.shape[0], th.r
    nx = Theta.empty(p, q, r)
    e = Expect(r)
    ll = ct.c_double()
    SX, SY, G = (np.asfortranarray(st[k]) for k in ("SX", "SY", "G"))
    t, ns, es = th.struct(), nx.struct(), e.struct()
    rc = lib().ppls_finalize_host(dptr(SX), dptr(SY), dptr(G), float(np.sum(X * X)), float(np.sum(Y * Y)),
                                  float(X.shape[0]), p, q, r, ct.byref(t), typ, ct.byref(ns), ct.byref(es),
                                  ct.byref(ll))
    assert rc == 0
    nx.pull(ns)
    e.pull(es)
    return nx, e, ll.value


@pytest.mark.parametrize("r,typ", [(1, "SVD"), (2, "SVD"), (3, "QR"), (5, "SVD")])
def test_host_finalize_matches_oracle_em_step(r, typ):
    from ppls_amd._lib import Theta
    X, Y, th0 = make_problem(120, 17, 13, r, seed=40 + r)
    th = Theta(**th0)
    coef = o.mu_coefficients(th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    st = o.sweep_stats(X, Y, th0["W"], th0["C"], coef)
    nx, e, ll = _finalize(th, st, X, Y, 0 if typ == "SVD" else 1)
    ref_e = o.expect_m(X, Y, th0["W"], th0["C"], th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    ref_m = o.maximiz_m(ref_e, X, Y, typ)
    ref_ll = o.logl_w(X, Y, th0["W"], th0["C"], th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    assert abs(ll - ref_ll) / abs(ref_ll) < 1e-12
    assert np.allclose(e.Ctt, np.diag(ref_e["Ctt"]), rtol=1e-11)
    assert np.allclose(e.Cuu, np.diag(ref_e["Cuu"]), rtol=1e-11)
    assert np.allclose(e.Cut, np.diag(ref_e["Cut"]), rtol=1e-11)
    assert abs(e.Cee - ref_e["Cee"][0, 0]) / ref_e["Cee"][0, 0] < 1e-11
    assert abs(e.Cff - ref_e["Cff"][0, 0]) / ref_e["Cff"][0, 0] < 1e-11
    assert np.allclose(e.Chh, ref_e["Chh"], rtol=1e-10, atol=1e-14)
    assert np.allclose(nx.W, ref_m["W"], atol=1e-12)
    assert np.allclose(nx.C, ref_m["C"], atol=1e-12)
    assert np.allclose(nx.B, np.diag(ref_m["B"]), rtol=1e-11)
    assert np.allclose(nx.sigT, np.diag(ref_m["sigT"]), rtol=1e-11)
    assert abs(nx.sigE - ref_m["sigE"]) < 1e-12 and abs(nx.sigF - ref_m["sigF"]) < 1e-12
    assert abs(nx.sigH - ref_m["sigH"]) < 1e-12


def test_mu_coefficients_match_oracle(L):
    from ppls_amd._lib import Theta, dptr
    _, _, th0 = make_problem(10, 5, 4, 3, seed=9)
    th = Theta(**th0)
    out = np.zeros(12)
    t = th.struct()
    assert L.ppls_mu_coefficients(ct.byref(t), 3, dptr(out)) == 0
    ref = o.mu_coefficients(th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    assert np.allclose(out, np.concatenate([ref["alpha"], ref["beta"], ref["gamma"], ref["delta"]]), rtol=1e-14)


def test_context_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ppls_amd import Context, PplsError
    with pytest.raises(PplsError):
        Context(0)


def test_population_rows_per_shard():
    # population j = global rows [N_1+..+N_{j-1}, N_1+..+N_j) intersected with each rank's shard
    from ppls_amd.api import pop_rows
    sizes = [7, 0, 5, 9]
    for nranks in (1, 2, 3, 4):
        tot = np.zeros(4, dtype=np.int64)
        for rank in range(nranks):
            r0 = 21 * rank // nranks
            nl = 21 * (rank + 1) // nranks - r0
            loc, t = pop_rows(sizes, r0, nl)
            assert loc.sum() == nl and list(t) == sizes
            tot += loc
        assert list(tot) == sizes
    assert list(pop_rows([10, 10], 5, 10)[0]) == [5, 5]
