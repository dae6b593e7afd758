"""The device synthetic generator (ppls_generate_synthetic; simulC semantics, src/loglC.cpp:268-315,
generalised to r > 1) against its CPU restatement oracle/philox.py.

* the device Philox4x32-10 block function reproduces the published known-answer vectors and equals
  the CPU restatement bitwise on random counters and keys;
* generated X, Y (and the fp32-stored form) equal the CPU restatement on a shard in the middle of
  the row range, to a few ulp (the Box-Muller log/cos/sin round differently in the device and host
  math libraries; the uniforms themselves are exact).
"""
import numpy as np
import pytest

from oracle import philox as ph

pytestmark = pytest.mark.gpu

EPS = np.finfo(np.float64).eps


@pytest.fixture(scope="module")
def ctx():
    from ppls_amd import Context
    c = Context(0)
    yield c
    c.close()


def test_device_philox_known_answers(ctx):
    for c, k, r in ph.KAT:
        out = ctx.philox4x32_10(np.array(c, dtype=np.uint32), k[0] | (k[1] << 32))
        assert tuple(int(x) for x in out[0]) == r


def test_device_philox_equals_restatement(ctx):
    rng = np.random.default_rng(7)
    ctr = rng.integers(0, 2 ** 32, size=(4096, 4), dtype=np.uint64).astype(np.uint32)
    for key in (0, 20261015, 0xFFFFFFFFFFFFFFFF, int(rng.integers(0, 2 ** 63))):
        dev = ctx.philox4x32_10(ctr, key)
        assert np.array_equal(dev, ph.philox4x32_10(ctr, key & 0xFFFFFFFF, key >> 32))


def _truth(p, q, r, seed=11):
    from ppls_amd import Theta
    rng = np.random.default_rng(seed)
    W = np.linalg.qr(rng.standard_normal((p, r)))[0]
    C = np.linalg.qr(rng.standard_normal((q, r)))[0]
    k = np.arange(r)
    return Theta(W, C, np.exp(np.log(1.5) - 0.3 * k), 0.5, 0.4, 0.1, np.exp(-0.1 * k))


@pytest.mark.parametrize("dtype", [0, 1], ids=["f64", "f32_storage"])
@pytest.mark.parametrize("p,q,r", [(37, 23, 3), (130, 64, 1), (64, 200, 10)])
def test_generated_rows_equal_restatement(ctx, dtype, p, q, r):
    n_total, row0, nl, seed = 5000, 1234, 501, 20261015
    th = _truth(p, q, r)
    ctx.set_option("dtype", dtype)
    try:
        ctx.generate_synthetic(n_total, p, q, th, seed=seed, row0=row0, n_local=nl)
        X, Y = ctx.get_data()
    finally:
        ctx.set_option("dtype", 0)
    Xr, Yr, _, _ = ph.generate(row0, nl, p, q, th.W, th.C, th.B, th.sigT, th.sigE, th.sigF, th.sigH, seed)
    for D, R in ((X, Xr), (Y, Yr)):
        if dtype:   # stored as fp32: the restatement rounded to fp32, within one fp32 ulp
            R32 = R.astype(np.float32).astype(np.float64)
            assert np.all(np.abs(D - R32) <= np.spacing(np.abs(R32).astype(np.float32)).astype(np.float64))
        else:
            assert np.abs(D - R).max() <= 64 * EPS * max(1.0, np.abs(R).max())
    # shard invariance: the same rows generated as part of a larger shard are identical
    ctx.generate_synthetic(n_total, p, q, th, seed=seed, row0=row0 - 100, n_local=nl + 200)
    X2, Y2 = ctx.get_data(100, nl)
    if not dtype:
        assert np.array_equal(X2, X) and np.array_equal(Y2, Y)
