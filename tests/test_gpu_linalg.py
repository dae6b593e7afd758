"""The hand-written batched inverse of SPD matrices (ppls_amd/csrc/ppls_linalg.hip: blocked Cholesky,
T = L^-1, T'T; the observed-information inverse of variances.PPLS_simult, EM_W_multi.R:852-856)
against numpy and rocSOLVER's potrf + potri.

Tolerance: backward-stable inverses differ by ~cond(A) eps: |inv - ref| <= 50 cond eps |ref|.
Non-positive-definite or non-finite input: info = the 1-based column of the first bad pivot (as
LAPACK's potrf), the other matrices of the batch unaffected.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from ppls_amd import Context
    c = Context(0)
    yield c
    c.close()


def _spd(rng, p, cond=1e3):
    Q = np.linalg.qr(rng.standard_normal((p, p)))[0]
    ev = np.geomspace(1.0, cond, p)
    rng.shuffle(ev)
    A = (Q * ev) @ Q.T
    return (A + A.T) / 2


def _check(inv, A, cond):
    ref = np.linalg.inv(A)
    err = np.abs(inv - ref).max() / np.abs(ref).max()
    assert err < 50 * cond * np.finfo(float).eps, err
    assert np.array_equal(inv, inv.T)


@pytest.mark.parametrize("p,a", [(1, 1), (5, 2), (63, 1), (64, 3), (65, 2), (130, 1), (257, 2), (700, 3)])
def test_spd_inverse_matches_numpy(ctx, p, a):
    rng = np.random.default_rng(p * 10 + a)
    A = np.stack([_spd(rng, p) for _ in range(a)])
    inv, info, _ = ctx.spd_inverse(A, 1)
    assert (info == 0).all()
    for z in range(a):
        _check(inv[z], A[z], 1e3)
    inv2, info2, _ = ctx.spd_inverse(A, 2)   # rocSOLVER potrf + potri
    assert (info2 == 0).all()
    assert np.abs(inv - inv2).max() / np.abs(inv2).max() < 1e-12


def test_spd_inverse_ill_conditioned(ctx):
    rng = np.random.default_rng(3)
    A = _spd(rng, 300, cond=1e9)
    inv, info, _ = ctx.spd_inverse(A, 1)
    assert info[0] == 0
    _check(inv, A, 1e9)


def test_spd_inverse_not_positive_definite(ctx):
    """A negative eigenvalue in matrix 1 of 3: its info names the first pivot that fails (the same
    column as rocSOLVER's potrf), matrices 0 and 2 are inverted as if alone."""
    rng = np.random.default_rng(4)
    p = 150
    A = np.stack([_spd(rng, p) for _ in range(3)])
    A[1, 100, 100] = -1e4   # the leading minor of order 101 is not positive definite
    inv, info, _ = ctx.spd_inverse(A, 1)
    _, info2, _ = ctx.spd_inverse(A, 2)
    assert info[0] == 0 and info[2] == 0 and info[1] > 0
    assert info[1] == info2[1]
    _check(inv[0], A[0], 1e3)
    _check(inv[2], A[2], 1e3)


def test_spd_inverse_non_finite(ctx):
    rng = np.random.default_rng(5)
    A = np.stack([_spd(rng, 90) for _ in range(2)])
    A[0, 70, 70] = np.nan
    A[1, 3, 2] = A[1, 2, 3] = np.inf
    _, info, _ = ctx.spd_inverse(A, 1)
    assert info[0] == 71 and info[1] > 0


def test_spd_inverse_timing_vs_rocsolver(ctx):
    """Five 2000 x 2000 matrices (variances at C3): record both device times.  The speed comparison
    itself lives in tools/bench_spd_inverse.py (profiles/r5_spd_inverse_bench.txt: 4.4x); here only a
    gross regression fails -- the hand-written path at more than twice rocSOLVER's time -- so clock
    or load noise cannot fail a correctness suite."""
    rng = np.random.default_rng(6)
    p, a = 2000, 5
    B = rng.standard_normal((p, p)) / np.sqrt(p)
    A0 = B @ B.T + np.eye(p)
    A = np.stack([A0 + 0.01 * z * np.eye(p) for z in range(a)])
    t1 = min(ctx.spd_inverse(A, 1)[2] for _ in range(3))
    t2 = min(ctx.spd_inverse(A, 2)[2] for _ in range(2))
    inv, info, _ = ctx.spd_inverse(A, 1)
    assert (info == 0).all()
    _check(inv[0], A[0], np.linalg.cond(A0))
    print(f"spd inverse {a} x {p}: hand-written {t1:.2f} ms, rocSOLVER {t2:.2f} ms")
    assert t1 < 2.0 * t2


def test_spd_inverse_random_sizes(ctx):
    """Random sizes and batch counts (partial last blocks of every width, batches of 1 to 6)."""
    rng = np.random.default_rng(8)
    for _ in range(12):
        p = int(rng.integers(1, 400))
        a = int(rng.integers(1, 7))
        A = np.stack([_spd(rng, p, cond=10.0 ** rng.uniform(0, 6)) for _ in range(a)])
        inv, info, _ = ctx.spd_inverse(A, 1)
        assert (info == 0).all(), (p, a, info)
        for z in range(a):
            _check(inv[z], A[z], np.linalg.cond(A[z]))
