"""The int8-MFMA Gram of the cross-products in its Chinese-remainder form (ppls_ozaki.hip; VERDICT r5
item 3): S = [X Y]'[X Y] (the sums EM_W_multi.R:689-690, 732-733 read off it, and variances' X'X
:846) from v_mfma_i32_32x32x32_i8 SYRKs of residue planes.

Checked against EXACT sums: every sampled entry's reference is the correctly rounded sum of the
exact products (Dekker's two-product split, then math.fsum over products and their errors).  Per
entry the int8 result must lie within

  (a) its a-priori bound  2^-(s_i+1) sum_k |x_kj| + 2^-(s_j+1) sum_k |x_ki| + n 2^-(s_i + s_j + 2)
      + 2 2^-53 |S_ij|   (the rounding of x to x' = rint(x 2^s), s the column's scaling the library
      reports, the one final rounding, and the reference's own rounding to fp64), and
  (b) the fp64 GEMM's own bound  u sum_k |x_ki x_kj|,  u = 2^-53,

on Gaussian data (fp64 and fp32 storage, row counts across the 65,536-row SYRK splits and partial
64-row stages, odd widths).  The fp64 MFMA Gram's own error on the same entries is printed beside it.
Then the fits: the cross-product EM run with the int8 Gram equals the streaming one (log-likelihood
1e-12, loadings 1e-10), and data whose column spread the scheme cannot cover fall back to the fp64
Gram (gram_info) with the same fit.
"""
import math

import numpy as np
import pytest

from conftest import make_problem

pytestmark = pytest.mark.gpu

U = 2.0 ** -53


def _split(a):
    c = 134217729.0 * a
    hi = c - (c - a)
    return hi, a - hi


def exact_dot(a, b):
    """The correctly rounded value of sum_k a_k b_k (fp64 inputs) and sum_k |a_k b_k|."""
    p = a * b
    ah, al = _split(a)
    bh, bl = _split(b)
    e = ((ah * bh - p) + ah * bl + al * bh) + al * bl
    return math.fsum(np.concatenate([p, e])), math.fsum(np.abs(p))


def _check_entries(D, G, shift, nsample, rng, label):
    n, p = D.shape
    mx = np.abs(D).max(axis=0)
    s_ = np.asarray(shift, dtype=np.float64)
    assert len(s_) == p
    asum = np.abs(D).sum(axis=0)
    worst_a = worst_b = 0.0
    pairs = [(i, i) for i in range(min(p, 8))] + [(int(rng.integers(p)), int(rng.integers(p))) for _ in range(nsample)]
    for i, j in pairs:
        if mx[i] == 0 or mx[j] == 0:
            assert G[i, j] == 0.0
            continue
        s, sa = exact_dot(D[:, i], D[:, j])
        err = abs(G[i, j] - s)
        # the integer rounding of x, the one rounding of the exact integer sum, and the rounding of
        # the reference s itself (the correctly rounded exact sum: |G - s| can reach a whole ulp when
        # the scaled integer sum and the exact sum straddle a midpoint)
        bound = 2.0 ** -(s_[i] + 1) * asum[j] + 2.0 ** -(s_[j] + 1) * asum[i] + n * 2.0 ** -(s_[i] + s_[j] + 2) \
            + 2 * U * abs(s)
        assert err <= bound * (1 + 1e-12), (label, i, j, err, bound)
        worst_a = max(worst_a, err / bound)
        if sa > 0:
            worst_b = max(worst_b, err / (U * sa))
    return worst_a, worst_b


def _check_shift_rule(D, shift, L):
    """The scalings follow the plan (ppls_capi.cpp gram_run_oz): s_j = L_j - e_j with max|D_j| < 2^e_j,
    L_j = 55 + ceil(log2 c_j), c_j = 2^e_j sqrt(n / sum D_j^2) -- columns whose log2 c_j lies within
    1e-9 of an integer are skipped (the device's sum of squares may round the other way) -- and
    L = max_j L_j."""
    n = D.shape[0]
    mx = np.abs(D).max(axis=0)
    ss = (D * D).sum(axis=0)
    Lmax = 55
    for j in np.nonzero(mx > 0)[0]:
        e = math.frexp(mx[j])[1]
        lc = math.log2(max(1.0, 2.0 ** e * math.sqrt(n / ss[j])))
        Lj = e + int(shift[j])
        Lmax = max(Lmax, Lj)
        if abs(lc - round(lc)) > 1e-9:
            assert Lj == 55 + math.ceil(lc), (j, Lj, lc)
    assert Lmax == L


def _check_integer_pipeline(D, G, shift, pairs):
    """Bit for bit: G_ij = the correctly rounded 2^-(s_i + s_j) sum_k x'_ki x'_kj, x' = rint(x 2^s) in
    Python integers (the residues, SYRKs and CRT reproduce the integer sum exactly)."""
    from fractions import Fraction
    s_ = [int(v) for v in shift]
    for i, j in pairs:
        xi = [round(Fraction(float(a)) * Fraction(2) ** s_[i]) for a in D[:, i]]
        xj = [round(Fraction(float(a)) * Fraction(2) ** s_[j]) for a in D[:, j]]
        want = float(Fraction(sum(a * b for a, b in zip(xi, xj))) * Fraction(2) ** -(s_[i] + s_[j]))
        assert G[i, j] == want, (i, j, G[i, j].hex(), want.hex())


@pytest.mark.parametrize("dtype", [0, 1], ids=["f64", "f32"])
@pytest.mark.parametrize("n,p,q", [(1, 3, 2), (5, 17, 4), (127, 40, 9), (3000, 300, 31), (70_001, 70, 13),
                                   (140_000, 33, 5)])
def test_int8_gram_matches_exact_sums(dtype, n, p, q):
    from ppls_amd import Context
    X, Y, _ = make_problem(n, p, q, 1, seed=n + p)
    if dtype:
        X = X.astype(np.float32).astype(np.float64)
        Y = Y.astype(np.float32).astype(np.float64)
    rng = np.random.default_rng(7)
    with Context(0) as c:
        c.set_option("dtype", dtype)
        c.set_data(X, Y)
        for which, D in ((0, X), (1, Y)):
            G, info = c.gram_int8(which)
            assert 12 <= info["nmod"] <= 20 and info["L"] <= 62
            _check_shift_rule(D, info["shift"], info["L"])
            assert np.array_equal(G, G.T)
            wa, wb = _check_entries(D, G, info["shift"], 200 if n < 100_000 else 60, rng, (which, n, p))
            if n <= 5000:
                k = D.shape[1]
                _check_integer_pipeline(D, G, info["shift"], [(0, 0), (k - 1, 0), (k - 1, k - 1)] +
                                        [(int(rng.integers(k)), int(rng.integers(k))) for _ in range(12)])
            Gf, _ = c.gram(which)   # the fp64 MFMA Gram, for the record
            if n >= 100:
                assert wb <= 1.0, (which, wb)   # (b): within the fp64 GEMM's own bound
            print(f"n={n} which={which} dtype={dtype}: nmod {info['nmod']} L {info['L']}: int8 error / a-priori "
                  f"bound {wa:.3g}, / (u sum|x x|) {wb:.3g}; fp64-MFMA max |diff| to int8 "
                  f"{np.abs(Gf - G).max() / max(np.abs(G).max(), 1e-300):.2e} rel")


@pytest.mark.parametrize("dtype,n,p,q", [(0, 1_000_000, 300, 100), (1, 500_000, 1500, 100)], ids=["c3_rows_f64", "c5_rows_f32"])
def test_int8_gram_full_row_counts(dtype, n, p, q):
    """At the bench configs' row counts (C3's 1e6 rows in 16 SYRK splits, C5's 5e5 fp32-stored rows in 8;
    fewer columns so the host reference stays cheap): sampled entries of the joint Gram within the
    a-priori bound and within u sum|x_ki x_kj| against double-double exact sums.  Per-column widths
    keep every sum_k x'^2 below n 2^112: 17 moduli at both row counts (one shared width took 18 at
    1e6 rows)."""
    from ppls_amd import Context
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, p)) * np.exp(rng.uniform(-3, 3, p))   # columns of different scales
    Y = rng.standard_normal((n, q))
    if dtype:
        X = X.astype(np.float32).astype(np.float64)
        Y = Y.astype(np.float32).astype(np.float64)
    with Context(0) as c:
        c.set_option("dtype", dtype)
        c.set_data(X, Y)
        for which, D in ((0, X), (1, Y)):
            G, info = c.gram_int8(which)
            assert info["L"] <= 62 and info["nmod"] == 17, info["nmod"]
            _check_shift_rule(D, info["shift"], info["L"])
            wa, wb = _check_entries(D, G, info["shift"], 24, rng, (which, n, p))
            assert wb <= 1.0, (which, wb)
            print(f"n={n} which={which} dtype={dtype}: nmod {info['nmod']} L {info['L']}: / a-priori {wa:.3g}, "
                  f"/ (u sum|x x|) {wb:.3g}, SYRK {info['ms'][1]:.1f} ms")


def test_int8_joint_gram_blocks():
    """The joint [X Y]'[X Y] over the padded columns (what forms S): its X'X and Y'Y blocks equal the
    per-block int8 Grams bit for bit (each column's scaling depends on that column alone, integer sums
    are exact), the X'Y block matches exact sums within its bound, padding columns are 0."""
    from ppls_amd import Context
    n, p, q = 9000, 61, 45
    X, Y, _ = make_problem(n, p, q, 1, seed=3)
    with Context(0) as c:
        c.set_data(X, Y)
        GJ, info = c.gram_int8(2)
        GX, ix = c.gram_int8(0)
        GY, iy = c.gram_int8(1)
    ldx = GJ.shape[0] - (q + 1) // 2 * 2   # fp64 rows of p <= 2048 columns are padded to even lengths
    assert ldx >= p
    assert np.array_equal(info["shift"][:p], ix["shift"]) and np.array_equal(info["shift"][ldx:ldx + q], iy["shift"])
    assert np.all(info["shift"][p:ldx] == 0)
    assert np.array_equal(GJ[:p, :p], GX)
    assert np.array_equal(GJ[ldx:ldx + q, ldx:ldx + q], GY)
    assert np.all(GJ[p:ldx, :] == 0) and np.all(GJ[:, p:ldx] == 0)
    D = np.hstack([X, np.zeros((n, ldx - p)), Y, np.zeros((n, GJ.shape[0] - ldx - q))])
    _check_entries(D, GJ, info["shift"], 150, np.random.default_rng(2), "joint")


@pytest.mark.parametrize("dtype", [0, 1], ids=["f64", "f32"])
def test_xprod_fit_with_int8_gram_equals_streaming(dtype):
    """The EM loop from S formed by the int8 Gram = the streaming fit (the iterates of
    EM_W_multi.R:780-793 to rounding); gram_info names the Gram that ran."""
    from ppls_amd import Context, Theta
    n, p, q, r = 20_000, 150, 90, 4
    X, Y, th0 = make_problem(n, p, q, r, seed=11)
    th = Theta(th0["W"], th0["C"], th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    with Context(0) as c:
        c.set_option("dtype", dtype)
        c.set_data(X, Y)
        c.set_option("xprod", 0)
        est_s, ll_s, _, _ = c.em_run(th, 12, -np.inf, 0, want_eout=False)
        c.set_option("xprod", 1)
        c.set_option("gram_int8", 1)
        est_x, ll_x, _, _ = c.em_run(th, 12, -np.inf, 0, want_eout=False)
        gi = c.gram_info()
        assert gi["int8"] and c.xprod_info(r)["ready"]
        assert np.abs(ll_x - ll_s).max() / np.abs(ll_s).max() < 1e-12
        assert np.abs(est_x.W - est_s.W).max() < 1e-10 and np.abs(est_x.C - est_s.C).max() < 1e-10
        # option changes drop S; the fp64 Gram forms it again and gives the same fit
        c.set_option("gram_int8", 0)
        est_f, ll_f, _, _ = c.em_run(th, 12, -np.inf, 0, want_eout=False)
        assert not c.gram_info()["int8"]
        assert np.abs(ll_f - ll_x).max() / np.abs(ll_s).max() < 1e-12


def test_int8_workspace_reused_across_release_and_new_data():
    """The residue planes outlive ppls_xprod_release and new data (a workspace, ppls.h "gram_int8"):
    S formed again after a release is bitwise the same (integer sums); a smaller problem in the larger
    workspace and the workspace freed by gram_int8 = 0 and allocated again give exact-sum results."""
    from ppls_amd import Context, Theta
    n, p, q, r = 30_000, 200, 70, 3
    X, Y, th0 = make_problem(n, p, q, r, seed=21)
    th = Theta(th0["W"], th0["C"], th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    rng = np.random.default_rng(5)
    with Context(0) as c:
        c.set_data(X, Y)
        c.set_option("xprod", 1)
        c.set_option("gram_int8", 1)
        est1, ll1, _, _ = c.em_run(th, 8, -np.inf, 0, want_eout=False)
        assert c.gram_info()["int8"]
        c.xprod_release()
        est2, ll2, _, _ = c.em_run(th, 8, -np.inf, 0, want_eout=False)
        assert c.gram_info()["int8"]
        assert np.array_equal(ll1, ll2) and np.array_equal(est1.W, est2.W) and np.array_equal(est1.C, est2.C)
        X2, Y2, _ = make_problem(4000, 90, 33, 1, seed=22)
        c.set_data(X2, Y2)
        for step in range(2):
            G, info = c.gram_int8(0)
            _check_entries(X2, G, info["shift"], 60, rng, ("reuse", step))
            _check_integer_pipeline(X2, G, info["shift"], [(0, 0), (89, 3), (17, 17)])
            c.set_option("gram_int8", 0)   # frees the workspace; the next formation allocates it again
            c.set_option("gram_int8", 1)


def test_int8_gram_falls_back_when_the_spread_is_too_wide():
    """A column whose largest value dwarfs its typical ones needs L > 62 bits (c_j = 2^e_j sqrt(n /
    sum x^2) huge): the int8 form declines and S comes from the fp64 MFMA Gram -- same fit."""
    from ppls_amd import Context, PplsError, Theta
    n, p, q, r = 40_000, 40, 30, 2
    X, Y, th0 = make_problem(n, p, q, r, seed=5)
    # column 3: one huge value among O(1) ones: c_3 ~ 2^30 / 1e9 sqrt(n) ~ 215 > 2^7, L = 63 (a lone
    # outlier gives c <= 2 sqrt(n): at n = 4,000 it would still fit in L = 62)
    X[17, 3] = 1e9
    th = Theta(th0["W"], th0["C"], th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    with Context(0) as c:
        c.set_data(X, Y)
        with pytest.raises(PplsError):
            c.gram_int8(0)
        c.set_option("xprod", 0)
        _, ll_s, _, _ = c.em_run(th, 6, -np.inf, 0, want_eout=False)
        c.set_option("xprod", 1)
        c.set_option("gram_int8", 1)
        _, ll_x, _, _ = c.em_run(th, 6, -np.inf, 0, want_eout=False)
        assert not c.gram_info()["int8"]
        assert np.abs(ll_x - ll_s).max() / np.abs(ll_s).max() < 1e-12


@pytest.mark.parametrize("k", [2, 3])
def test_int8_gram_sharded_equals_unsharded(k):
    """Row shards each forming their S by the int8 form (their own column plans), ONE all-reduce of S
    (host reducer), then the iterations: ranks bitwise identical, the fit equal to the unsharded int8 and
    streaming fits.  One rank's outlier makes only that rank fall back to the fp64 Gram: no collective
    depends on the choice."""
    from ppls_amd import Context, Theta
    from test_gpu_multirank import _run_ranks
    n, p, q, r = 60_000, 60, 40, 2   # shards of >= 20,000 rows: the outlier's c ~ 1.05 sqrt(rows) > 2^7
    X, Y, th0 = make_problem(n, p, q, r, seed=k)
    th = Theta(th0["W"], th0["C"], th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])

    def fit(c, Xs, Ys, n_total, xprod):
        c.set_option("xprod", xprod)
        c.set_option("gram_int8", 1)
        c.set_data(Xs, Ys, n_total=n_total)
        est, ll, _, _ = c.em_run(th, 8, -np.inf, 0, want_eout=False)
        return est, ll, c.gram_info()["int8"] if xprod else None

    for outlier in (False, True):
        Xo = X.copy()
        if outlier:
            Xo[n - 5, 2] = 1e6   # in the last shard only: L = 63 there
        with Context(0) as c:
            ref_s = fit(c, Xo, Y, None, 0)

        def work(rank, c):
            r0, nl = Context.shard_range(n, k, rank)
            return fit(c, Xo[r0:r0 + nl], Y[r0:r0 + nl], n, 1)

        res = _run_ranks(k, work)
        for est, ll, _ in res:
            assert np.array_equal(est.W, res[0][0].W) and np.array_equal(ll, res[0][1])
        used = [u for _, _, u in res]
        assert used[:-1] == [True] * (k - 1) and used[-1] == (not outlier), used
        est, ll, _ = res[0]
        assert np.abs(ll - ref_s[1]).max() / np.abs(ref_s[1]).max() < 1e-11
        if not outlier:   # (a 1e6 entry makes the loadings sensitive to any reordering of the sums)
            assert np.abs(est.W - ref_s[0].W).max() < 1e-9 and np.abs(est.C - ref_s[0].C).max() < 1e-9


@pytest.mark.parametrize("xy", ["X", "Y"])
def test_variances_with_int8_gram(xy):
    """variances.PPLS_simult (EM_W_multi.R:830-860) with its X'X / Y'Y from the int8 form (option
    gram_int8, no S formed): equal to the oracle at the same tolerances as the fp64 Gram's test."""
    import ppls_amd
    from ppls_amd import Context
    from oracle import ppls_oracle as o
    X, Y, th0 = make_problem(1500, 150, 131, 4, seed=67)
    fit = o.ppls_simult(X, Y, 4, EMsteps=15, atol=-np.inf, theta0=th0)
    D = X if xy == "X" else Y
    ref = o.variances_ppls_simult(fit, D, xy)
    with Context(0) as c:
        c.set_data(X, Y)
        c.set_option("gram_int8", 1)
        got = ppls_amd.variances_PPLS_simult(fit, None, xy, ctx=c)
        assert c.gram_info()["int8"]
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
    assert np.abs(got["W"] - ref["W"]).max() < 1e-10
    for i in range(4):
        assert rel(got["varMatrix"][i], ref["varMatrix"][i]) < 1e-8
    assert rel(got["seLoad"], ref["seLoad"]) < 1e-8


@pytest.mark.parametrize("case", range(12))
def test_int8_gram_fuzz(case):
    """Randomised shapes and column distributions (Gaussian, Student-t with 3 degrees of freedom,
    sparse columns, constant columns, integer-valued columns, scales over 1e-6 .. 1e6): wherever the
    int8 form runs (L <= 62), every sampled entry is within its a-priori bound (rigorous: the rounding
    of x' and one final rounding), and for n <= 3000 equal bit for bit to the correctly rounded
    integer sum; where it declines, PplsError (the fp64 Gram then forms S)."""
    from ppls_amd import Context, PplsError
    rng = np.random.default_rng(1000 + case)
    n = int(rng.choice([7, 65, 900, 3000, 20_000, 70_000]))
    p, q = int(rng.integers(1, 90)), int(rng.integers(1, 40))

    def cols(k):
        out = np.empty((n, k))
        for j in range(k):
            kind = rng.integers(5)
            if kind == 0:
                v = rng.standard_normal(n)
            elif kind == 1:
                v = rng.standard_t(3, n)
            elif kind == 2:
                v = rng.standard_normal(n) * (rng.uniform(size=n) < 0.05)
            elif kind == 3:
                v = np.full(n, rng.uniform(-2, 2))
            else:
                v = rng.integers(-1000, 1000, n).astype(np.float64)
            out[:, j] = v * 10.0 ** rng.uniform(-6, 6)
        return out

    X, Y = cols(p), cols(q)
    dtype = int(case % 2)
    if dtype:
        X = X.astype(np.float32).astype(np.float64)
        Y = Y.astype(np.float32).astype(np.float64)
    with Context(0) as c:
        c.set_option("dtype", dtype)
        c.set_data(X, Y)
        for which, D in ((0, X), (1, Y)):
            try:
                G, info = c.gram_int8(which)
            except PplsError:
                continue
            assert np.array_equal(G, G.T)
            _check_entries(D, G, info["shift"], 40, rng, ("fuzz", case, which, n))
            if n <= 3000:
                k = D.shape[1]
                _check_integer_pipeline(D, G, info["shift"], [(int(rng.integers(k)), int(rng.integers(k))) for _ in range(8)])


@pytest.mark.parametrize("config", ["c3", "c5"])
def test_int8_gram_full_size_fit_equals_streaming(config):
    """The bench configs at full size with S from the int8 Gram (C3: 1e6 x 4000 fp64, 18 moduli; C5:
    5e5 x 10,500 fp32-stored, 17 moduli): the cross-product EM iterations equal the streaming ones at
    tests/test_gpu_xprod_full.py's tolerances (loglik 1e-12 relative, loadings 1e-10)."""
    import bench
    from ppls_amd import Context, Theta
    cfg = bench.CONFIGS[config]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    truth, th0 = bench.make_truth_and_theta0(p, q, r)
    th = Theta(th0["W"], th0["C"], th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"]) \
        if isinstance(th0, dict) else th0
    steps = 3
    with Context(0) as c:
        if cfg.get("storage") == "f32":
            c.set_option("dtype", 1)
        c.generate_synthetic(n, p, q, truth, seed=20261015)
        c.set_option("xprod", 0)
        est_s, ll_s, _, _ = c.em_run(th, steps, -np.inf, 0, want_eout=False)
        c.set_option("xprod", 1)
        c.set_option("gram_int8", 1)
        est_x, ll_x, _, _ = c.em_run(th, steps, -np.inf, 0, want_eout=False)
        gi = c.gram_info()
        assert gi["int8"] and 12 <= gi["nmod"] <= 20, gi
    assert np.abs(ll_x - ll_s).max() / np.abs(ll_s).max() < 1e-12
    assert np.abs(est_x.W - est_s.W).max() < 1e-10 and np.abs(est_x.C - est_s.C).max() < 1e-10
