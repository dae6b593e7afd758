"""The N > 1 data-parallel path through the library itself (device sweeps, library reductions).

Rows are sharded over ranks (EM_W_multi.R:689-712 and :732-733 are sums over rows), each rank's
context sweeps its own rows and every collective of the library -- the per-iteration
[X'mu_T | Y'mu_U | Gram] statistics, ||X||^2 and ||Y||^2, the initialiser's and meta_*'s sums --
goes through ppls_set_reducer, the host-side reduction hook:

* k contexts on GPU 0 in one process, one host thread per rank, summing in rank order: the sharded
  fit must equal the unsharded fit (1e-12) and every rank must hold bit-identical estimates;
* two processes on GPU 0 with torch.distributed gloo as the reducer (the RCCL path's structure
  with gloo doing the all-reduce), checked against the CPU oracle.
"""
import os
import socket
import threading

import numpy as np
import pytest

from conftest import ROOT, make_problem
from oracle import ppls_oracle as o

pytestmark = pytest.mark.gpu


class ThreadAllReduce:
    """Sum over k host threads, in rank order (so every rank gets the bitwise-same result)."""

    def __init__(self, k):
        self.k = k
        self.bar = threading.Barrier(k, timeout=120)
        self.bufs = [None] * k
        self.calls = 0

    def fn(self, rank):
        def reduce(buf):
            self.bufs[rank] = buf.copy()
            self.bar.wait()
            tot = self.bufs[0].copy()
            for b in self.bufs[1:]:
                tot += b
            self.bar.wait()   # everyone has read the inputs before the next call overwrites them
            if rank == 0:
                self.calls += 1
            buf[:] = tot
        return reduce


def _run_ranks(k, work):
    """work(rank, ctx) on k threads, each with its own context on GPU 0; returns the results."""
    from ppls_amd import Context
    red = ThreadAllReduce(k)
    out, errs = [None] * k, []

    def body(rank):
        try:
            with Context(0) as c:
                c.set_reducer(red.fn(rank))
                out[rank] = work(rank, c)
        except BaseException as e:   # noqa: BLE001
            errs.append(e)
            red.bar.abort()

    ths = [threading.Thread(target=body, args=(i,)) for i in range(k)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=300)
    if errs:
        raise errs[0]
    assert red.calls > 0
    return out


def _theta(th):
    from ppls_amd import Theta
    return Theta(th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])


@pytest.mark.parametrize("k,n,p,q,r,dtype", [(3, 3001, 300, 200, 4, 0), (4, 2000, 700, 90, 10, 0),
                                             (2, 1500, 260, 130, 3, 1), (4, 3, 20, 12, 2, 0),
                                             (4, 3, 20, 12, 2, 1)],
                         ids=["split_k3", "panel_k4", "panel_fp32_k2", "split_empty_shard",
                              "panel_fp32_empty_shard"])
def test_k_contexts_sharded_equal_unsharded(k, n, p, q, r, dtype):
    from ppls_amd import Context
    X, Y, th0 = make_problem(n, p, q, r, seed=n + k)
    steps = 6

    def fit(c, Xs, Ys, n_total):
        c.set_option("dtype", dtype)
        c.set_data(Xs, Ys, n_total=n_total)
        est, ll, eout, _ = c.em_run(_theta(th0), steps, -np.inf, 0)
        return est, ll, eout, c.sweep_info(r)["variant"]

    with Context(0) as c:
        ref = fit(c, X, Y, None)

    def work(rank, c):
        r0, nl = Context.shard_range(n, k, rank)
        return fit(c, X[r0:r0 + nl], Y[r0:r0 + nl], n)

    res = _run_ranks(k, work)
    assert min(Context.shard_range(n, k, rk)[1] for rk in range(k)) >= (0 if n < k else 1)
    assert res[0][3] == ref[3] == ("split512" if (r <= 8 and not dtype and p <= 2048) else "panel")
    for est, ll, eout, _ in res:
        assert np.array_equal(est.W, res[0][0].W) and np.array_equal(est.C, res[0][0].C)
        assert np.array_equal(ll, res[0][1])
        assert np.array_equal(eout.Ctt, res[0][2].Ctt) and eout.Cee == res[0][2].Cee
    est, ll, eout, _ = res[0]
    # (3 rows with p >> n: an ill-posed fit that amplifies the sharded sums' rounding ~100x)
    tol = 1e-12 if n >= 100 else 1e-10
    assert np.abs(ll - ref[1]).max() / np.abs(ref[1]).max() < tol
    assert np.abs(est.W - ref[0].W).max() < tol and np.abs(est.C - ref[0].C).max() < tol
    assert np.abs(est.B - ref[0].B).max() / np.abs(ref[0].B).max() < tol
    assert abs(est.sigE - ref[0].sigE) / ref[0].sigE < tol
    # Eout rows stay sharded: the concatenation is the unsharded mu_T (a rank with no rows holds none)
    mu = np.vstack([e.mu_T.reshape(-1, r) for _, _, e, _ in res])
    assert np.abs(mu - ref[2].mu_T).max() / np.abs(ref[2].mu_T).max() < tol


def test_k_contexts_initialiser_and_meta_sharded():
    """PPLS (sequential initialiser) and meta_PPLSi on 3 row shards equal the unsharded fits."""
    from ppls_amd import Context
    from ppls_amd.api import initial_guess
    k, n, p, q, a = 3, 900, 60, 40, 2
    X, Y, _ = make_problem(n, p, q, a, seed=5)
    inits = [initial_guess(p, q, "equal") for _ in range(a)]
    sizes = [400, 200, 300]
    init = initial_guess(p, q, "equal")

    def fits(c):
        f = c.ppls(a, 20, 1e-4, inits)
        m = c.meta_ppls(sizes, 30, 1e-6, init)
        return f, m

    with Context(0) as c:
        c.set_data(X, Y)
        ref = fits(c)

    def work(rank, c):
        r0, nl = Context.shard_range(n, k, rank)
        c.set_data(X[r0:r0 + nl], Y[r0:r0 + nl], n_total=n)
        c.row0 = r0
        return fits(c)

    res = _run_ranks(k, work)
    for f, m in res:
        assert np.array_equal(f["W"], res[0][0]["W"]) and np.array_equal(m[0], res[0][1][0])
    f, m = res[0]
    assert np.abs(f["W"] - ref[0]["W"]).max() < 1e-12 and np.abs(f["C"] - ref[0]["C"]).max() < 1e-12
    assert np.abs(f["sig"] - ref[0]["sig"]).max() < 1e-12
    assert np.abs(m[0] - ref[1][0]).max() < 1e-12 and np.abs(m[2] - ref[1][2]).max() < 1e-11
    assert np.allclose(m[3], ref[1][3], rtol=1e-12, atol=0, equal_nan=True)


@pytest.mark.timeout(120)
def test_k_contexts_meta_with_an_empty_shard():
    """meta_PPLSi's device loop with a rank that holds no rows (its workgroup split never
    ended there, and the others waited in the next all-reduce).  Shards [0, 500), [], [500, 700),
    [700, 900): the empty rank launches no sweep, zeroes its statistics and joins every collective;
    all ranks are bitwise equal and equal the unsharded fit."""
    from ppls_amd import Context
    from ppls_amd.api import initial_guess
    n, p, q = 900, 60, 40
    X, Y, _ = make_problem(n, p, q, 1, seed=11)
    sizes = [300, 350, 250]
    init = initial_guess(p, q, "equal")
    shards = [(0, 500), (500, 0), (500, 200), (700, 200)]

    with Context(0) as c:
        c.set_data(X, Y)
        ref = c.meta_ppls(sizes, 25, 1e-6, init)

    def work(rank, c):
        r0, nl = shards[rank]
        c.set_data(X[r0:r0 + nl], Y[r0:r0 + nl], n_total=n)
        c.row0 = r0
        return c.meta_ppls(sizes, 25, 1e-6, init)

    res = _run_ranks(len(shards), work)
    for m in res:
        assert np.array_equal(m[0], res[0][0]) and np.array_equal(m[2], res[0][2])
    m = res[0]
    assert np.abs(m[0] - ref[0]).max() < 1e-12 and np.abs(m[1] - ref[1]).max() < 1e-12
    assert np.abs(m[2] - ref[2]).max() < 1e-11
    assert np.allclose(m[3], ref[3], rtol=1e-12, atol=0, equal_nan=True)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, steps, q_out):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from conftest import make_problem as mk
    from ppls_amd import Context, Theta

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        X, Y, th0 = mk(2501, 120, 80, 3, seed=321)
        r0, nl = Context.shard_range(X.shape[0], world, rank)

        def allreduce(buf):
            dist.all_reduce(torch.from_numpy(buf))   # in place on the library's host staging buffer

        with Context(0) as c:
            c.set_reducer(allreduce)
            c.set_data(X[r0:r0 + nl], Y[r0:r0 + nl], n_total=X.shape[0])
            th = Theta(th0["W"], th0["C"], th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
            est, ll, eout, _ = c.em_run(th, steps, -np.inf, 0)
            q_out.put((rank, est.W, est.C, est.B, est.sigT, (est.sigE, est.sigF, est.sigH), ll, eout.mu_T))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_two_processes_device_sweep():
    import torch.multiprocessing as mp
    world, steps = 2, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(rk, world, port, steps, q)) for rk in range(world)]
    for pr in procs:
        pr.start()
    try:
        res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    finally:
        for pr in procs:
            pr.join(timeout=60)
    assert all(pr.exitcode == 0 for pr in procs)
    for other in res[1:]:   # identical finalize on identical reduced statistics
        for a, b in zip(res[0][1:7], other[1:7]):
            assert np.array_equal(np.asarray(a), np.asarray(b))
    X, Y, th0 = make_problem(2501, 120, 80, 3, seed=321)
    ref = o.ppls_simult(X, Y, 3, EMsteps=steps, atol=-np.inf, theta0=th0)
    e = ref["estimates"]
    assert np.abs(res[0][6] - ref["loglik"]).max() / np.abs(ref["loglik"]).max() < 1e-10
    assert np.abs(res[0][1] - e["W"]).max() < 1e-8 and np.abs(res[0][2] - e["C"]).max() < 1e-8
    mu = np.vstack([res[0][7], res[1][7]])
    assert np.abs(mu - ref["Expectations"]["mu_T"]).max() / np.abs(ref["Expectations"]["mu_T"]).max() < 1e-8


def test_k_contexts_device_stop_rule():
    """A finite atol with sharded ranks: every rank enqueues every iteration (the collective sequence
    must match), the device stop flag makes them all end at the same iteration as the unsharded fit."""
    from ppls_amd import Context
    k, n, p, q, r = 3, 1200, 80, 50, 3
    X, Y, th0 = make_problem(n, p, q, r, seed=77)

    def fit(c, Xs, Ys, n_total):
        c.set_data(Xs, Ys, n_total=n_total)
        est, ll, eout, _ = c.em_run(_theta(th0), 120, 0.5, 0)
        return est, ll

    with Context(0) as c:
        ref = fit(c, X, Y, None)
    assert 2 < len(ref[1]) < 120

    def work(rank, c):
        r0, nl = Context.shard_range(n, k, rank)
        return fit(c, X[r0:r0 + nl], Y[r0:r0 + nl], n)

    res = _run_ranks(k, work)
    for est, ll in res:
        assert len(ll) == len(ref[1]) and np.array_equal(ll, res[0][1])
        assert np.array_equal(est.W, res[0][0].W)
    assert np.abs(res[0][1] - ref[1]).max() / np.abs(ref[1]).max() < 1e-12
    assert np.abs(res[0][0].W - ref[0].W).max() < 1e-12


def test_k_contexts_stop_launching_after_convergence():
    """With collectives every rank breaks at the same iteration soon after the device stop rule
    fires (not after all EMsteps): the number of all-reduces stays near the stopping iteration
    plus the host's look-ahead of 8 iterations, and the fit equals the unsharded one."""
    from ppls_amd import Context
    k, n, p, q, r, steps = 3, 1500, 70, 40, 2, 5000
    X, Y, th0 = make_problem(n, p, q, r, seed=91)

    def fit(c, Xs, Ys, n_total):
        c.set_data(Xs, Ys, n_total=n_total)
        est, ll, _, _ = c.em_run(_theta(th0), steps, 1e-3, 0)
        return est, ll

    with Context(0) as c:
        ref = fit(c, X, Y, None)
    stop = len(ref[1])
    assert 3 <= stop < 1000

    red = ThreadAllReduce(k)
    out, errs = [None] * k, []

    def body(rank):
        try:
            with Context(0) as c:
                c.set_reducer(red.fn(rank))
                r0, nl = Context.shard_range(n, k, rank)
                out[rank] = fit(c, X[r0:r0 + nl], Y[r0:r0 + nl], n)
        except BaseException as e:   # noqa: BLE001
            errs.append(e)
            red.bar.abort()

    ths = [threading.Thread(target=body, args=(i,)) for i in range(k)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=300)
    if errs:
        raise errs[0]
    # set_data's ||X||^2 all-reduce + one per iteration up to stop + 1 + look-ahead
    assert red.calls <= stop + 1 + 8 + 3, (red.calls, stop)
    for est, ll in out:
        assert len(ll) == stop and np.array_equal(ll, out[0][1])
    assert np.abs(out[0][1] - ref[1]).max() / np.abs(ref[1]).max() < 1e-12


def test_c4_full_size_eight_shards():
    """BASELINE config C4 at its full size through the sharded library path: n = 1e6, p = q = 2000,
    r = 5 over 8 row shards (8 contexts on GPU 0, 4 GB each, the host reducer standing in for RCCL),
    3 EM iterations from the bench's theta0.  Sharded must equal unsharded to 1e-12 and all 8 ranks
    must hold bitwise-identical estimates (EM_W_multi.R:689-712, :732-733 are row sums)."""
    from ppls_amd import Context, Theta
    k, n, p, q, r, steps = 8, 1_000_000, 2000, 2000, 5, 3

    def polar(M):
        U, _, Vt = np.linalg.svd(M, full_matrices=False)
        return U @ Vt

    kk = np.arange(r)   # bench.py's truth and theta0
    truth = Theta(polar(np.random.default_rng(1).standard_normal((p, r))),
                  polar(np.random.default_rng(2).standard_normal((q, r))),
                  np.exp(np.log(1.5) - 0.3 * kk), 0.5, 0.5, 0.1, np.exp(-0.1 * kk))
    th0 = dict(W=polar(np.random.default_rng(3).standard_normal((p, r))),
               C=polar(np.random.default_rng(4).standard_normal((q, r))),
               B=np.eye(r), sigE=1.0, sigF=1.0, sigH=1.0, sigT=np.eye(r))

    def fit(c, row0, n_local):
        c.generate_synthetic(n, p, q, truth, seed=20261015, row0=row0, n_local=n_local)
        est, ll, _, _ = c.em_run(_theta(th0), steps, -np.inf, 0, want_eout=False)
        return est, ll, c.sweep_kernel(r)

    with Context(0) as c:
        ref = fit(c, 0, n)
    res = _run_ranks(k, lambda rank, c: fit(c, *Context.shard_range(n, k, rank)))
    assert res[0][2] == ref[2] and res[0][2].startswith("split<5,")
    for est, ll, _ in res:
        for a, b in ((est.W, res[0][0].W), (est.C, res[0][0].C), (est.B, res[0][0].B),
                     (est.sigT, res[0][0].sigT), (ll, res[0][1])):
            assert np.array_equal(a, b)
        assert (est.sigE, est.sigF, est.sigH) == (res[0][0].sigE, res[0][0].sigF, res[0][0].sigH)
    est, ll, _ = res[0]
    assert np.abs(ll - ref[1]).max() / np.abs(ref[1]).max() < 1e-12
    assert np.abs(est.W - ref[0].W).max() < 1e-12 and np.abs(est.C - ref[0].C).max() < 1e-12
    assert np.abs(est.B - ref[0].B).max() / np.abs(ref[0].B).max() < 1e-12
    assert abs(est.sigE - ref[0].sigE) / ref[0].sigE < 1e-12


def test_c5_full_size_eight_shards():
    """BASELINE config C5 at its full size through the sharded library path: n = 5e5, p = 1e4, q = 500,
    r = 10, fp32 storage (the panel sweep) over 8 row shards (8 contexts on GPU 0, 2.6 GB each, the host
    reducer standing in for RCCL), 2 EM iterations: sharded = unsharded to 1e-12, ranks bitwise equal."""
    from ppls_amd import Context, Theta
    k, n, p, q, r, steps = 8, 500_000, 10_000, 500, 10, 2

    def polar(M):
        U, _, Vt = np.linalg.svd(M, full_matrices=False)
        return U @ Vt

    kk = np.arange(r)
    truth = Theta(polar(np.random.default_rng(1).standard_normal((p, r))),
                  polar(np.random.default_rng(2).standard_normal((q, r))),
                  np.exp(np.log(1.5) - 0.3 * kk), 0.5, 0.5, 0.1, np.exp(-0.1 * kk))
    th0 = dict(W=polar(np.random.default_rng(3).standard_normal((p, r))),
               C=polar(np.random.default_rng(4).standard_normal((q, r))),
               B=np.eye(r), sigE=1.0, sigF=1.0, sigH=1.0, sigT=np.eye(r))

    def fit(c, row0, n_local):
        c.set_option("dtype", 1)
        c.generate_synthetic(n, p, q, truth, seed=20261015, row0=row0, n_local=n_local)
        est, ll, _, _ = c.em_run(_theta(th0), steps, -np.inf, 0, want_eout=False)
        return est, ll, c.sweep_info(r)["variant"]

    with Context(0) as c:
        ref = fit(c, 0, n)
    res = _run_ranks(k, lambda rank, c: fit(c, *Context.shard_range(n, k, rank)))
    assert res[0][2] == ref[2] == "panel"
    for est, ll, _ in res:
        for a, b in ((est.W, res[0][0].W), (est.C, res[0][0].C), (est.B, res[0][0].B), (ll, res[0][1])):
            assert np.array_equal(a, b)
    est, ll, _ = res[0]
    assert np.abs(ll - ref[1]).max() / np.abs(ref[1]).max() < 1e-12
    assert np.abs(est.W - ref[0].W).max() < 1e-12 and np.abs(est.C - ref[0].C).max() < 1e-12
    assert np.abs(est.B - ref[0].B).max() / np.abs(ref[0].B).max() < 1e-12
