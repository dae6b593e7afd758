"""ALGORITHM-LEVEL test of the data-parallel decomposition, world size 2 on CPU (gloo).

This checks the sharding algorithm, not the device path: per EM iteration each rank reduces ITS
rows to the sufficient statistics [X'mu_T | Y'mu_U | Gram] with the ORACLE's sweep_stats (no GPU
here), the ranks all-reduce them (the one RCCL call per iteration on the GPU), and every rank runs
the SAME finalize (the library's ppls_finalize_host, i.e. the device finalize's ppls_math.h code
compiled for the host) -- no broadcast.  Checks: the sharded run equals the unsharded oracle
PPLS_simult, and both ranks hold bit-identical parameters after every iteration.  The same
decomposition through the device sweep is tests/test_gpu_multirank.py (k contexts, two gloo
processes, and the full-size C4 eight-shard run).
"""
import ctypes as ct
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, make_problem


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, steps, q_out):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from conftest import make_problem as mk
    from oracle import ppls_oracle as o
    from ppls_amd import Context
    from ppls_amd._lib import Expect, Theta, dptr, lib

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    X, Y, th0 = mk(301, 23, 17, 3, seed=123)
    row0, nl = Context.shard_range(X.shape[0], world, rank)
    Xs, Ys = X[row0:row0 + nl], Y[row0:row0 + nl]
    # PPLS_simult canonicalises theta0 first (:773-778); th0 is already in canonical order
    th = Theta(**th0)
    ssq = torch.tensor([np.sum(Xs * Xs), np.sum(Ys * Ys)], dtype=torch.float64)
    dist.all_reduce(ssq)
    trace = []
    for _ in range(steps):
        cf = o.mu_coefficients(np.diag(th.B), th.sigE, th.sigF, th.sigH, np.diag(th.sigT))
        st = o.sweep_stats(Xs, Ys, th.W, th.C, cf)
        buf = torch.from_numpy(np.concatenate([st["SX"].ravel(order="F"), st["SY"].ravel(order="F"),
                                               st["G"].ravel(order="F")]))
        dist.all_reduce(buf)                         # the per-iteration all-reduce
        b = buf.numpy()
        p, q, r = th.W.shape[0], th.C.shape[0], th.r
        SX = np.asfortranarray(b[:p * r].reshape((p, r), order="F"))
        SY = np.asfortranarray(b[p * r:(p + q) * r].reshape((q, r), order="F"))
        G = np.asfortranarray(b[(p + q) * r:].reshape((2 * r, 2 * r), order="F"))
        nx = Theta.empty(p, q, r)
        e = Expect(r)
        ll = ct.c_double()
        t, ns, es = th.struct(), nx.struct(), e.struct()
        rc = lib().ppls_finalize_host(dptr(SX), dptr(SY), dptr(G), float(ssq[0]), float(ssq[1]),
                                      float(X.shape[0]), p, q, r, ct.byref(t), 0, ct.byref(ns),
                                      ct.byref(es), ct.byref(ll))
        assert rc == 0
        nx.pull(ns)
        trace.append(ll.value)   # logl of the theta this sweep used
        th = nx
    q_out.put((rank, th.W.copy(), th.C.copy(), th.B.copy(), th.sigT.copy(),
               (th.sigE, th.sigF, th.sigH), trace))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_em_equals_unsharded_oracle(world):
    from oracle import ppls_oracle as o
    steps = 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    # every rank ran the same finalize on the same reduced statistics -> identical theta
    for other in res[1:]:
        for a, b in zip(res[0][1:6], other[1:6]):
            assert np.array_equal(np.asarray(a), np.asarray(b))
    X, Y, th0 = make_problem(301, 23, 17, 3, seed=123)
    ref = o.ppls_simult(X, Y, 3, EMsteps=steps, atol=-np.inf, theta0=th0)
    # trace[i] = logl(theta_i) for i = 0..steps-1; the reference's loglik[i] = logl(theta_{i+1})
    trace = np.array(res[0][6])
    assert np.allclose(trace[1:], ref["loglik"][:-1], rtol=1e-12, atol=0)
    # un-canonicalised final W vs the oracle's canonicalised estimates: compare via canonicalize
    W, C, B, T = o.canonicalize(res[0][1], res[0][2], np.diag(res[0][3]), np.diag(res[0][4]))
    assert np.abs(W - ref["estimates"]["W"]).max() < 1e-10
    assert np.abs(C - ref["estimates"]["C"]).max() < 1e-10


def _meta_worker(rank, world, port, q_out):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from oracle import ppls_oracle as o
    from ppls_amd.api import pop_rows
    from ppls_amd import Context

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    g = np.load(os.path.join(ROOT, "tests", "golden", "meta_random_k3_p24_q18.npz"))
    import json
    sizes = json.loads(str(g["meta"]))["sizes"]
    X, Y = g["X"], g["Y"]
    n = X.shape[0]
    row0, nl = Context.shard_range(n, world, rank)
    loc, tot = pop_rows(sizes, row0, nl)
    cf = o.mu_coefficients(np.eye(1) * 1.2, 0.7, 0.6, 0.3, np.eye(1) * 0.9)
    w, c = g["init_W"].reshape(-1, 1), g["init_C"].reshape(-1, 1)
    out = []
    r0 = row0
    for j in range(len(sizes)):   # this rank's rows of population j: one segment sweep + all-reduce
        Xj, Yj = X[r0:r0 + loc[j]], Y[r0:r0 + loc[j]]
        st = o.sweep_stats(Xj, Yj, w, c, cf)
        buf = torch.from_numpy(np.concatenate([st["SX"].ravel(), st["SY"].ravel(), st["G"].ravel(),
                                               [np.sum(Xj * Xj), np.sum(Yj * Yj)]]))
        dist.all_reduce(buf)
        out.append(buf.numpy().copy())
        r0 += loc[j]
    q_out.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_meta_population_statistics(world):
    """meta_* on sharded rows: each rank sweeps the intersection of its shard with each population
    block; the all-reduced per-population statistics equal the unsharded ones."""
    import json
    from oracle import ppls_oracle as o
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_meta_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    g = np.load(os.path.join(ROOT, "tests", "golden", "meta_random_k3_p24_q18.npz"))
    sizes = json.loads(str(g["meta"]))["sizes"]
    X, Y = g["X"], g["Y"]
    cf = o.mu_coefficients(np.eye(1) * 1.2, 0.7, 0.6, 0.3, np.eye(1) * 0.9)
    w, c = g["init_W"].reshape(-1, 1), g["init_C"].reshape(-1, 1)
    Ni = np.concatenate([[0], np.cumsum(sizes)])
    for j in range(len(sizes)):
        Xj, Yj = X[Ni[j]:Ni[j + 1]], Y[Ni[j]:Ni[j + 1]]
        st = o.sweep_stats(Xj, Yj, w, c, cf)
        ref = np.concatenate([st["SX"].ravel(), st["SY"].ravel(), st["G"].ravel(), [np.sum(Xj * Xj), np.sum(Yj * Yj)]])
        for rk in range(world):
            assert np.allclose(res[rk][1][j], ref, rtol=1e-12, atol=1e-10)


def _xprod_worker(rank, world, port, steps, q_out):
    """The cross-product form's N > 1 decomposition: each rank forms S over ITS
    rows (oracle.crossproducts), ONE all-reduce of S, then every iteration is computed from S
    (oracle.xprod_stats) and finalized identically on every rank, with no per-iteration collective."""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from conftest import make_problem as mk
    from oracle import ppls_oracle as o
    from ppls_amd import Context
    from ppls_amd._lib import Expect, Theta, dptr, lib

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    X, Y, th0 = mk(301, 23, 17, 3, seed=123)
    row0, nl = Context.shard_range(X.shape[0], world, rank)
    Xs, Ys = X[row0:row0 + nl], Y[row0:row0 + nl]
    S = torch.from_numpy(o.crossproducts(Xs, Ys))
    dist.all_reduce(S)                                   # the one collective of the fit
    S = S.numpy()
    p, q = X.shape[1], Y.shape[1]
    ssqX, ssqY = float(np.trace(S[:p, :p])), float(np.trace(S[p:, p:]))   # ||X||^2, ||Y||^2 from S
    th = Theta(**th0)
    trace = []
    for _ in range(steps):
        cf = o.mu_coefficients(np.diag(th.B), th.sigE, th.sigF, th.sigH, np.diag(th.sigT))
        st = o.xprod_stats(S, p, th.W, th.C, cf)
        r = th.r
        SX, SY, G = (np.asfortranarray(st[k]) for k in ("SX", "SY", "G"))
        nx = Theta.empty(p, q, r)
        e = Expect(r)
        ll = ct.c_double()
        t, ns, es = th.struct(), nx.struct(), e.struct()
        rc = lib().ppls_finalize_host(dptr(SX), dptr(SY), dptr(G), ssqX, ssqY, float(X.shape[0]), p, q, r,
                                      ct.byref(t), 0, ct.byref(ns), ct.byref(es), ct.byref(ll))
        assert rc == 0
        nx.pull(ns)
        trace.append(ll.value)
        th = nx
    q_out.put((rank, th.W.copy(), th.C.copy(), th.B.copy(), th.sigT.copy(),
               (th.sigE, th.sigF, th.sigH), trace))
    dist.barrier()
    dist.destroy_process_group()


def test_crossproduct_stats_equal_sweep_stats():
    """oracle.xprod_stats from S == oracle.sweep_stats from the rows (the identity of §12)."""
    from oracle import ppls_oracle as o
    X, Y, th0 = make_problem(400, 31, 19, 4, seed=8)
    cf = o.mu_coefficients(th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    a = o.sweep_stats(X, Y, th0["W"], th0["C"], cf)
    b = o.xprod_stats(o.crossproducts(X, Y), 31, th0["W"], th0["C"], cf)
    for k in ("SX", "SY", "G"):
        assert np.abs(a[k] - b[k]).max() / np.abs(a[k]).max() < 1e-13


def test_sharded_crossproduct_em_equals_unsharded_oracle():
    from oracle import ppls_oracle as o
    world, steps = 2, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xprod_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for a, b in zip(res[0][1:6], res[1][1:6]):
        assert np.array_equal(np.asarray(a), np.asarray(b))   # identical on every rank, no broadcast
    X, Y, th0 = make_problem(301, 23, 17, 3, seed=123)
    ref = o.ppls_simult(X, Y, 3, EMsteps=steps, atol=-np.inf, theta0=th0)
    trace = np.array(res[0][6])
    assert np.allclose(trace[1:], ref["loglik"][:-1], rtol=1e-11, atol=0)
    W, C, B, T = o.canonicalize(res[0][1], res[0][2], np.diag(res[0][3]), np.diag(res[0][4]))
    assert np.abs(W - ref["estimates"]["W"]).max() < 1e-10
    assert np.abs(C - ref["estimates"]["C"]).max() < 1e-10

