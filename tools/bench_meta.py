"""Time meta_PPLSi (EM_W_multi.R:509-589) on the device at a bench workload with K populations, against
one r = 1 sweep of the same data (the sequential initialiser's step: tools/bench_init.py).

    python tools/bench_meta.py [c3|c2|c4s|c5|c5s] [--K 4] [--steps 20] [--host]

--host: the per-population host loop (option meta_device = 0) instead of the device loop.
fp32-storage configs (c5, c5s) store X, Y in fp32 (option dtype 1): the panel sweep, one launch per
population and EM step (round 6).

One meta EM step = one segmented r = 1 sweep over all rows (each workgroup's rows in one
population, with that population's scalars) + a reduction per population + the device M-step /
log-likelihood / stop-rule kernel.  Per-step time = (t(steps) - t(5)) / (steps - 5) with atol = -Inf
(every step runs; the difference removes setup: population sums of squares, allocations).  Prints
one JSON line.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context, initial_guess  # noqa: E402


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "c3"
    K = int(sys.argv[sys.argv.index("--K") + 1]) if "--K" in sys.argv else 4
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 20
    host = "--host" in sys.argv
    cfg = CONFIGS[cfgname]
    n, p, q = cfg["n"], cfg["p"], cfg["q"]
    truth, _ = make_truth_and_theta0(p, q, 1)
    ctx = Context(0)
    esz = 4 if cfg.get("storage") == "f32" else 8
    if esz == 4:
        ctx.set_option("dtype", 1)
    ctx.set_option("meta_device", 0 if host else 1)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    # K populations of unequal sizes (level order: contiguous row blocks)
    w = np.linspace(1.4, 0.6, K)
    sizes = np.floor(w / w.sum() * n).astype(np.int64)
    sizes[-1] = n - sizes[:-1].sum()
    init = initial_guess(p, q, "equal")
    ctx.meta_ppls(sizes, 2, -np.inf, init)   # warm-up
    ts = {}
    for s in (5, steps):
        best = None
        for _ in range(3):
            ctx.synchronize()
            t0 = time.perf_counter()
            W, C, params, lg = ctx.meta_ppls(sizes, s, -np.inf, init)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        ts[s] = best
        assert lg.shape[0] == s + 1 and np.isfinite(lg).all()
    path = ctx.meta_info()
    per_step = (ts[steps] - ts[5]) / (steps - 5)
    # one r = 1 sweep of the whole data: the initialiser's rank-1 fit, steps x (sweep + step kernel)
    inits = [initial_guess(p, q, "equal")]
    ctx.ppls(1, 2, -np.inf, inits)
    tr = {}
    for s in (5, steps):
        best = None
        for _ in range(3):
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.ppls(1, s, -np.inf, inits)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        tr[s] = best
    r1_step = (tr[steps] - tr[5]) / (steps - 5)
    out = dict(workload=cfg["name"], K=K, population_rows=[int(x) for x in sizes], steps=steps,
               meta_seconds={str(k): v for k, v in ts.items()}, meta_ms_per_step=1e3 * per_step,
               rank1_ms_per_step=1e3 * r1_step, ratio=per_step / r1_step,
               meta_TBps=esz * n * (p + q) / per_step / 1e12, storage="f32" if esz == 4 else "f64", path=path,
               what="meta EM step: one segmented r = 1 sweep + K reductions + the device M-step kernel; "
                    "rank-1 step: one r = 1 sweep + the device rank-1 step kernel (PPLSi)")
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
