"""Interleaved A/B of context options at a bench config: ms per EM iteration (device-resident loop,
no host sync inside), plus the last log-likelihood and ||W'W - I|| of the state, so a faster variant
that changes the numbers shows it.

    python tools/option_ab.py <config> "<key=val[,key=val]>" ["<key=val,...>" ...] [--reps 3] [--iters 60]

An empty spec ("") is the defaults.  Each arm restarts from theta0 (3 warm-up iterations).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def parse(spec):
    return [(kv.split("=")[0], int(kv.split("=")[1], 0)) for kv in spec.split(",") if kv]


def main():
    args = sys.argv[1:]
    reps, iters = 3, 60
    if "--reps" in args:
        i = args.index("--reps"); reps = int(args[i + 1]); del args[i:i + 2]
    if "--iters" in args:
        i = args.index("--iters"); iters = int(args[i + 1]); del args[i:i + 2]
    cfgname, specs = args[0], args[1:] or [""]
    cfg = CONFIGS[cfgname]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    if cfg.get("storage") == "f32":
        ctx.set_option("dtype", 1)
    truth, th0 = make_truth_and_theta0(p, q, r)
    n = int(os.environ.get("AB_N", n))   # row-count override (same p, q, r, storage)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    res = {s: [] for s in specs}
    keys = sorted({k for s in specs for k, _ in parse(s)})
    for rep in range(reps):
        for s in specs:
            for k in keys:   # back to the defaults, then this arm's values
                ctx.set_option(k, {"polar1": 1, "nt": -1, "pipe": 1, "xprod_waves": 4, "exact_gram": 1, "dots_pair": -1, "xprod": 0,
                                 "var_chol": 1, "vorth": 8, "meta_device": 1, "xprod_fuse": 1}.get(k, 0))
            for k, v in parse(s):
                ctx.set_option(k, v)
            ctx.em_begin(th0)
            ctx.em_iterate(3)
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.em_iterate(iters)
            ctx.synchronize()
            res[s].append((time.perf_counter() - t0) / iters * 1e3)
            est, ll = ctx.em_state()
            orth = max(np.abs(est.W.T @ est.W - np.eye(r)).max(), np.abs(est.C.T @ est.C - np.eye(r)).max())
            print(f"{cfgname} [{s or 'defaults'}] rep {rep}: {res[s][-1]:.4f} ms/iter, loglik[-1] {ll[-1]:.13e}, "
                  f"|W'W-I| {orth:.1e}", flush=True)
    for s in specs:
        print(f"{cfgname} [{s or 'defaults'}]: min {min(res[s]):.4f} ms/iter, median {np.median(res[s]):.4f}",
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
