"""PPLS(X, Y, a, 20, 1e-4, initialGuess) at a bench config on resident synthetic data: wall seconds of
the whole sequential fit with 'o2m' starting values (joint Gram + host singular pairs + the device
refits of earlier components) beside 'equal' and 'random'.
    python3 tools/bench_o2m.py [c3|c5]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from ppls_amd import PPLS, Context  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    cfg = bench.CONFIGS[name]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    with Context(0) as ctx:
        if cfg.get("storage") == "f32":
            ctx.set_option("dtype", 1)
        truth, _ = bench.make_truth_and_theta0(p, q, r)
        ctx.generate_synthetic(n, p, q, truth, seed=20261015)
        for kind in ("equal", "random", "o2m", "o2m"):
            ctx.synchronize()
            t0 = time.perf_counter()
            f = PPLS(None, None, r, 20, 1e-4, kind, rng=np.random.default_rng(1), ctx=ctx)
            ctx.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps(dict(config=name, initialGuess=kind, seconds=dt, steps=[int(v) for v in f["Other_output"]["Number_steps"]],
                                  loglik_last=float(f["Other_output"]["Loglikelihoods"][-1]))), flush=True)


if __name__ == "__main__":
    main()
