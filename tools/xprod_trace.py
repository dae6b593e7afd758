"""Where one cross-product iteration's time goes: HIP-event time of the tile kernel,
wall time per iteration of em_iterate reading S, and the finalize's per-block phase stamps
(set_option("ftrace", 1)) right after a tile kernel.

    python tools/xprod_trace.py [config=c3] [iters=2000]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ppls_amd import Context  # noqa: E402

cfgname = sys.argv[1] if len(sys.argv) > 1 else "c3"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
cfg = bench.CONFIGS[cfgname]
n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
truth, th0 = bench.make_truth_and_theta0(p, q, r)
with Context(0) as ctx:
    if cfg.get("storage") == "f32":
        ctx.set_option("dtype", 1)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    ctx.set_option("xprod", 1)
    g, _ = ctx.xprod_prepare()
    ctx.em_begin(th0)
    ctx.em_iterate(5)
    ctx.synchronize()
    for rep in range(3):
        ctx.set_option("timing", 1)
        ctx.sweep_timing(reset=True)
        t0 = time.perf_counter()
        ctx.em_iterate(iters)
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / iters
        ctx.set_option("timing", 0)
        kms, nl = ctx.sweep_timing(reset=True)
        print(f"{cfgname} rep {rep}: {1e6 * dt:.2f} us per iteration, tile kernel {1e3 * kms / nl:.2f} us "
              f"({nl} timed), rest {1e6 * dt - 1e3 * kms / nl:.2f} us", flush=True)
    ctx.set_option("ftrace", 1)
    for it in range(4):
        ctx.em_iterate(1)
        ctx.synchronize()
        tr = ctx.finalize_trace()
        print(f"{cfgname} finalize after tile, iter {it}: " +
              "; ".join(f"block {b}: " + " ".join(f"{i}={v}" for i, v in enumerate(s) if v is not None)
                        for b, s in tr.items()), flush=True)
    ctx.set_option("ftrace", 0)
