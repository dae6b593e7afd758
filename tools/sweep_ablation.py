"""Timing experiments on the sweep kernel (results are garbage while 'ablate' is set).

    python tools/sweep_ablation.py [c3|c2]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def time_sweep(ctx, steps=10):
    ctx.em_iterate(2)
    ctx.synchronize()
    ctx.set_option("timing", 1)
    ctx.sweep_timing(reset=True)
    ctx.em_iterate(steps)
    ctx.synchronize()
    ms, n = ctx.sweep_timing(reset=True)
    ctx.set_option("timing", 0)
    return ms / max(n, 1)


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c3"
    cfg = CONFIGS[cfgname]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    nbytes = 8 * n * (p + q)
    variants = [dict(threads=512, rp=1)]
    if r <= 4:
        variants.append(dict(threads=512, rp=2))
    if r <= 3:
        variants.append(dict(threads=1024, rp=1))
    for var in variants:
        for ab in (0, 1, 2, 3):
            for grid in (0,):
                ctx.set_option("threads", var["threads"])
                ctx.set_option("rows_per_step", var["rp"])
                ctx.set_option("ablate", ab)
                ctx.set_option("grid", grid)
                ctx.em_begin(th0)
                t = time_sweep(ctx)
                print(f"{cfgname} threads={var['threads']} rp={var['rp']} ablate={ab} grid={grid or 'auto'}: "
                      f"{t:.3f} ms  {nbytes / t / 1e6:.0f} GB/s", flush=True)
    ctx.set_option("ablate", 0)
    ctx.close()


if __name__ == "__main__":
    main()
