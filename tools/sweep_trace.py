"""Per-workgroup timeline of the split sweep (set_option("strace", 1)): when workgroups start, finish
their ring prologue, finish the row loop and finish writing partials, relative to the first entry.

    python tools/sweep_trace.py [config]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c4s"
    cfg = CONFIGS[cfgname]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    grid = ctx.sweep_info(r)["grid"]
    ctx.set_option("strace", 1)
    ctx.em_begin(th0)
    for it in range(4):
        ctx.em_iterate(1)
        t = ctx.sweep_trace(grid)
        q50 = lambda v: np.percentile(v, [0, 50, 100])  # noqa: E731
        print(f"{cfgname} iter {it} grid {grid}: entry {q50(t[:, 0]).round(1)} us, prologue done "
              f"{q50(t[:, 1]).round(1)}, loop done {q50(t[:, 2]).round(1)}, partials written "
              f"{q50(t[:, 3]).round(1)} (min/median/max)", flush=True)
    ctx.set_option("strace", 0)
    ctx.close()


if __name__ == "__main__":
    main()
