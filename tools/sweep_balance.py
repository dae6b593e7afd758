"""Is the split sweep's tail (workgroups finishing their row loops at different times) a property of
the workgroup index -- i.e. of where it runs -- or noise?  Per workgroup: row-loop time over many
iterations (strace), its correlation between even and odd iterations, and the spread by b % 8 (the
XCD a workgroup lands on under round-robin dispatch).

    python tools/sweep_balance.py [config] [iterations] [balance 0|1]   (default 0: the even split)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c4s"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    bal = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    cfg = CONFIGS[cfgname]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    grid = ctx.sweep_info(r)["grid"]
    ctx.set_option("balance", bal)
    ctx.set_option("strace", 1)
    ctx.em_begin(th0)
    ctx.em_iterate(2)
    loops, ends = [], []
    for _ in range(iters):
        ctx.em_iterate(1)
        t = ctx.sweep_trace(grid)
        loops.append(t[:, 2] - t[:, 1])      # row loop (after the ring prologue)
        ends.append(t[:, 3])                 # partials written, relative to the first entry
    ctx.set_option("strace", 0)
    ctx_w = ctx.sweep_balance()
    ctx.close()
    L = np.array(loops)
    E = np.array(ends)
    mean = L.mean(axis=0)
    even, odd = L[0::2].mean(axis=0), L[1::2].mean(axis=0)
    corr = np.corrcoef(even, odd)[0, 1]
    w, _ = ctx_w
    print(f"balance {bal}: XCD-class weights {np.round(w, 4).tolist()}")
    print(f"{cfgname}: grid {grid}, {iters} iterations; row-loop us per workgroup: mean {mean.mean():.1f}, "
          f"min {mean.min():.1f}, max {mean.max():.1f}; kernel end (max over WGs) {E.max(axis=1).mean():.1f} us, "
          f"median WG end {np.median(E, axis=1).mean():.1f} us")
    print(f"  correlation of per-WG loop time, even vs odd iterations: {corr:.3f} "
          f"(near 1: the slow workgroups are the same every time)")
    print(f"  per-iteration std of loop time across WGs {L.std(axis=1).mean():.2f} us; "
          f"std of the per-WG mean {mean.std():.2f} us")
    for x in range(8):
        sel = mean[x::8]
        print(f"  b % 8 == {x}: mean {sel.mean():.1f} us, min {sel.min():.1f}, max {sel.max():.1f}")
    order = np.argsort(mean)[::-1][:12]
    print("  slowest workgroups:", ", ".join(f"{b}({mean[b]:.1f})" for b in order))


if __name__ == "__main__":
    main()
