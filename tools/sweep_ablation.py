"""Timing experiments on the sweep kernel variants, interleaved in one process.

    python tools/sweep_ablation.py [c3|c2] [--ablate]

'ablate' runs (timing only; results garbage while set): 1 = skip per-row compute, 2 = skip the
HBM->LDS copies, 3 = both.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def time_sweep(ctx, steps=8):
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
    do_ablate = "--ablate" in sys.argv
    cfg = CONFIGS[cfgname]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    nbytes = 8 * n * (p + q)
    variants = [dict(kernel=2, rp=0, pipe=1, grid=0)]
    for rp in (1, 2):
        for pipe in (1, 0):
            for grid in (0, 512):
                variants.append(dict(kernel=3, rp=rp, pipe=pipe, grid=grid))
    res = {}
    for rnd in range(2):
        for i, var in enumerate(variants):
            for ab in ((0, 1, 2, 3) if do_ablate and rnd == 0 else (0,)):
                ctx.set_option("kernel", var["kernel"])
                ctx.set_option("rows_per_step", var["rp"])
                ctx.set_option("pipe", var["pipe"])
                ctx.set_option("grid", var["grid"])
                ctx.set_option("ablate", ab)
                ctx.em_begin(th0)
                t = time_sweep(ctx)
                res.setdefault((i, ab), []).append(t)
    ctx.set_option("ablate", 0)
    for (i, ab), ts in sorted(res.items()):
        t = min(ts)
        print(f"{cfgname} {variants[i]} ablate={ab}: {t:.3f} ms  {nbytes / t / 1e6:.0f} GB/s", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
