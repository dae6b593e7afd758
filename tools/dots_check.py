"""Panel dots: the LDS-DMA ring kernel (ablate bit 9) against the register-staged default, on the
test shapes (fp64 and fp32 storage), then sweep timing of both at C5 / C5d.

    python tools/dots_check.py [--no-time]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, d)
import numpy as np  # noqa: E402
from conftest import make_problem  # noqa: E402
from ppls_amd import Context, Theta  # noqa: E402

SHAPES = [(200, 50, 50, 2), (97, 33, 7, 1), (301, 64, 31, 5), (50, 9, 12, 8), (3, 5, 4, 2), (1, 6, 3, 1),
          (700, 1025, 3, 2), (400, 3, 1500, 3), (150, 17, 14, 10), (90, 24, 20, 16), (5000, 300, 40, 7)]


def th(d):
    return Theta(d["W"], d["C"], d["B"], d["sigE"], d["sigF"], d["sigH"], d["sigT"])


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def main():
    ctx = Context(0)
    bad = 0
    for dt in (0, 1):
        ctx.set_option("dtype", dt)
        ctx.set_option("sweep", 3)
        for (n, p, q, r) in SHAPES:
            X, Y, th0 = make_problem(n, p, q, r, seed=n + p + q + r)
            ctx.set_data(X, Y)
            ctx.set_option("ablate", 0)
            a = ctx.estep(th(th0))
            ctx.set_option("ablate", 512)
            b = ctx.estep(th(th0))
            ctx.set_option("ablate", 0)
            e = (rel(b.mu_T, a.mu_T), rel(b.mu_U, a.mu_U), rel(b.Chh, a.Chh), abs(b.Cee - a.Cee) / abs(a.Cee))
            ok = max(e) < 1e-11
            bad += not ok
            print(f"dtype={dt} n={n} p={p} q={q} r={r} errs={e} {'OK' if ok else 'BAD'}", flush=True)
    ctx.close()
    print("BAD CASES:", bad, flush=True)
    if bad or "--no-time" in sys.argv:
        return
    from bench import CONFIGS, make_truth_and_theta0
    from team_ablation import time_sweep
    for cfgname in ("c5", "c5d"):
        cfg = CONFIGS[cfgname]
        ctx = Context(0)
        if cfg.get("storage") == "f32":
            ctx.set_option("dtype", 1)
        truth, th0 = make_truth_and_theta0(cfg["p"], cfg["q"], cfg["r"])
        ctx.generate_synthetic(cfg["n"], cfg["p"], cfg["q"], truth, seed=20261015)
        ctx.set_option("sweep", 3)
        for ab in (0, 512, 0, 512):
            ctx.set_option("ablate", ab)
            ctx.em_begin(th0)
            print(f"{cfgname} ablate={ab}: sweep {time_sweep(ctx):.3f} ms", flush=True)
        ctx.set_option("ablate", 0)
        ctx.close()


if __name__ == "__main__":
    main()
