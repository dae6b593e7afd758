"""MFMA Gram timings of this tree's library: the joint S = [X Y]'[X Y] (xprod_prepare) at C3 and C5
and X'X alone (ppls_gram) at C3, best of reps, with the fp64 TF/s of the useful flops n P (P + 1)
(lower triangle incl. the diagonal, real columns) -- for same-box A/B of Gram kernel variants
(tools/gram_ab.sh).

    python tools/gram_probe.py [reps=3]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ppls_amd import Context  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for name in ("c3", "c5"):
    cfg = bench.CONFIGS[name]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    truth, _ = bench.make_truth_and_theta0(p, q, r)
    with Context(0) as ctx:
        if cfg.get("storage") == "f32":
            ctx.set_option("dtype", 1)
        ctx.generate_synthetic(n, p, q, truth, seed=20261015)
        ctx.set_option("xprod", 1)
        ts = []
        for _ in range(reps + 1):
            ctx.xprod_release()
            ms, _ = ctx.xprod_prepare()
            ts.append(ms)
        best = min(ts[1:])
        useful = float(n) * (p + q) * (p + q + 1.0)   # lower triangle incl. the diagonal, real columns
        print(f"{name} S: {best:8.2f} ms  useful {useful / best / 1e9:6.2f} TF/s  (all {[round(t, 2) for t in ts]})",
              flush=True)
        if name == "c3":
            g = [ctx.gram(0, 0, want=False)[1] for _ in range(reps + 1)]
            fl = float(n) * p * (p + 1.0)
            print(f"{name} X'X: {min(g[1:]):8.2f} ms  useful {fl / min(g[1:]) / 1e9:6.2f} TF/s", flush=True)
