"""Same-box A/B of the MFMA Gram's scheduling variants (context option "gram" = PPLS_GRAM_SKIP 1 |
PPLS_GRAM_DYN 2): the joint S = [X Y]'[X Y] at C3 and C5 formed by each variant in turn
(interleaved rounds, best of them), with the fp64 TF/s of the executed 128 x 128 tiles and of the
useful lower triangle n P (P + 1); then parity: X'X of every variant at one split count must equal
variant 0's bit for bit (each item's sums are the same whichever workgroup runs it), and the
statistics read off each variant's S must agree to 1e-12.

    python tools/gram_variants.py [rounds=2] [configs=c3,c5]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ppls_amd import Context  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
names = sys.argv[2].split(",") if len(sys.argv) > 2 else ["c3", "c5"]
VARIANTS = (0, 1, 2, 3)
for name in names:
    cfg = bench.CONFIGS[name]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    truth, th0 = bench.make_truth_and_theta0(p, q, r)
    with Context(0) as ctx:
        if cfg.get("storage") == "f32":
            ctx.set_option("dtype", 1)
        ctx.generate_synthetic(n, p, q, truth, seed=20261015)
        ctx.set_option("xprod", 1)
        info = ctx.xprod_info(r)
        P = int(round((info["bytes_per_pass"] / 8) ** 0.5))
        useful = float(n) * P * (P + 1)
        times = {v: [] for v in VARIANTS}
        stats = {}
        for rd in range(rounds + 1):
            for v in VARIANTS:
                ctx.set_option("gram", v)
                ctx.xprod_release()
                ms, _ = ctx.xprod_prepare()
                if rd > 0:
                    times[v].append(ms)
                if rd == rounds:
                    stats[v] = ctx.xprod_stats(th0)
        for v in VARIANTS:
            best = min(times[v])
            print(f"{name} S variant {v}: {best:8.2f} ms  executed {info['gram_flops'] / best / 1e9:6.2f} TF/s  "
                  f"useful {useful / best / 1e9:6.2f} TF/s  (all {[round(t, 2) for t in times[v]]})", flush=True)
        for v in VARIANTS[1:]:
            d = max(float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)) for a, b in zip(stats[v], stats[0]))
            print(f"{name} stats from S, variant {v} vs 0: max rel diff {d:.2e}", flush=True)
            assert d < 1e-12, (name, v, d)
        ns = 2 if P > 8000 else 12
        G = {}
        for v in VARIANTS:
            ctx.set_option("gram", v)
            G[v] = ctx.gram(0, ns, want=True)[0]
        for v in VARIANTS[1:]:
            eq = bool(np.array_equal(G[v], G[0]))
            print(f"{name} X'X nsplit {ns}, variant {v} == variant 0 bitwise: {eq}", flush=True)
            assert eq, (name, v)
        ctx.set_option("gram", 3)
