"""Panel sweep variants on the C5 shape (timing only): MFMA dots (default) vs tiled VALU dots, VALU
accumulation (default) vs MFMA accumulation.  (A row-per-lane VALU dots form, removed in round 1,
measured 13.1 ms fp64 / 6.7 ms fp32 per dots pass: profiles/r1_c5_*_dots_variants.txt.)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c5"
    cfg = CONFIGS[cfgname]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    if "--f32" in sys.argv:
        ctx.set_option("dtype", 1)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    ctx.set_option("sweep", 3)
    ctx.em_begin(th0)
    for rep in range(2):
        for ab, name in ((0, "mfma dots + valu acc"), (128, "mfma dots + mfma acc"), (32, "tiled dots + valu acc")):
            ctx.set_option("ablate", ab)
            ctx.em_iterate(1)
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.em_iterate(4)
            ctx.synchronize()
            dt = (time.perf_counter() - t0) / 4
            print(f"{cfgname} {name}: {dt * 1e3:.3f} ms per iteration", flush=True)
    ctx.set_option("ablate", 0)
    ctx.close()


if __name__ == "__main__":
    main()
