"""Timing experiments on the wide-data sweeps (team single pass vs panel two passes).

    python tools/team_ablation.py [c5|c5d] [r] [--quick]

Team ablate bits (timing only; results garbage while set): 32 = no team exchange, 64 = no dots /
update arithmetic, 128 = no HBM -> LDS copies.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def time_sweep(ctx, steps=6):
    ctx.em_iterate(1)
    ctx.synchronize()
    ctx.set_option("timing", 1)
    ctx.sweep_timing(reset=True)
    ctx.em_iterate(steps)
    ctx.synchronize()
    ms, n = ctx.sweep_timing(reset=True)
    ctx.set_option("timing", 0)
    return ms / max(n, 1)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    cfgname = args[0] if args else "c5"
    cfg = dict(CONFIGS[cfgname])
    if len(args) > 1:                          # optional r override
        cfg["r"] = int(args[1])
        cfgname += f"_r{cfg['r']}"
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    if cfg.get("storage") == "f32":
        ctx.set_option("dtype", 1)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    nbytes = (4 if cfg.get("storage") == "f32" else 8) * n * (p + q)
    runs = [("panel", 3, 0), ("team", 4, 0), ("team no-xch", 4, 32), ("team no-math", 4, 64),
            ("team no-dma", 4, 128), ("team no-xch no-math", 4, 96), ("team barriers only", 4, 224)]
    if "--quick" in sys.argv:
        runs = runs[:2]
    for name, sweep, ab in runs:
        ctx.set_option("sweep", sweep)
        ctx.set_option("ablate", ab)
        ctx.em_begin(th0)
        t = time_sweep(ctx)
        print(f"{cfgname} {name:22s} ablate={ab:3d}: {t:8.3f} ms  {nbytes / t / 1e6:6.0f} GB/s "
              f"({ctx.sweep_info(r)['variant']}, grid {ctx.sweep_info(r)['grid']})", flush=True)
    ctx.set_option("ablate", 0)
    ctx.close()


if __name__ == "__main__":
    main()
