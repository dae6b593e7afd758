"""Panel accumulation: sweep time against the row-chunk count (option "grid") on one config.

    python tools/chunk_sweep.py [c5|c5d] ch1 ch2 ...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def time_sweep(ctx, steps=6):
    """Average sweep-kernel time (HIP events) over `steps` device-resident EM iterations."""
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
    cfgname = sys.argv[1]
    cfg = CONFIGS[cfgname]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    if cfg.get("storage") == "f32":
        ctx.set_option("dtype", 1)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    ctx.set_option("sweep", 3)
    for ch in [0] + [int(a) for a in sys.argv[2:]]:
        ctx.set_option("grid", ch)
        ctx.em_begin(th0)
        t = time_sweep(ctx)
        print(f"{cfgname} chunks={ch or 'auto'} ({ctx.sweep_info(r)['grid']}): {t:.3f} ms", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
