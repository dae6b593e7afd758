"""Per-iteration overhead breakdown (finalize roles, reduction) at a bench config; timing only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c3"
    cfg = CONFIGS[cfgname]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    for ab in (0, 1 | 2, 1 | 2 | 4, 1 | 2 | 8, 1 | 2 | 4 | 8):
        ctx.set_option("ablate", ab)
        ctx.em_begin(th0)
        ctx.em_iterate(3)
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.em_iterate(50)
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / 50
        print(f"{cfgname} ablate={ab:2d}: {dt * 1e3:.4f} ms per iteration", flush=True)
    ctx.set_option("ablate", 0)
    ctx.close()


if __name__ == "__main__":
    main()
