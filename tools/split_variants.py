"""Split-sweep variants at a bench config (rows per step, pipelining, non-temporal DMA): sweep time
from HIP events and ms per EM iteration; timing only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c4s"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    cfg = CONFIGS[cfgname]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    variants = [dict(), dict(ablate=1 | 4 | 8), dict(ablate=2 | 4 | 8)]
    for rep in range(reps):
        for v in variants:
            for k, val in v.items():
                ctx.set_option(k, val)
            ctx.em_begin(th0)
            ctx.em_iterate(3)
            ctx.synchronize()
            ctx.set_option("timing", 1)
            ctx.sweep_timing(reset=True)
            t0 = time.perf_counter()
            ctx.em_iterate(40)
            ctx.synchronize()
            dt = (time.perf_counter() - t0) / 40 * 1e3
            ctx.set_option("timing", 0)
            kms, nl = ctx.sweep_timing(reset=True)
            print(f"{cfgname} {v} [{ctx.sweep_kernel(r)}]: sweep {kms / max(nl, 1):.4f} ms, {dt:.4f} ms/iter", flush=True)
            ctx.set_option("ablate", 0)
    ctx.close()


if __name__ == "__main__":
    main()
