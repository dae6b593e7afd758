"""A/B of the finalize polar paths (option polar1: Cholesky-QR1 fast path vs Cholesky-QR2 only) at
bench configs: ms per EM iteration, interleaved repeats; timing only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def main():
    for cfgname in sys.argv[1:] or ["c5s"]:
        cfg = CONFIGS[cfgname]
        n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
        ctx = Context(0)
        if cfg.get("storage") == "f32":
            ctx.set_option("dtype", 1)
        truth, th0 = make_truth_and_theta0(p, q, r)
        ctx.generate_synthetic(n, p, q, truth, seed=20261015)
        res = {0: [], 1: []}
        for rep in range(3):
            for fast in (1, 0):
                ctx.set_option("polar1", fast)
                ctx.em_begin(th0)
                ctx.em_iterate(3)
                ctx.synchronize()
                t0 = time.perf_counter()
                ctx.em_iterate(60)
                ctx.synchronize()
                res[fast].append((time.perf_counter() - t0) / 60 * 1e3)
                _, ll = ctx.em_state()
                print(f"{cfgname} polar1={fast} rep {rep}: {res[fast][-1]:.4f} ms/iter, loglik[-1] {ll[-1]:.12e}",
                      flush=True)
        print(f"{cfgname}: polar1=1 min {min(res[1]):.4f} ms, polar1=0 min {min(res[0]):.4f} ms, "
              f"saved {min(res[0]) - min(res[1]):.4f} ms per iteration", flush=True)
        ctx.set_option("polar1", 1)
        ctx.close()


if __name__ == "__main__":
    main()
