"""A/B of the finalize polar team size (option team_rows: rows of X'mu per team member) at bench
configs: ms per EM iteration, interleaved repeats; timing only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def main():
    rows = [int(v) for v in os.environ.get("TEAM_ROWS", "1024,2048,4096").split(",")]
    for cfgname in sys.argv[1:] or ["c4s"]:
        cfg = CONFIGS[cfgname]
        n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
        ctx = Context(0)
        if cfg.get("storage") == "f32":
            ctx.set_option("dtype", 1)
        truth, th0 = make_truth_and_theta0(p, q, r)
        ctx.generate_synthetic(n, p, q, truth, seed=20261015)
        res = {k: [] for k in rows}
        for rep in range(3):
            for tr in rows:
                ctx.set_option("team_rows", tr)
                ctx.em_begin(th0)
                ctx.em_iterate(3)
                ctx.synchronize()
                t0 = time.perf_counter()
                ctx.em_iterate(60)
                ctx.synchronize()
                res[tr].append((time.perf_counter() - t0) / 60 * 1e3)
        print(cfgname + ": " + ", ".join(f"team_rows={k}: min {min(v):.4f} ms/iter" for k, v in res.items()), flush=True)
        ctx.set_option("team_rows", 0)
        ctx.close()


if __name__ == "__main__":
    main()
