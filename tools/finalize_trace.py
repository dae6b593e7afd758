"""Phase timeline of the finalize kernel (wall-clock stamps written by the kernel itself)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402

SLOTS = {0: "start", 1: "gram1 summed over the team", 2: "chol1+inv / serial scalars", 3: "gram2 summed",
         4: "serial r x r (chol2, Jacobi, products)", 5: "output written", 6: "chol2", 7: "T V",
         8: "Jacobi", 13: "pass-1 rows", 14: "gram1 block sum", 15: "pass-2 rows"}


def main():
    for cfgname in sys.argv[1:] or ["c3"]:
        cfg = CONFIGS[cfgname]
        n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
        ctx = Context(0)
        truth, th0 = make_truth_and_theta0(p, q, r)
        ctx.generate_synthetic(min(n, 200_000), p, q, truth, seed=20261015)
        ctx.set_option("ftrace", 1)
        ctx.set_option("polar1", int(os.environ.get("POLAR1", "1")))
        ctx.em_begin(th0)
        skip = int(os.environ.get("SKIP", "0"))   # steady state: trace after SKIP iterations
        if skip:
            ctx.em_iterate(skip)
        for it in range(skip, skip + 4):
            ctx.em_iterate(1)
            tr = ctx.finalize_trace()
            raw = tr[0][10:]
            if raw[1] and raw[2]:
                us = tr[0][5]
                what = "Jacobi sweeps" if isinstance(raw[0], int) else "team barrier 1 all arrived at (us)"
                print(f"  block 0: {what} {raw[0]}, core clock {(raw[2] - raw[1]) / (us * 1e3):.2f} GHz")
            print(f"{cfgname} polar1={os.environ.get('POLAR1', '1')} iter {it}: " + "; ".join(
                f"block {b}: " + " ".join(f"{s}={v}" for s, v in enumerate(ts) if v is not None and s not in (10, 11, 12))
                for b, ts in tr.items()), flush=True)
        ctx.set_option("ftrace", 0)
        ctx.close()


if __name__ == "__main__":
    main()
