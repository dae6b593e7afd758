"""The Gram that forms S at a bench config, both forms, for profiling (rocprofv3 --kernel-trace):
    python3 tools/bench_gram.py [c3|c5] [--reps N]
Prints per form: the Gram's device ms, and for the int8 form its stages and moduli."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (CONFIGS, make_truth_and_theta0)
from ppls_amd import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="c3")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--forms", default="1,0")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    with Context(0) as ctx:
        if cfg.get("storage") == "f32":
            ctx.set_option("dtype", 1)
        truth, _ = bench.make_truth_and_theta0(p, q, r)
        ctx.generate_synthetic(n, p, q, truth, seed=20261015)
        ctx.set_option("xprod", 1)
        for form in (int(v) for v in a.forms.split(",")):
            ctx.set_option("gram_int8", form)
            for rep in range(a.reps):
                ctx.xprod_release()
                ms, _ = ctx.xprod_prepare()
                gi = ctx.gram_info()
                print(json.dumps(dict(config=a.config, gram_int8=form, rep=rep, gram_ms=ms, info=gi)), flush=True)


if __name__ == "__main__":
    main()
