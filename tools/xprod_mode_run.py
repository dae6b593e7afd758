"""One cross-product em_iterate run at a config with option xprod_pipe = mode (for a kernel trace).

    python tools/xprod_mode_run.py <config> <mode> [iters=200]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ppls_amd import Context  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1]]
mode = int(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 200
truth, th0 = bench.make_truth_and_theta0(cfg["p"], cfg["q"], cfg["r"])
with Context(0) as ctx:
    if cfg.get("storage") == "f32":
        ctx.set_option("dtype", 1)
    ctx.generate_synthetic(cfg["n"], cfg["p"], cfg["q"], truth, seed=20261015)
    ctx.set_option("xprod", 1)
    ctx.set_option("xprod_pipe", mode)
    ctx.em_begin(th0)
    ctx.em_iterate(iters)
    ctx.synchronize()
    print("done", mode, flush=True)
