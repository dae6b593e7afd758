"""The cross-product iteration per mode of option "xprod_pipe" (0 serial tile + finalize, 1 pipelined on
CU-partitioned streams, 2 pipelined on plain streams with the finalize's at top priority): us per
iteration of em_iterate reading S, HIP-event time of the pass (1, 2) or tile (0) kernel, the
log-likelihood after the run (the modes must agree), and the CU masks HIP reports for mode 1.

    python tools/xprod_pipe_probe.py [config=c3] [iters=1000]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ppls_amd import Context  # noqa: E402

cfgname = sys.argv[1] if len(sys.argv) > 1 else "c3"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
cfg = bench.CONFIGS[cfgname]
n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
truth, th0 = bench.make_truth_and_theta0(p, q, r)
with Context(0) as ctx:
    if cfg.get("storage") == "f32":
        ctx.set_option("dtype", 1)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    ctx.set_option("xprod", 1)
    ctx.xprod_prepare()
    for rep in range(2):
        for mode in (0, 1, 2):
            ctx.set_option("xprod_pipe", mode)
            ctx.em_begin(th0)
            ctx.em_iterate(5)
            ctx.synchronize()
            ctx.set_option("timing", 1)
            ctx.sweep_timing(reset=True)
            t0 = time.perf_counter()
            ctx.em_iterate(iters)
            ctx.synchronize()
            dt = (time.perf_counter() - t0) / iters
            ctx.set_option("timing", 0)
            kms, nl = ctx.sweep_timing(reset=True)
            _, ll = ctx.em_state()
            extra = ""
            if mode == 1:
                a, b, cus = ctx.xprod_pipe_masks(12)
                extra = (f" masks: pass/apply {sum(bin(w).count('1') for w in a)} CUs {[hex(w) for w in a]}, "
                         f"finalize {sum(bin(w).count('1') for w in b)} CUs {[hex(w) for w in b]} (asked {cus})")
            print(f"{cfgname} rep {rep} mode {mode}: {1e6 * dt:.2f} us/iteration, kernel {1e3 * kms / max(nl, 1):.2f} us "
                  f"({nl} timed), loglik[-1] {ll[-1]!r}{extra}", flush=True)
