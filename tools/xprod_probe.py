"""Cross-product form (option "xprod") at the bench workloads: time to form S, per-iteration wall
time of em_iterate reading S, the apply kernels' HIP-event time, against the streaming sweep.

    python tools/xprod_probe.py [c3 c4s c5s c5 ...] [--steps K] [--rw N]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c3"])
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rw", type=int, default=0)
    ap.add_argument("--stream-steps", type=int, default=20)
    args = ap.parse_args()
    from ppls_amd import Context
    for key in args.configs:
        cfg = bench.CONFIGS[key]
        n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
        with Context(0) as ctx:
            if cfg.get("storage") == "f32":
                ctx.set_option("dtype", 1)
            truth, th0 = bench.make_truth_and_theta0(p, q, r)
            ctx.generate_synthetic(n, p, q, truth, seed=20261015)
            # streaming reference
            ctx.em_begin(th0)
            ctx.em_iterate(3)
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.em_iterate(args.stream_steps)
            ctx.synchronize()
            t_stream = (time.perf_counter() - t0) / args.stream_steps
            _, ll_s = ctx.em_state()
            # cross-products
            ctx.set_option("xprod", 1)
            ctx.set_option("xprod_rw", args.rw)
            gram_ms, tot_ms = ctx.xprod_prepare()
            info = ctx.xprod_info(r)
            ctx.em_begin(th0)
            ctx.em_iterate(3)
            ctx.synchronize()
            ctx.set_option("timing", 1)
            ctx.sweep_timing(reset=True)
            t0 = time.perf_counter()
            ctx.em_iterate(args.steps)
            ctx.synchronize()
            t_xp = (time.perf_counter() - t0) / args.steps
            ctx.set_option("timing", 0)
            kms, launches = ctx.sweep_timing(reset=True)
            _, ll_x = ctx.em_state()
            k = min(len(ll_s), len(ll_x))
            rel = float(np.abs(ll_x[:k] - ll_s[:k]).max() / np.abs(ll_s[:k]).max())
            apply_ms = kms / max(launches, 1)
            print(f"{key}: stream {1e3 * t_stream:.3f} ms/it ({1 / t_stream:.1f} it/s) | S: Gram {gram_ms:.1f} ms "
                  f"({info['gram_flops'] / (gram_ms * 1e-3) / 1e12:.1f} TF/s), total {tot_ms:.1f} ms | "
                  f"xprod {1e3 * t_xp:.4f} ms/it ({1 / t_xp:.0f} it/s), apply+gram kernels {1e3 * apply_ms:.1f} us "
                  f"({info['bytes_per_pass'] / (apply_ms * 1e-3) / 1e12:.2f} TB/s of S, rows={info['rows_per_wave']}) | "
                  f"break-even {tot_ms / (1e3 * (t_stream - t_xp)):.0f} iterations | loglik rel diff {rel:.1e}",
                  flush=True)


if __name__ == "__main__":
    main()
