"""variances.PPLS_simult at a BASELINE shape: MFMA Gram X'X rate and the whole call.

    python tools/bench_variances.py [--config c3|c2|c5] [--reps 3] [--no-full]

Data: the bench's synthetic simulC model generated on the device; the fit is a short device
PPLS_simult run (its Expectations feed variances).  Prints one JSON line: Gram kernel time and
fp64 MFMA TFLOP/s (executed tile flops and the useful n p (p + 1) SYRK flops) against the 78.6 TF
fp64 matrix peak, and the wall time of the whole variances call (Cxt pass, Gram, per-component
p x p build + inverse + copies), after one untimed call, for the hand-written Cholesky inverse
(var_chol 1), rocSOLVER's potrf/potri (2) and its LU (0) in turn.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import CONFIGS, FP64_PEAK_TF, make_truth_and_theta0  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--nsplit", type=int, default=0)
    ap.add_argument("--em-steps", type=int, default=3)
    ap.add_argument("--no-full", action="store_true", help="skip the whole variances call")
    ap.add_argument("--chol", type=int, default=1, help="the arm variances_s reports: 1 Cholesky (default), 2 rocSOLVER Cholesky, 0 LU")
    ap.add_argument("--full-reps", type=int, default=3, help="timed whole calls per arm after one warm-up")
    ap.add_argument("--gram-int8", type=int, default=0, help="1: X'X by the int8 CRT form (option gram_int8)")
    args = ap.parse_args()
    from ppls_amd import Context
    cfg = CONFIGS[args.config]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    if cfg.get("storage") == "f32":
        ctx.set_option("dtype", 1)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    ctx.gram(0, args.nsplit, want=False)   # warm-up (code object load, allocations)
    times = [ctx.gram(0, args.nsplit, want=False)[1] for _ in range(args.reps)]
    ms = float(np.median(times))
    nb = (p + 127) // 128
    tiles = nb * (nb + 1) // 2
    exec_flops = 2.0 * n * tiles * 128 * 128
    useful = float(n) * p * (p + 1)
    out = dict(config=cfg["name"], gram_kernel_ms=ms, gram_kernel_ms_all=times,
               gram_exec_tflops=exec_flops / ms / 1e9, gram_useful_tflops=useful / ms / 1e9,
               fp64_mfma_peak_tflops=FP64_PEAK_TF, mfma_frac=exec_flops / ms / 1e9 / FP64_PEAK_TF,
               tiles=tiles)
    if args.gram_int8:
        ctx.set_option("gram_int8", 1)
        ctx.gram_int8(0, want=False)
        infos = [ctx.gram_int8(0, want=False)[1] for _ in range(args.reps)]
        out["gram_int8"] = dict(total_ms=[i["ms"][3] for i in infos], syrk_ms=[i["ms"][1] for i in infos],
                                nmod=infos[0]["nmod"], L=infos[0]["L"])
    if not args.no_full:
        est, ll, eout, _ = ctx.em_run(th0, args.em_steps, -np.inf, 0, want_eout=True, want_mu=True)
        arms = {"chol": 1, "chol_rocsolver": 2, "lu": 0}
        secs = {k: [] for k in arms}
        for rep in range(args.full_reps + 1):   # rep 0: warm-up (rocSOLVER/rocBLAS code objects, handle)
            for k, v in arms.items():
                ctx.set_option("var_chol", v)
                t0 = time.perf_counter()
                W, Bx, V, se, _, _ = ctx.variances(eout.mu_T, eout.Ctt, est.sigE, 0, full=False)
                if rep:
                    secs[k].append(time.perf_counter() - t0)
                out[f"seLoad_median_{k}"] = float(np.median(se))
                out[f"seLoad_finite_{k}"] = bool(np.all(np.isfinite(se)))
        ctx.set_option("var_chol", args.chol)
        for k in arms:
            out[f"variances_s_{k}"] = secs[k]
        out["variances_s"] = float(np.median(secs[{1: "chol", 2: "chol_rocsolver", 0: "lu"}[args.chol]]))
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
