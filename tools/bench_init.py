"""Time the sequential initialiser PPLS(X, Y, a, 20, 1e-4, initialGuess) on a bench workload.

    python tools/bench_init.py [c3|c2] [--kind equal|random]

Prints one JSON line: wall time, EM steps, seconds per step (one r = 1 sweep + the device rank-1
update kernel), and the r = 1 sweep kernel time from HIP events."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context, initial_guess  # noqa: E402
import numpy as np  # noqa: E402


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "c3"
    kind = sys.argv[sys.argv.index("--kind") + 1] if "--kind" in sys.argv else "random"
    cfg = CONFIGS[cfgname]
    n, p, q, a = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    truth, _ = make_truth_and_theta0(p, q, a)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    rng = np.random.default_rng(1)
    inits = [initial_guess(p, q, kind, rng) for _ in range(a)]
    ctx.ppls(1, 1, 1e-4, inits[:1])          # warm-up (allocations, first launches)
    ctx.synchronize()
    ctx.set_option("timing", 1)
    ctx.sweep_timing(reset=True)
    t0 = time.perf_counter()
    f = ctx.ppls(a, 20, 1e-4, inits)
    dt = time.perf_counter() - t0
    ms, launches = ctx.sweep_timing(reset=True)
    ctx.set_option("timing", 0)
    steps = int(sum(f["Other_output"]["Number_steps"]))
    sweeps = steps + len(f["B"])
    out = dict(workload=cfg["name"], a=a, EMsteps=20, atol=1e-4, initialGuess=kind, seconds=dt,
               em_steps=steps, sweeps=sweeps, ms_per_sweep=1e3 * dt / sweeps,
               # launches that found the fit already ended exit at once; average over the real sweeps
               sweep_kernel_ms=ms / sweeps, sweep_launches=launches,
               sweep_TBps=8 * n * (p + q) / (ms / sweeps * 1e-3) / 1e12,
               number_steps=[int(x) for x in f["Other_output"]["Number_steps"]],
               loglikelihoods=[float(x) for x in f["Other_output"]["Loglikelihoods"]])
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
