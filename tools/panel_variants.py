"""Time the wide-p panel sweep under experiment switches (set_option("ablate", bits)).

    python tools/panel_variants.py <config> bits[@grid] [bits[@grid] ...] [--ldpad 0|1,...]

(config: a bench.py CONFIGS key; split-sweep timing ablations: 1 no compute, 2 no HBM copies,
4 skip the polar, 8 skip the scalar finalize)

For each bits value: 2 warm-up EM iterations, then 8 timed ones; prints the average sweep time
(HIP events around every sweep launch) and the EM iterations/s.  Run it under
rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("PPLS_PKG_ROOT"):   # A/B against another build of the package (a copied ppls_amd/)
    sys.path.insert(0, os.environ["PPLS_PKG_ROOT"])
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def main():
    cfgname = sys.argv[1]
    args = sys.argv[2:]
    pads = [1]
    if "--ldpad" in args:   # row padding of the data (ld_of); each value regenerates the data
        i = args.index("--ldpad")
        pads = [int(v) for v in args[i + 1].split(",")]
        del args[i:i + 2]
    specs = [(int(b.split("@")[0], 0), int(b.split("@")[1]) if "@" in b else 0) for b in args] or [(0, 0)]
    cfg = CONFIGS[cfgname]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    if cfg.get("storage") == "f32":
        ctx.set_option("dtype", 1)
    truth, th0 = make_truth_and_theta0(p, q, r)
    cur = None
    for b, g, pad in [(b, g, pad) for pad in pads for b, g in specs] * 2:   # each twice (clock drift)
        if cur != pad:
            ctx.set_option("ldpad", pad)
            ctx.generate_synthetic(n, p, q, truth, seed=20261015)
            cur = pad
        ctx.set_option("ablate", b)
        ctx.set_option("grid", g)   # panel: accumulation row chunks (0 = auto)
        ctx.em_begin(th0)
        ctx.em_iterate(2)
        ctx.synchronize()
        ctx.set_option("timing", 1)
        ctx.sweep_timing(reset=True)
        t0 = time.perf_counter()
        ctx.em_iterate(8)
        ctx.synchronize()
        dt = time.perf_counter() - t0
        ms, launches = ctx.sweep_timing(reset=True)
        ctx.set_option("timing", 0)
        try:
            _, ll = ctx.em_state()
            tail = f"loglik[-1] {ll[-1]:.10e}"
        except Exception as e:   # noqa: BLE001 (timing ablations that break the results)
            tail = f"(no valid state: {e})"
        print(f"{cfgname} ldpad={pad} ablate={b:#x} grid={g}: sweep {ms / max(launches, 1):.3f} ms, {8 / dt:.1f} it/s, {tail}",
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
