"""What bounds one EM iteration at a sweep shape: the full sweep vs its DMA ring alone (ablate bit 1:
no compute) vs its compute alone (bit 2: no HBM copies), timed with HIP events around the sweep
launches, and the whole iteration (sweep + reduce + finalize) with the defaults.  Interleaved reps.

    python tools/share_floor.py [config] [reps]     (default c4s)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c4s"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    cfg = CONFIGS[cfgname]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ctx = Context(0)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    nbytes = 8 * n * (p + q)
    for rep in range(reps):
        ctx.em_begin(th0)
        ctx.em_iterate(3)
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.em_iterate(200)
        ctx.synchronize()
        it_ms = (time.perf_counter() - t0) / 200 * 1e3
        line = [f"{cfgname} rep {rep}: iteration {it_ms:.4f} ms"]
        for ab, label in ((0, "sweep"), (1, "DMA ring only"), (2, "compute only")):
            ctx.em_begin(th0)
            ctx.set_option("ablate", ab)
            ctx.em_iterate(3)
            ctx.synchronize()
            ctx.set_option("timing", 1)
            ctx.sweep_timing(reset=True)
            ctx.em_iterate(50)
            ctx.synchronize()
            ms, k = ctx.sweep_timing(reset=True)
            ctx.set_option("timing", 0)
            ctx.set_option("ablate", 0)
            line.append(f"{label} {ms / k:.4f} ms ({nbytes / (ms / k * 1e-3) / 1e12:.2f} TB/s)")
        print("; ".join(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
