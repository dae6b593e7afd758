"""Driver for rocprofv3 --pmc passes over the split sweep: c4s (or argv[1]) data, `ablate` bits from
argv[2] (0 full kernel, 2 compute only: no HBM copies), 6 EM iterations.  Timing/counters only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4s"]
ab = int(sys.argv[2]) if len(sys.argv) > 2 else 0
ctx = Context(0)
truth, th0 = make_truth_and_theta0(cfg["p"], cfg["q"], cfg["r"])
ctx.generate_synthetic(cfg["n"], cfg["p"], cfg["q"], truth, seed=20261015)
ctx.set_option("ablate", ab)
ctx.em_begin(th0)
ctx.em_iterate(6)
ctx.synchronize()
ctx.close()
print("done", ab)
