"""Repeated int8 Gram formations on one context (allocation churn probe): per call the wall time, the
HIP-event phases and the SYRK kernel time, so slow calls can be told apart (allocation vs kernel)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
which = int(sys.argv[3]) if len(sys.argv) > 3 else 0
with Context(0) as ctx:
    truth, _ = make_truth_and_theta0(cfg["p"], cfg["q"], cfg["r"])
    ctx.generate_synthetic(cfg["n"], cfg["p"], cfg["q"], truth, seed=20261015)
    ctx.set_option("gram_int8", 1)
    for k in range(reps):
        t0 = time.perf_counter()
        _, info = ctx.gram_int8(which, want=False)
        print(json.dumps(dict(rep=k, wall_ms=1e3 * (time.perf_counter() - t0), ms=info["ms"])), flush=True)
