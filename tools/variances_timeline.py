"""Timeline of one variances.PPLS_simult call at a bench config (C3 by default): run under
rocprofv3 --kernel-trace --memory-copy-trace; three calls separated by idle gaps, the last analysed
with tools/call_timeline.py --analyze <dir>.  Prints each call's wall time."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_truth_and_theta0  # noqa: E402
from ppls_amd import Context  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
ctx = Context(0)
if cfg.get("storage") == "f32":
    ctx.set_option("dtype", 1)
truth, th0 = make_truth_and_theta0(cfg["p"], cfg["q"], cfg["r"])
ctx.generate_synthetic(cfg["n"], cfg["p"], cfg["q"], truth, seed=20261015)
est, ll, eout, _ = ctx.em_run(th0, 3, -np.inf, 0, want_eout=True, want_mu=True)
secs = []
for rep in range(3):
    ctx.synchronize()
    time.sleep(0.06)
    t0 = time.perf_counter()
    ctx.variances(eout.mu_T, eout.Ctt, est.sigE, 0, full=False)
    ctx.synchronize()
    secs.append(time.perf_counter() - t0)
print(json.dumps(dict(config=cfg["name"], variances_seconds=secs)), flush=True)
ctx.close()
