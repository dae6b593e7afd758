"""Per-component, per-step comparison of the device initialiser with the oracle on one shape
(diagnostics for a randomised-parity failure).  usage: python tools/init_case_probe.py i n p q a"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import make_problem  # noqa: E402
from oracle import ppls_oracle as o  # noqa: E402
from ppls_amd import Context  # noqa: E402

i, n, p, q, a = (int(v) for v in sys.argv[1:6])
X, Y, _ = make_problem(n, p, q, a, seed=2000 + i)
rng = np.random.default_rng(3000 + i)
inits = [o.initial_guess(p, q, "random", rng) for _ in range(a)]
for steps in (1, 2, 4, 8):
    ref = o.ppls(X, Y, a, steps, -np.inf, inits)
    for xp in (0, 1):
        with Context(0) as c:
            c.set_option("xprod", xp)
            c.set_data(X, Y)
            f = c.ppls(a, steps, -np.inf, inits)
        dW = np.abs(f["W"] - ref["W"]).max(axis=0)
        dC = np.abs(f["C"] - ref["C"]).max(axis=0)
        dl = [float(np.abs(np.asarray(f["Other_output"]["logvalue"][k]) - ref["Other_output"]["logvalue"][k]).max())
              for k in range(a)]
        dsig = np.abs(np.asarray(f["sig"]) - ref["sig"]).max(axis=1)
        print(f"steps {steps} xprod {xp}: dW {dW} dC {dC} dlogvalue {np.array(dl)} dsig {dsig}", flush=True)
