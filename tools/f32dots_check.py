"""A full C5 fit (n = 5e5, p = 1e4, q = 500, r = 10, fp32 storage; bench.py's truth and theta0, 3
EM iterations, streaming panel sweep) with this tree's library: estimates and log-likelihood trace to
gpurun_out/f32dots_<arm>.npz, for comparing an experiment build (tools/f32dots_variant.py) with the
product's fp64 arithmetic.

    python tools/f32dots_check.py <arm>       (run from the tree whose library is compared)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
from ppls_amd import Context  # noqa: E402

arm = sys.argv[1]
cfg = bench.CONFIGS["c5"]
n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
truth, th0 = bench.make_truth_and_theta0(p, q, r)
with Context(0) as ctx:
    ctx.set_option("dtype", 1)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015)
    est, ll, eout, _ = ctx.em_run(th0, 3, -np.inf, 0)
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.getcwd()), "gpurun_out", f"f32dots_{arm}.npz")
    np.savez(out, W=est.W, C=est.C, B=est.B, sigT=est.sigT, sig=[est.sigE, est.sigF, est.sigH], ll=ll,
             mu_T=eout.mu_T[:20000])
    print(arm, "loglik", ll.tolist(), "->", out)
