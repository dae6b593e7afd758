"""Diagnostic: statistics from S by the lower-triangle kernel (option xprod_kernel 3) against the
row-tile kernel (2), per block of the output -- the script that located the reduce-scatter pad race
(DESIGN.md §12).  python tools/dbg_tri.py"""
import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from conftest import make_problem
from oracle import ppls_oracle as o
from ppls_amd import Context, Theta
for (n,p,q,r) in [(200,24,18,3),(300,50,50,2),(400,300,131,5)]:
    X, Y, th0 = make_problem(n, p, q, r, seed=1)
    th = Theta(th0["W"], th0["C"], th0["B"], th0["sigE"], th0["sigF"], th0["sigH"], th0["sigT"])
    with Context(0) as c:
        c.set_data(X, Y)
        res = {}
        for k in (2, 3):
            c.set_option("xprod_kernel", k)
            res[k] = c.xprod_stats(th)
    for name, a, b in zip(("SX","SY","G"), res[3], res[2]):
        d = np.abs(a - b)
        bad = np.argwhere(d > 1e-9 * np.abs(b).max())
        print((n,p,q,r), name, "maxrel", d.max() / np.abs(b).max(), "bad idx", bad[:12].tolist(), len(bad))
