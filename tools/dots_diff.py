"""Compare the panel dots forms (ablate bits: 8192 in-tile B, 4096 flips 32/64 rows per wave) on the
E-step's mu_T for a few fp32/fp64 shapes: python tools/dots_diff.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ppls_amd import Context, Theta  # noqa: E402
from tests.conftest import make_problem  # noqa: E402


def main():
    c = Context(0)
    c.set_option("sweep", 3)
    for dt in (1, 0):
        c.set_option("dtype", dt)
        for n, p, q, r in [(333, 37, 23, 3), (333, 700, 41, 10), (333, 130, 96, 1), (5000, 37, 23, 3),
                           (333, 64, 32, 3), (333, 33, 1, 3)]:
            X, Y, th = make_problem(n, p, q, r, seed=40 + r)
            c.set_data(X, Y)
            t = Theta(th["W"], th["C"], th["B"], th["sigE"], th["sigF"], th["sigH"], th["sigT"])
            out = {}
            for ab in (8192, 0, 4096, 4096 | 8192):
                c.set_option("ablate", ab)
                out[ab] = c.estep(t).mu_T
            ref = out[8192]
            for ab in (0, 4096, 4096 | 8192):
                d = np.abs(out[ab] - ref)
                bad = np.argwhere(d > 1e-12 * np.abs(ref).max())
                print(f"dtype {dt} n={n} p={p} q={q} r={r} ablate {ab:#x}: max diff {d.max():.3e}, "
                      f"bad rows {sorted(set(bad[:, 0].tolist()))[:12]} ({len(bad)} entries)", flush=True)
    c.close()


if __name__ == "__main__":
    main()
