"""Fixture of the reference's own example run (R CMD check of Package/PPLS.Rcheck) -- test data.

Writes tests/golden/rcheck_ppls_ex.npz:
  * exX, exY      -- `scale(matrix(rnorm(100*10),100,10))`, `scale(matrix(rnorm(100*12),100,12))`
                     of PPLS.Rcheck/PPLS-Ex.R:39-40, drawn with R's default stream after cleanEx()'s
                     `set.seed(1)` (restated in oracle/r_rng.py);
  * random_*      -- the three `'random'` starting values the second example's PPLSi calls draw next
                     (EM_W_multi.R:133: runif(p), runif(q), rchisq(1,1), rchisq(2,100), rchisq(2,10));
  * table_*       -- the variance tables the reference printed for the four example fits
                     (PPLS-Ex_x64.Rout:54-58, :59-64, :66-73, :74-83; the i386 run prints the same),
                     transcribed as data: LV, ssq(T)/ssq(X), ssq(U)/ssq(Y), sigH^2/ssq(U), log LR,
                     #steps, last incr.

Run from the repo root: `python tests/golden/make_rcheck.py`.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.r_rng import ppls_example_data  # noqa: E402

# PPLS-Ex_x64.Rout:54-58  PPLS(X = exX, Y = exY, nr_comp = 3, EMsteps = 1e4)
TABLE_EQUAL = [[1, 0.049, 0.047, 0.023, 0.000, 729, 0],
               [2, 0.117, 0.093, 0.023, 10.631, 811, 0],
               [3, 0.197, 0.271, 0.223, -12.895, 87, 0]]
# :59-64  ... initialGuess = "random"
TABLE_RANDOM = [[1, 0.049, 0.047, 0.023, 0.000, 733, 0],
                [2, 0.117, 0.093, 0.023, 10.631, 761, 0],
                [3, 0.197, 0.271, 0.223, -12.899, 92, 0]]
# :66-73  nr_comp = 1, initialGuess = "custom", customGuess = list(W = orth(1:10), C = orth(1:12),
#          B = 0.1, sigE = 1, sigF = 1, sigH = 1, sigT = 0.1)
TABLE_CUSTOM = [[1, 0.047, 0.048, 0.017, 0, 863, 0]]
# :74-83  nr_comp = 2, constraints = list(fconstraint(list(B = 1)), fconstraint(list(sigT = 1)))
TABLE_CONSTRAINED = [[1, 0.052, 0.045, 0.027, 0.000, 667, 0],
                     [2, 0.161, 0.091, 0.026, 8.699, 862, 0]]


def main():
    exX, exY, rng = ppls_example_data()
    rw, rc, rs = [], [], []
    for _ in range(3):
        rw.append(rng.runif(10))
        rc.append(rng.runif(12))
        b = rng.rchisq(1, 1)[0]
        siglat = rng.rchisq(2, 100) / 100
        sig = rng.rchisq(2, 10) / 100
        rs.append([b, sig[0], sig[1], siglat[0], siglat[1]])    # B, sigE, sigF, sigH, sigT
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rcheck_ppls_ex.npz")
    np.savez(out, exX=exX, exY=exY, random_W=np.array(rw).T, random_C=np.array(rc).T,
             random_s=np.array(rs), table_equal=np.array(TABLE_EQUAL, dtype=float),
             table_random=np.array(TABLE_RANDOM, dtype=float),
             table_custom=np.array(TABLE_CUSTOM, dtype=float),
             table_constrained=np.array(TABLE_CONSTRAINED, dtype=float))
    print("wrote", out)


if __name__ == "__main__":
    main()
