"""Debug: one int8-Gram entry on the device against exact integer arithmetic (tests/test_gpu_ozaki.py
case n=127, p=40, q=9, Y block, entry (5, 7))."""
import math
import sys
from fractions import Fraction

import numpy as np

sys.path.insert(0, "tests")
from conftest import make_problem  # noqa: E402
from ppls_amd import Context  # noqa: E402

X, Y, _ = make_problem(127, 40, 9, 1, seed=127 + 40)
with Context(0) as c:
    c.set_data(X, Y)
    G, info = c.gram_int8(1)
print(info)
L = info["L"]
D = Y
e = [math.frexp(np.abs(D[:, k]).max())[1] for k in range(D.shape[1])]
worst = 0
for i in range(D.shape[1]):
    for j in range(D.shape[1]):
        xi = [round(Fraction(float(a)) * 2 ** (L - e[i])) for a in D[:, i]]
        xj = [round(Fraction(float(a)) * 2 ** (L - e[j])) for a in D[:, j]]
        Z = sum(a * b for a, b in zip(xi, xj))
        r = float(Fraction(Z) * Fraction(2) ** (e[i] + e[j] - 2 * L))
        if r != G[i, j]:
            worst += 1
            print(i, j, "device", G[i, j].hex(), "exact-int", r.hex(), "Z bits", Z.bit_length(), "Z", Z)
print("entries differing from the correctly rounded integer sum:", worst)
