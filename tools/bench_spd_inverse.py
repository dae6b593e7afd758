"""Device time of the batched SPD inverse (ppls_linalg.hip, method 1) against rocSOLVER potrf + potri
(method 2) over p, a batch of 5 (variances at C3: p = 2000, a = 5).  Prints one line per p."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ppls_amd import Context  # noqa: E402


def main():
    ps = [int(x) for x in sys.argv[1:]] or [64, 128, 256, 512, 1024, 2000]
    a = 5
    with Context(0) as ctx:
        for p in ps:
            rng = np.random.default_rng(p)
            B = rng.standard_normal((p, p)) / np.sqrt(p)
            A0 = B @ B.T + np.eye(p)
            A = np.stack([A0 + 0.01 * z * np.eye(p) for z in range(a)])
            t1 = min(ctx.spd_inverse(A, 1)[2] for _ in range(3))
            t2 = min(ctx.spd_inverse(A, 2)[2] for _ in range(2))
            print(f"p {p:5d} x {a}: hand-written {t1:8.3f} ms   rocSOLVER {t2:8.3f} ms   "
                  f"({2 * a * p**3 / 2 / (t1 * 1e-3) / 1e12:.2f} TF/s at p^3 flops)", flush=True)


if __name__ == "__main__":
    main()
