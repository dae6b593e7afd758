import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def make_problem(n, p, q, r, seed=0, sigE=0.5, sigF=0.6, sigH=0.1):
    """Small model-based problem (simulC semantics) + a perturbed theta0 -- test data only."""
    rng = np.random.default_rng(seed)

    def polar(M):
        U, _, Vt = np.linalg.svd(M, full_matrices=False)
        return U @ Vt

    W = polar(rng.standard_normal((p, r)))
    C = polar(rng.standard_normal((q, r)))
    t = np.exp(-0.1 * np.arange(r))
    b = np.exp(np.log(1.5) - 0.3 * np.arange(r))
    T = rng.standard_normal((n, r)) * t
    U = T * b + sigH * rng.standard_normal((n, r))
    X = T @ W.T + sigE * rng.standard_normal((n, p))
    Y = U @ C.T + sigF * rng.standard_normal((n, q))
    th0 = dict(W=polar(W + 0.5 * rng.standard_normal((p, r))), C=polar(C + 0.5 * rng.standard_normal((q, r))),
               B=np.diag(np.linspace(1.2, 0.7, r)), sigE=0.9, sigF=0.8, sigH=0.3,
               sigT=np.diag(np.linspace(1.1, 0.6, r)))
    return X, Y, th0


@pytest.fixture
def problem():
    return make_problem
