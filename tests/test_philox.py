"""CPU: the generator's restatement (oracle/philox.py) is pinned by Philox4x32-10's published
known-answer vectors, and its normals/moments behave as the simulC model says."""
import numpy as np

from oracle import philox as ph


def test_philox_known_answer_vectors():
    for c, k, r in ph.KAT:
        out = ph.philox4x32_10(np.array(c, dtype=np.uint32), *k)
        assert tuple(int(x) for x in out[0]) == r


def test_uniforms_in_open_unit_interval_and_normals_standard():
    u1, u2 = ph.uniforms(20261015, 0, np.arange(200_000, dtype=np.uint64))
    assert u1.min() > 0 and u1.max() < 1 and u2.min() > 0 and u2.max() < 1
    z = ph.normals(20261015, 0, np.arange(400_000, dtype=np.uint64))
    assert abs(z.mean()) < 0.01 and abs(z.var() - 1) < 0.01
    # different streams are different sequences
    assert not np.allclose(z[:100], ph.normals(20261015, 1, np.arange(100, dtype=np.uint64)))


def test_generate_model_moments():
    rng = np.random.default_rng(0)
    p, q, r = 20, 15, 2
    W = np.linalg.qr(rng.standard_normal((p, r)))[0]
    C = np.linalg.qr(rng.standard_normal((q, r)))[0]
    X, Y, T, U = ph.generate(0, 40_000, p, q, W, C, [1.5, 1.2], [1.0, 0.8], 0.5, 0.4, 0.1, 3)
    # Cov(X) = W diag(t^2) W' + sigE^2 I, Cov(U, T) = diag(b t^2)
    SX = X.T @ X / X.shape[0]
    assert np.abs(SX - (W * [1.0, 0.64]) @ W.T - 0.25 * np.eye(p)).max() < 0.05
    assert np.abs(np.mean(U * T, axis=0) - np.array([1.5, 1.2 * 0.64])).max() < 0.05
    # row-range invariance (counter-based)
    X2, _, _, _ = ph.generate(100, 50, p, q, W, C, [1.5, 1.2], [1.0, 0.8], 0.5, 0.4, 0.1, 3)
    assert np.array_equal(X2, X[100:150])
