"""TEST INFRASTRUCTURE (oracle) -- CPU restatement of the synthetic-data generator.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module; the product
path (ppls_amd/) never imports it.

The generator follows the simulC model of the reference (src/loglC.cpp:268-315: X = T W' + sigE E,
Y = U C' + sigF F, U = T B + H, T = N(0,1) diag(sigT)), generalised to r > 1 (the reference's
simulC breaks for r > 1, loglC.cpp:309).  The reference draws its normals from R's RNG, which is not
reproducible here; the build uses a counter-based generator instead so that the data are independent
of the shard count and reproducible on CPU and GPU:

* Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3", SC'11;
  the Random123 library's philox4x32_R with R = 10): per round
  (c0, c1, c2, c3) -> (hi(M1 c2) ^ c1 ^ k0, lo(M1 c2), hi(M0 c0) ^ c3 ^ k1, lo(M0 c0)),
  M0 = 0xD2511F53, M1 = 0xCD9E8D57, then the key is bumped by (0x9E3779B9, 0xBB67AE85).
  Pinned by the published known-answer vectors (KAT below, from Random123's kat_vectors).
* normal pair index e >> 1 of stream m under key seed: counter {pair lo, pair hi, m, 0};
  u1 = (bits53(w1:w0) + 1/2) 2^-53, u2 = (bits53(w3:w2) + 1/2) 2^-53 (the top 53 bits of each
  64-bit word pair), Box-Muller z0 = sqrt(-2 ln u1) cos(2 pi u2), z1 = ... sin(...); element e takes
  z0 for even e and z1 for odd e.
* streams: 0 = E (X noise, element index row * p + col), 1 = F (Y noise, row * q + col),
  2 = T latent (row * r + k), 3 = H latent (row * r + k).

Exactness: the Philox words and the uniforms are integer/exact arithmetic and agree bitwise with the
device; the normals go through log/cos/sin, whose last-ulp rounding differs between the device math
library and the host's, so the normals (and X, Y) agree to a few ulp, not bitwise.
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)

# Random123 kat_vectors, philox4x32 10: (counter[4], key[2]) -> result[4]
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def philox4x32_10(ctr, k0, k1):
    """ctr: (N, 4) uint32 counters; key (k0, k1) -> (N, 4) uint32."""
    c = np.asarray(ctr, dtype=np.uint32).reshape(-1, 4).astype(np.uint64)
    c0, c1, c2, c3 = c[:, 0], c[:, 1], c[:, 2], c[:, 3]
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0), p1 & MASK32,
                          (p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1), p0 & MASK32)
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return np.stack([c0, c1, c2, c3], axis=1).astype(np.uint32)


def counters(stream, pairs):
    pairs = np.asarray(pairs, dtype=np.uint64)
    ctr = np.zeros((pairs.size, 4), dtype=np.uint32)
    ctr[:, 0] = (pairs & MASK32).astype(np.uint32)
    ctr[:, 1] = (pairs >> np.uint64(32)).astype(np.uint32)
    ctr[:, 2] = stream
    return ctr


def uniforms(seed, stream, pairs):
    """The two 53-bit uniforms (u1, u2) of each pair index."""
    seed = int(seed)
    w = philox4x32_10(counters(stream, pairs), seed & 0xFFFFFFFF, seed >> 32).astype(np.uint64)
    a = ((w[:, 1] << np.uint64(32)) | w[:, 0]) >> np.uint64(11)
    b = ((w[:, 3] << np.uint64(32)) | w[:, 2]) >> np.uint64(11)
    return (a.astype(np.float64) + 0.5) * 2.0 ** -53, (b.astype(np.float64) + 0.5) * 2.0 ** -53


def normals(seed, stream, e):
    """Standard normal of element index e (array) of the stream."""
    e = np.asarray(e, dtype=np.uint64)
    u1, u2 = uniforms(seed, stream, e >> np.uint64(1))
    rad = np.sqrt(-2.0 * np.log(u1))
    ang = 6.283185307179586 * u2
    return np.where((e & np.uint64(1)) == 1, rad * np.sin(ang), rad * np.cos(ang))


def generate(row0, nrows, p, q, W, C, b, t, sigE, sigF, sigH, seed):
    """Rows [row0, row0 + nrows) of the synthetic X (nrows x p), Y (nrows x q) and latent T, U."""
    W, C = np.asarray(W, dtype=float), np.asarray(C, dtype=float)
    r = W.shape[1]
    rows = np.arange(row0, row0 + nrows, dtype=np.uint64)
    el = rows[:, None] * np.uint64(r) + np.arange(r, dtype=np.uint64)[None, :]
    T = np.asarray(t, dtype=float)[None, :] * normals(seed, 2, el.ravel()).reshape(nrows, r)
    U = T * np.asarray(b, dtype=float)[None, :] + sigH * normals(seed, 3, el.ravel()).reshape(nrows, r)

    def obs(L, M, cols, sig, stream):
        s = np.zeros((nrows, cols))
        for k in range(r):   # the device's fma order: k = 0 .. r-1
            s = s + L[:, k:k + 1] * M[:, k][None, :]
        e = rows[:, None] * np.uint64(cols) + np.arange(cols, dtype=np.uint64)[None, :]
        return s + sig * normals(seed, stream, e.ravel()).reshape(nrows, cols)

    return obs(T, W, p, sigE, 0), obs(U, C, q, sigF, 1), T, U
