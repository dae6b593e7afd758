"""The int8 Gram's integer arithmetic on the host (ppls_ozaki.hip's residue and CRT functions, the
same source the kernels run; no GPU): residues of x' = rint(x 2^shift) against Python integers, and
the Chinese-remainder reconstruction (Garner digits, 192-bit Horner, one rounding) against Python's
correctly rounded float(int) over the whole range (-M/2, M/2), M = the product of the moduli."""
import ctypes as ct
import math
import random

import pytest

from ppls_amd import _lib


@pytest.fixture(scope="module")
def L():
    return _lib.lib()


def _moduli(L, k):
    return [L.ppls_oz_modulus(i) for i in range(k)]


def test_moduli_pairwise_coprime(L):
    m = _moduli(L, 20)
    assert m[0] == 256 and all(2 <= v <= 256 for v in m)
    for i in range(20):
        for j in range(i):
            assert math.gcd(m[i], m[j]) == 1, (m[i], m[j])


def test_residues_of_scaled_integers(L):
    rng = random.Random(1)
    out = ct.c_int()
    for _ in range(3000):
        x = rng.uniform(-1, 1) * 2.0 ** rng.randint(-30, 30)
        e = math.frexp(x)[1] if x else 0
        shift = rng.randint(40, 62) - e   # |x'| < 2^62
        xs = round(math.ldexp(x, shift))  # rint: Python's round is round-half-even, as rint
        for l in range(20):
            assert L.ppls_oz_residue_host(x, shift, l, ct.byref(out)) == 0
            m = L.ppls_oz_modulus(l)
            r = out.value
            assert -(m // 2) <= r <= m // 2 and -128 <= r <= 127
            assert (r - xs) % m == 0, (x, shift, l, r, xs % m)


def test_residues_at_the_limb_extremes(L):
    """The fp32 residue form (five 13-bit limbs of |x'|, |t| < 2^23, one rint against 1.5 2^23): the
    largest integers (|x'| up to 2^62 - 2^10), every limb at its maximum, single limbs, both signs,
    and the rounding boundaries of t / m -- a congruent residue within [-m//2, m//2] every time."""
    out = ct.c_int()
    vals = {0, 1, 2 ** 62 - 2 ** 10, (2 ** 53 - 1) * 2 ** 9, 2 ** 52 * 1023, 8191, 8191 * 2 ** 13, 8191 * 2 ** 26,
            8191 * 2 ** 39}
    vals |= {sum(8191 << (13 * i) for i in range(k)) for k in range(1, 5)}   # all-ones limbs (< 2^53: exact)
    for m_ in (255, 253, 251, 173):
        vals |= {m_ * k + d for k in (1, 1000, 2 ** 20, 2 ** 40) for d in (m_ // 2, m_ // 2 + 1, -(m_ // 2), 0)}
    for v in sorted(vals):
        for sgn in (1, -1):
            xs = sgn * v
            x = float(xs)
            if int(x) != xs:   # (only exactly representable integers: shift 0 keeps them)
                continue
            for l in range(20):
                assert L.ppls_oz_residue_host(x, 0, l, ct.byref(out)) == 0
                m = L.ppls_oz_modulus(l)
                r = out.value
                assert -(m // 2) <= r <= m // 2 and (r - xs) % m == 0, (xs, m, r)


@pytest.mark.parametrize("nmod", [12, 16, 18, 20])
def test_crt_round_trip(L, nmod):
    m = _moduli(L, nmod)
    M = math.prod(m)
    rng = random.Random(nmod)
    arr = (ct.c_int * nmod)()
    out = ct.c_double()
    vals = [0, 1, -1, M // 2, -(M // 2) + (1 if M % 2 == 0 else 0), 2 ** 53 + 1, -(2 ** 70) - 3]
    vals += [rng.randrange(-(M // 2) + 1, M // 2) for _ in range(2000)]
    vals += [rng.randrange(-2 ** b, 2 ** b) for b in (20, 40, 53, 54, 64, 65, 96, 120) for _ in range(100)
             if 2 ** b < M // 2]
    for v in vals:
        for l in range(nmod):
            arr[l] = v % m[l]
        assert L.ppls_oz_crt_host(arr, nmod, ct.byref(out)) == 0
        assert out.value == float(v), (nmod, v, out.value, float(v))
