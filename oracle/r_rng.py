"""R's default random number stream, restated in Python -- TEST INFRASTRUCTURE ONLY.

Used to regenerate the inputs of the reference's own example run (the R CMD check of
Package/PPLS.Rcheck: `PPLS-Ex.R:39-40` draws `exX`, `exY` right after `cleanEx()`, which runs
`RNGkind("default", "default"); set.seed(1)`) and the `'random'` starting values of `PPLSi`
(`Package/PPLS/R/EM_W_multi.R:133`: `orth(runif(p))`, `orth(runif(q))`, `rchisq(1,1)`,
`rchisq(2,100)/100`, `rchisq(2,10)/100`), so the oracle and the device path can be checked
against the outputs the reference printed (`PPLS.Rcheck/PPLS-Ex_x64.Rout:54-83`).

R is not in this image; these are the published algorithms R documents for its defaults
(`?RNGkind`: Mersenne-Twister, normal.kind "Inversion"; `?rgamma`, `?rexp`), restated:

* ``RRNG.set_seed``  R's `set.seed` for Mersenne-Twister: the integer seed is scrambled by 50
  rounds of the LCG ``s <- 69069 s + 1 (mod 2^32)``, then 625 further LCG outputs fill
  ``dummy[0..624]`` (``dummy[0]`` is the position ``mti``, reset to 624, so the first draw
  regenerates the whole state); ``mt = dummy[1..624]``.
* ``unif_rand``      MT19937 (Matsumoto & Nishimura 1998) genrand with tempering, times
  2.3283064365386963e-10 (2^-32), then R's fixup keeping the value inside (0, 1).
* ``norm_rand``      Inversion: ``u = floor(2^27 u1) + u2``; ``qnorm(u / 2^27)``.
* ``qnorm``          Wichura's AS241 (PPND16) rational approximations, in R's evaluation order.
* ``exp_rand``       Ahrens & Dieter (1972) algorithm SA with the q_k = sum_{j<=k} ln2^j/j! table.
* ``rgamma``         Ahrens & Dieter (1974) GS for shape < 1, Ahrens & Dieter (1982) GD for
  shape >= 1, with R's constants; ``rchisq(df) = rgamma(df/2, scale=2)``.
* ``r_scale``        R's `scale(x)`: column means and `sqrt(sum(v^2)/(n-1))` accumulated in long
  double (R's LDOUBLE), applied with `sweep`.

Pinned by R's well-known outputs (tests/test_r_rng.py): `set.seed(1); rnorm(10)`,
`set.seed(1); runif(3)`, `set.seed(123); rnorm(3)`/`runif(3)`, `set.seed(1); rexp(3)`, and
end-to-end by the reference's printed example fits (tests/test_reference_examples.py).
"""
from __future__ import annotations

import math

import numpy as np

_N, _M = 624, 397
_MATRIX_A, _UPPER, _LOWER = 0x9908B0DF, 0x80000000, 0x7FFFFFFF
_I2_32M1 = 2.328306437080797e-10          # 1/(2^32 - 1), R's fixup constant
_BIG = 134217728.0                         # 2^27, Inversion's extra-precision split

# exp_rand's table: q[k-1] = sum_{j=1..k} ln(2)^j / j!, k = 1..16 (the printed doubles)
_EXP_Q = (0.6931471805599453, 0.9333736875190459, 0.9888777961838675, 0.9984959252914960040,
          0.9998292811061389, 0.9999833164100727, 0.9999985508231994, 0.9999998906925558,
          0.9999999924734159, 0.9999999995283275, 0.9999999999728814, 0.9999999999985598,
          0.9999999999999289, 0.9999999999999968, 0.9999999999999999, 1.0000000000000000)


def qnorm(p: float) -> float:
    """qnorm(p, 0, 1, lower.tail=TRUE, log.p=FALSE) -- AS241 (Wichura 1988)."""
    if math.isnan(p) or p < 0.0 or p > 1.0:
        return math.nan
    if p == 0.0:
        return -math.inf
    if p == 1.0:
        return math.inf
    q = p - 0.5
    if abs(q) <= 0.425:                    # 0.075 <= p <= 0.925
        r = 0.180625 - q * q
        return q * (((((((r * 2509.0809287301226727 +
                          33430.575583588128105) * r + 67265.770927008700853) * r +
                        45921.953931549871457) * r + 13731.693765509461125) * r +
                      1971.5909503065514427) * r + 133.14166789178437745) * r +
                    3.387132872796366608) \
            / (((((((r * 5226.495278852545925 +
                     28729.085735721942674) * r + 39307.89580009271061) * r +
                   21213.794301586595867) * r + 5394.1960214247511077) * r +
                 687.1870074920579083) * r + 42.313330701600911252) * r + 1.0)
    r = (0.5 - p + 0.5) if q > 0 else p    # min(p, 1-p)
    r = math.sqrt(-math.log(r))
    if r <= 5.0:
        r += -1.6
        val = (((((((r * 7.7454501427834140764e-4 +
                     .0227238449892691845833) * r + .24178072517745061177) *
                   r + 1.27045825245236838258) * r +
                  3.64784832476320460504) * r + 5.7694972214606914055) *
                r + 4.6303378461565452959) * r +
               1.42343711074968357734) \
            / (((((((r * 1.05075007164441684324e-9 + 5.475938084995344946e-4) *
                    r + .0151986665636164571966) * r +
                   .14810397642748007459) * r + .68976733498510000455) *
                 r + 1.6763848301838038494) * r +
                2.05319162663775882187) * r + 1.0)
    else:
        r += -5.0
        val = (((((((r * 2.01033439929228813265e-7 +
                     2.71155556874348757815e-5) * r +
                    .0012426609473880784386) * r + .026532189526576123093) *
                  r + .29656057182850489123) * r +
                 1.7848265399172913358) * r + 5.4637849111641143699) *
               r + 6.6579046435011037772) \
            / (((((((r * 2.04426310338993978564e-15 + 1.4215117583164458887e-7) *
                    r + 1.8463183175100546818e-5) * r +
                   7.868691311456132591e-4) * r + .0148753612908506148525)
                 * r + .13692988092273580531) * r +
                .59983220655588793769) * r + 1.0)
    return -val if q < 0.0 else val


class RRNG:
    """One R session's RNG state (Mersenne-Twister / Inversion, R's defaults)."""

    def __init__(self, seed: int = 1):
        self.set_seed(seed)

    # --- set.seed / MT19937 -------------------------------------------------------------------
    def set_seed(self, seed: int) -> None:
        s = seed & 0xFFFFFFFF
        for _ in range(50):                               # initial scrambling
            s = (69069 * s + 1) & 0xFFFFFFFF
        dummy = []
        for _ in range(_N + 1):                           # n_seed = 625 for Mersenne-Twister
            s = (69069 * s + 1) & 0xFFFFFFFF
            dummy.append(s)
        self.mt = dummy[1:]
        self.mti = _N                                     # FixupSeeds(initial): dummy[0] = 624
        self._gamma_a = None

    def _regen(self) -> None:
        mt = self.mt
        for kk in range(_N):
            y = (mt[kk] & _UPPER) | (mt[(kk + 1) % _N] & _LOWER)
            mt[kk] = mt[(kk + _M) % _N] ^ (y >> 1) ^ (_MATRIX_A if y & 1 else 0)
        self.mti = 0

    def _genrand(self) -> float:
        if self.mti >= _N:
            self._regen()
        y = self.mt[self.mti]
        self.mti += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y * 2.3283064365386963e-10

    def unif_rand(self) -> float:
        x = self._genrand()
        if x <= 0.0:
            return 0.5 * _I2_32M1
        if 1.0 - x <= 0.0:
            return 1.0 - 0.5 * _I2_32M1
        return x

    # --- deviates -----------------------------------------------------------------------------
    def norm_rand(self) -> float:
        u = self.unif_rand()
        u = float(int(_BIG * u)) + self.unif_rand()
        return qnorm(u / _BIG)

    def exp_rand(self) -> float:
        a = 0.0
        u = self.unif_rand()
        while u <= 0.0 or u >= 1.0:
            u = self.unif_rand()
        while True:
            u += u
            if u > 1.0:
                break
            a += _EXP_Q[0]
        u -= 1.0
        if u <= _EXP_Q[0]:
            return a + u
        i = 0
        ustar = self.unif_rand()
        umin = ustar
        while True:
            ustar = self.unif_rand()
            if umin > ustar:
                umin = ustar
            i += 1
            if not u > _EXP_Q[i]:
                break
        return a + umin * _EXP_Q[0]

    def rgamma1(self, a: float, scale: float = 1.0) -> float:
        if a <= 0.0 or scale <= 0.0:
            return 0.0 if (scale == 0.0 or a == 0.0) else math.nan
        if a < 1.0:                                       # GS algorithm
            e = 1.0 + 0.36787944117144233 * a
            while True:
                p = e * self.unif_rand()
                if p >= 1.0:
                    x = -math.log((e - p) / a)
                    if self.exp_rand() >= (1.0 - a) * math.log(x):
                        break
                else:
                    x = math.exp(math.log(p) / a)
                    if self.exp_rand() >= x:
                        break
            return scale * x
        # GD algorithm (a >= 1)
        q1, q2, q3, q4, q5, q6, q7 = 0.04166669, 0.02083148, 0.00801191, 0.00144121, -7.388e-5, \
            2.4511e-4, 2.424e-4
        a1, a2, a3, a4, a5, a6, a7 = 0.3333333, -0.250003, 0.2000062, -0.1662921, 0.1423657, \
            -0.1367177, 0.1233795
        s2 = a - 0.5
        s = math.sqrt(s2)
        d = 5.656854 - s * 12.0
        t = self.norm_rand()
        x = s + 0.5 * t
        ret = x * x
        if t >= 0.0:                                      # immediate acceptance
            return scale * ret
        u = self.unif_rand()
        if d * u <= t * t * t:                            # squeeze acceptance
            return scale * ret
        r = 1.0 / a
        q0 = ((((((q7 * r + q6) * r + q5) * r + q4) * r + q3) * r + q2) * r + q1) * r
        if a <= 3.686:
            b = 0.463 + s + 0.178 * s2
            si = 1.235
            c = 0.195 / s - 0.079 + 0.16 * s
        elif a <= 13.022:
            b = 1.654 + 0.0076 * s2
            si = 1.68 / s + 0.275
            c = 0.062 / s + 0.024
        else:
            b = 1.77
            si = 0.75
            c = 0.1515 / s

        def quot(tt):
            v = tt / (s + s)
            if abs(v) <= 0.25:
                return q0 + 0.5 * tt * tt * ((((((a7 * v + a6) * v + a5) * v + a4) * v + a3) * v
                                              + a2) * v + a1) * v
            return q0 - s * tt + 0.25 * tt * tt + (s2 + s2) * math.log(1.0 + v)

        if x > 0.0:                                       # quotient acceptance
            q = quot(t)
            if math.log(1.0 - u) <= q:
                return scale * ret
        while True:                                       # double-exponential rejection
            e = self.exp_rand()
            u = self.unif_rand()
            u = u + u - 1.0
            t = b - si * e if u < 0.0 else b + si * e
            if t >= -0.71874483771719:
                q = quot(t)
                if q > 0.0:
                    w = math.expm1(q)
                    if c * abs(u) <= w * math.exp(e - 0.5 * t * t):
                        break
        x = s + 0.5 * t
        return scale * x * x

    # --- vector forms (R's r* functions) ------------------------------------------------------
    def runif(self, n: int, lo: float = 0.0, hi: float = 1.0) -> np.ndarray:
        return np.array([lo + (hi - lo) * self.unif_rand() for _ in range(n)])

    def rnorm(self, n: int, mean: float = 0.0, sd: float = 1.0) -> np.ndarray:
        return np.array([mean + sd * self.norm_rand() for _ in range(n)])

    def rexp(self, n: int, rate: float = 1.0) -> np.ndarray:
        return np.array([self.exp_rand() / rate for _ in range(n)])

    def rgamma(self, n: int, shape: float, scale: float = 1.0) -> np.ndarray:
        return np.array([self.rgamma1(shape, scale) for _ in range(n)])

    def rchisq(self, n: int, df: float) -> np.ndarray:
        return np.array([self.rgamma1(df / 2.0, 2.0) for _ in range(n)])

    def matrix_rnorm(self, nrow: int, ncol: int) -> np.ndarray:
        """`matrix(rnorm(nrow*ncol), nrow, ncol)`: R fills column-major."""
        return self.rnorm(nrow * ncol).reshape(ncol, nrow).T.copy()


def r_scale(x: np.ndarray) -> np.ndarray:
    """R's `scale(x)` (center = TRUE, scale = TRUE) with long-double column sums like R's C code."""
    x = np.asarray(x, dtype=np.float64)
    n = x.shape[0]
    ld = np.longdouble
    center = np.array([float(np.sum(x[:, j].astype(ld), dtype=ld) / ld(n)) for j in range(x.shape[1])])
    xc = x - center
    sd = np.array([math.sqrt(float(np.sum((xc[:, j] * xc[:, j]).astype(ld), dtype=ld)) / max(1, n - 1))
                   for j in range(x.shape[1])])
    return xc / sd


def ppls_example_data():
    """`exX`, `exY` of Package/PPLS.Rcheck/PPLS-Ex.R:39-40 after cleanEx()'s set.seed(1); returns
    (exX, exY, rng) with the RNG positioned where the example script's next draw happens."""
    rng = RRNG(1)
    exX = r_scale(rng.matrix_rnorm(100, 10))
    exY = r_scale(rng.matrix_rnorm(100, 12))
    return exX, exY, rng
