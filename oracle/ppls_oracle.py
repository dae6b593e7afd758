"""CPU oracle for the PPLS_simult EM inner loop -- TEST INFRASTRUCTURE ONLY.

This module is a literal numpy restatement of the reference R code on the hot path. It is
the parity checker: only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline``
leg of ``bench.py`` may import it.  The product (``ppls_amd``) never calls it.

Every function cites the reference line it restates (paths relative to /root/reference):

* ``expect_m``           Package/PPLS/R/EM_W_multi.R:637-717 (closed form :668-714)
* ``expect_m_dense``     Package/PPLS/R/EM_W_multi.R:643-667 (debug=TRUE), sseXY_W :606-618
* ``maximiz_m``          Package/PPLS/R/EM_W_multi.R:729-742, tr() Package/PPLS/R/PJSC.R:1-5
* ``logl_w``             Package/PPLS/R/EM_W_multi.R:297-323
* ``loglc_fast``         Package/PPLS/src/loglC.cpp:318-338 (the ``src/`` copy; src-x64 has p, not p+q)
* ``ppls_simult``        Package/PPLS/R/EM_W_multi.R:758-807 (init :762-771 replaced by an explicit theta0,
                         or by ``ppls`` below with explicit per-component starting values)
* ``emstepc_fast``       Package/PPLS/src/loglC.cpp:340-397 (one rank-1 EM step)
* ``emstep_w``           Package/PPLS/R/EM_W_multi.R:51-73
* ``pplsi``              Package/PPLS/R/EM_W_multi.R:116-180 (one direction; fconstraint :85-92)
* ``ppls``               Package/PPLS/R/EM_W_multi.R:229-279 (sequential fit with deflation)
* ``initial_guess``      Package/PPLS/R/EM_W_multi.R:126-140 ('equal'; 'random' from an R stream,
                         oracle/r_rng.py, or numpy draws)
* ``initial_guess_o2m``  Package/PPLS/R/EM_W_multi.R:126-131 / :520-525 ('o2m'), over ``o2m_1``
* ``o2m_1``              OmicsPLS::o2m(X, Y, 1, 0, 0) (not vendored, no version pinned: DESCRIPTION
                         Imports "OmicsPLS"); the published O2PLS algorithm's n = 1, nx = ny = 0 case
* ``print_ppls``         Package/PPLS/R/EM_W_multi.R:336-354 (print.PPLS's variance table)
* ``scores_ppls``        Package/PPLS/R/EM_W_multi.R:411-420
* ``ppls_simult_to_o2m`` Package/PPLS/R/PPLS_to_o2m.R:82-140
* ``ppls_to_o2m``        Package/PPLS/R/PPLS_to_o2m.R:28-80 (literal, with the n x p products)
* ``meta_estep``         Package/PPLS/src/loglC.cpp:399-448 (one population's rank-1 E-step)
* ``meta_mstep``         Package/PPLS/src/loglC.cpp:452-474
* ``meta_emstep``        Package/PPLS/R/EM_W_multi.R:446-485 (populations = contiguous blocks :451-458)
* ``meta_pplsi``         Package/PPLS/R/EM_W_multi.R:509-589 (critfunc = identity, no sigma check)
* ``variances_ppls_simult`` Package/PPLS/R/EM_W_multi.R:830-860
* ``orth``               OmicsPLS::orth (not vendored); semantics Package/functions.R:252-260
* ``ssq``                OmicsPLS::ssq (not vendored); semantics Package/functions.R:380-385

Parity pinning: R/Rcpp/Eigen are absent from this image, so the reference cannot run here.
The restatement is pinned by the outputs the reference itself printed: the four example fits
of its R CMD check run (Package/PPLS.Rcheck/PPLS-Ex.R:39-53 -> PPLS-Ex_x64.Rout:54-83), whose
inputs and 'random' starting values are regenerated with R's default RNG (oracle/r_rng.py),
reproduce every printed step count, variance ratio and log LR (tests/test_reference_examples.py).
Also by the reference's known-answer identity checks (Package/rank_one_inverse.R:45-59,
Package/Benchmark.R:36-45) and its independent dense formulation (Expect_M(debug=TRUE)); see
tests/test_oracle.py.  ``orth`` comes from the un-vendored OmicsPLS/O2PLS; for the rank-1 fits
above any sign convention gives the same (mirrored) fit, so the wide-r ``orth`` stays
unpinned by a reference vector.

Conventions: R matrices are column-major; here X, Y are numpy arrays (n x p, n x q) and the
diagonal parameter matrices B, sigT are carried as r x r diagonal matrices exactly as in R.
"""
from __future__ import annotations

import math

import numpy as np


# ----------------------------------------------------------------------------- helpers

def tr(X):
    """tr() -- Package/PPLS/R/PJSC.R:1-5."""
    X = np.atleast_2d(np.asarray(X, dtype=np.float64))
    return float(np.sum(np.diag(X)))


def ssq(X):
    """OmicsPLS::ssq -- semantics Package/functions.R:380-385: sum(X^2)."""
    X = np.asarray(X, dtype=np.float64)
    return float(np.sum(X * X))


def orth(X, type="SVD"):
    """OmicsPLS::orth -- semantics Package/functions.R:252-260.

    type "SVD": thin SVD X = U S V' -> U V' (the polar factor; R's svd() is LAPACK dgesdd,
    numpy's svd is LAPACK gesdd as well).  type "QR": e = qr.Q(qr(X)) -- Householder QR, for which
    LINPACK dqrdc2 and LAPACK geqrf share the sign convention R[k,k] = -sign(x_kk)*||x|| -- then
    sign_e * e with the scalar sign_e = sign(crossprod(e[,1], X[,1])) (functions.R:257-259), so
    the first column points along X[,1].
    """
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    if type == "SVD":
        U, _, Vt = np.linalg.svd(X, full_matrices=False)
        return U @ Vt
    if type == "QR":
        Q, _ = np.linalg.qr(X, mode="reduced")
        return np.sign(Q[:, 0] @ X[:, 0]) * Q   # sign_e * e (functions.R:258-259; R's sign(0) = 0)
    raise ValueError("type must be 'SVD' or 'QR'")


def blockm(A, B, C):
    """blockm -- Package/PPLS/R/EM_W_multi.R:594-602."""
    return np.block([[A, B], [B.T, C]])


def sse_xy_w(W, C, B_T, sigX, sigY, sigH, sigT):
    """sseXY_W -- Package/PPLS/R/EM_W_multi.R:606-618 (the dense (p+q)^2 covariance)."""
    p = W.shape[0]
    q = C.shape[0]
    SX = (W @ sigT) @ (W @ sigT).T + sigX ** 2 * np.eye(p)
    SXY = W @ B_T @ (sigT @ sigT) @ C.T
    CBs = C @ B_T.T @ sigT
    SY = CBs @ CBs.T + (C @ C.T) * sigH ** 2 + sigY ** 2 * np.eye(q)
    return blockm(SX, SXY, SY)


def _diag(v):
    return np.diag(np.asarray(v, dtype=np.float64))


def coefficients(B, sigE, sigF, sigH, sigT):
    """Per-component Woodbury coefficients -- Expect_M closed form, EM_W_multi.R:669-686.

    B, sigT: r x r diagonal matrices (or vectors).  Returns vectors g, Kw, Kc, Kwc, c1, c2, c3.
    """
    t = np.diag(sigT) if np.ndim(sigT) == 2 else np.asarray(sigT, dtype=np.float64)
    b = np.diag(B) if np.ndim(B) == 2 else np.asarray(B, dtype=np.float64)
    g = t ** 2 * b ** 2 + sigH ** 2
    Kw = t ** 2 - t ** 4 * b ** 2 / sigF ** 2 + t ** 4 * b ** 2 * g / (sigF ** 2 * (g + sigF ** 2))
    Kc = g - t ** 4 * b ** 2 / sigE ** 2 + t ** 6 * b ** 2 / (sigE ** 2 * (t ** 2 + sigE ** 2))
    Kwc = (t ** 2 * b / (sigE ** 2 * sigF ** 2)
           - Kc * t ** 2 * b / (sigE ** 2 * sigF ** 2 * (Kc + sigF ** 2))
           - t ** 4 * b / (sigE ** 2 * sigF ** 2 * (t ** 2 + sigE ** 2))
           + Kc * t ** 4 * b / (sigE ** 2 * sigF ** 2 * (Kc + sigF ** 2) * (t ** 2 + sigE ** 2)))
    c1 = Kw / (sigE ** 2 * (Kw + sigE ** 2))
    c3 = Kc / (sigF ** 2 * (Kc + sigF ** 2))
    c2 = Kwc
    return dict(g=g, Kw=Kw, Kc=Kc, Kwc=Kwc, c1=c1, c2=c2, c3=c3)


# ----------------------------------------------------------------------------- E step

def expect_m(X, Y, W, C, B, sigE, sigF, sigH, sigT):
    """Expect_M closed form -- Package/PPLS/R/EM_W_multi.R:668-716.

    The matrix expressions are evaluated in R's left-to-right order.
    """
    X = np.asarray(X, dtype=np.float64)
    Y = np.asarray(Y, dtype=np.float64)
    W = np.asarray(W, dtype=np.float64).reshape(X.shape[1], -1)
    C = np.asarray(C, dtype=np.float64).reshape(Y.shape[1], -1)
    N, p = X.shape
    q = Y.shape[1]
    a = W.shape[1]
    B = _diag(np.diag(B) if np.ndim(B) == 2 else B)
    sigT = _diag(np.diag(sigT) if np.ndim(sigT) == 2 else sigT)
    cf = coefficients(B, sigE, sigF, sigH, sigT)
    c1 = _diag(cf["c1"])
    c2 = _diag(cf["c2"])
    c3 = _diag(cf["c3"])
    sT2 = sigT @ sigT
    sT4 = sT2 @ sT2
    B2 = B @ B
    varU = sT2 @ B2 + np.diag(np.full(a, sigH ** 2))                      # :688
    Xw = X @ W                                                            # :689
    Yc = Y @ C                                                            # :690
    mu_T = (sigE ** -2 * (Xw @ sT2) + sigF ** -2 * (Yc @ sT2 @ B) - Xw @ c1 @ sT2
            - Xw @ c2 @ sT2 @ B - Yc @ c2 @ sT2 - Yc @ c3 @ B @ sT2)       # :691-692
    mu_U = (sigE ** -2 * (Xw @ sT2 @ B) + sigF ** -2 * (Yc @ varU)
            - Xw @ c1 @ sT2 @ B - Xw @ c2 @ varU - Yc @ c2 @ sT2 @ B - Yc @ c3 @ varU)  # :693-694
    Ctt = (sT2 - sigE ** -2 * sT4 - sigF ** -2 * (sT4 @ B2) + sT4 @ c1 + 2 * (sT4 @ B @ c2)
           + sT4 @ B2 @ c3 + (mu_T.T @ mu_T) / N)                          # :696-697
    Cuu = (varU - sigE ** -2 * (sT4 @ B2) - sigF ** -2 * (varU @ varU) + sT4 @ B2 @ c1
           + 2 * (sT2 @ B @ varU @ c2) + varU @ varU @ c3 + (mu_U.T @ mu_U) / N)   # :698-699
    Cut = (sT2 @ B - sigE ** -2 * (sT4 @ B) - sigF ** -2 * (sT2 @ B @ varU) + sT4 @ B @ c1
           + sT2 @ varU @ c2 + sT4 @ B2 @ c2 + sT2 @ B @ varU @ c3 + (mu_U.T @ mu_T) / N)  # :700-701
    mu_E = X - sigE ** 2 * (Xw @ c1 @ W.T) - sigE ** 2 * (Yc @ c2 @ W.T)  # :703
    Cee = (p * sigE ** 2 - p * sigE ** 2 + sigE ** 4 * np.sum(np.diag(c1)) + ssq(mu_E) / N) / p   # :706
    mu_F = Y - sigF ** 2 * (Yc @ c3 @ C.T) - sigF ** 2 * (Xw @ c2 @ C.T)  # :708
    Cff = (q * sigF ** 2 - q * sigF ** 2 + sigF ** 4 * np.sum(np.diag(c3)) + ssq(mu_F) / N) / q   # :709
    mu_H = sigF ** -2 * sigH ** 2 * Yc - sigH ** 2 * (Xw @ c2 + Yc @ c3)  # :711
    Chh = np.diag(np.full(a, sigH ** 2 - sigH ** 4 / sigF ** 2)) + sigH ** 4 * c3 + (mu_H.T @ mu_H) / N  # :712
    I = np.eye(a)
    return dict(mu_T=mu_T, mu_U=mu_U, Ctt=np.abs(Ctt) * I, Cuu=np.abs(Cuu) * I, Cut=Cut * I,
                Cee=np.array([[Cee]]), Cff=np.array([[Cff]]), Chh=np.abs(Chh))   # :715-716


def expect_m_dense(X, Y, W, C, B, sigE, sigF, sigH, sigT):
    """Expect_M(debug=TRUE) -- Package/PPLS/R/EM_W_multi.R:643-667: dense Sigma^{-1} via solve().

    The reference's independent formulation; O(n (p+q)^2), small sizes only.
    """
    X = np.asarray(X, dtype=np.float64)
    Y = np.asarray(Y, dtype=np.float64)
    N, p = X.shape
    q = Y.shape[1]
    B = _diag(np.diag(B) if np.ndim(B) == 2 else B)
    sigT = _diag(np.diag(sigT) if np.ndim(sigT) == 2 else sigT)
    a = W.shape[1]
    sT2 = sigT @ sigT
    covT = np.vstack([W @ sT2, C @ B @ sT2])
    covU = np.vstack([W @ B @ sT2, C @ B @ B @ sT2 + sigH ** 2 * C])
    invS = np.linalg.solve(sse_xy_w(W, C, B, sigE, sigF, sigH, sigT), np.eye(p + q))
    XY = np.hstack([X, Y])
    mu_T = XY @ invS @ covT
    mu_U = XY @ invS @ covU
    sigU2 = sT2 @ B @ B + np.diag(np.full(a, sigH ** 2))
    Ctt = sT2 - covT.T @ invS @ covT + mu_T.T @ mu_T / N
    Cuu = sigU2 - covU.T @ invS @ covU + mu_U.T @ mu_U / N
    Cut = sT2 @ B - covU.T @ invS @ covT + mu_U.T @ mu_T / N
    covE = np.vstack([np.diag(np.full(p, sigE ** 2)), np.zeros((q, p))])
    mu_E = XY @ invS @ covE
    Cee = tr(np.diag(np.full(p, sigE ** 2)) - covE.T @ invS @ covE + mu_E.T @ mu_E / N) / p
    covF = np.vstack([np.zeros((p, q)), np.diag(np.full(q, sigF ** 2))])
    mu_F = XY @ invS @ covF
    Cff = tr(np.diag(np.full(q, sigF ** 2)) - covF.T @ invS @ covF + mu_F.T @ mu_F / N) / q
    covH = np.vstack([0 * W, sigH ** 2 * C])
    mu_H = XY @ invS @ covH
    Chh = np.diag(np.full(a, sigH ** 2)) - covH.T @ invS @ covH + mu_H.T @ mu_H / N
    I = np.eye(a)
    return dict(mu_T=mu_T, mu_U=mu_U, Ctt=np.abs(Ctt) * I, Cuu=np.abs(Cuu) * I, Cut=Cut * I,
                Cee=np.array([[Cee]]), Cff=np.array([[Cff]]), Chh=np.abs(Chh))


# ----------------------------------------------------------------------------- M step

def maximiz_m(fit, X, Y, type="SVD"):
    """Maximiz_M -- Package/PPLS/R/EM_W_multi.R:729-742."""
    a = fit["Ctt"].shape[0]
    I = np.eye(a)
    Ctt = fit["Ctt"]
    # B = Cut %*% solve(Ctt) * diag(1,a): Ctt is diagonal after the :715 mask, so LAPACK's
    # solve returns 1/Ctt_kk exactly rounded and the product is Cut_kk * (1/Ctt_kk).
    inv = np.linalg.solve(Ctt, I)
    return dict(
        W=orth(X.T @ fit["mu_T"], type=type),                            # :732
        C=orth(Y.T @ fit["mu_U"], type=type),                            # :733
        B=(fit["Cut"] @ inv) * I,                                        # :734
        sigE=math.sqrt(tr(fit["Cee"]) / fit["Cee"].shape[1]),            # :735
        sigF=math.sqrt(tr(fit["Cff"]) / fit["Cff"].shape[1]),            # :736
        sigH=math.sqrt(tr(fit["Chh"]) / fit["Chh"].shape[1]),            # :737
        sigT=np.sqrt(Ctt * I),                                           # :738
    )


# ----------------------------------------------------------------------------- log-likelihood

def loglc_fast(W, C, X, Y, sigX, sigY, sig2T, c1, c2, c3, Kc):
    """loglC_fast -- Package/PPLS/src/loglC.cpp:318-338 (Eigen, single-threaded)."""
    W = np.asarray(W, dtype=np.float64).reshape(X.shape[1], -1)
    C = np.asarray(C, dtype=np.float64).reshape(Y.shape[1], -1)
    sig2X = sigX * sigX
    sig2Y = sigY * sigY
    N = X.shape[0]
    p = W.shape[0]
    q = C.shape[0]
    a = W.shape[1]
    sig2T = np.asarray(sig2T, dtype=np.float64).ravel()
    Kc = np.asarray(Kc, dtype=np.float64).ravel()
    Logdiag = (np.sum(np.log(sig2X + sig2T)) + (p - a) * math.log(sig2X)
               + np.sum(np.log(sig2Y + Kc)) + (q - a) * math.log(sig2Y))      # :331
    XW = X @ W                                                                # :332
    YC = Y @ C                                                                # :333
    traceL = 1 / sig2X * float(np.sum(X * X)) + 1 / sig2Y * float(np.sum(Y * Y))   # :334
    for i in range(a):                                                        # :335
        traceL += (-c1[i] * float(XW[:, i] @ XW[:, i]) - 2 * c2[i] * float(XW[:, i] @ YC[:, i])
                   - c3[i] * float(YC[:, i] @ YC[:, i]))
    return -0.5 * N * (p + q) * math.log(2 * math.pi) - 0.5 * N * Logdiag - 0.5 * traceL   # :336


def logl_coefficients(B_T, sigX, sigY, sigH, sigT):
    """The coefficient block of logl_W -- Package/PPLS/R/EM_W_multi.R:304-320.

    Differs from Expect_M's block only in taking g = sqrt(...) and then squaring it (:312).
    """
    t = np.diag(sigT) if np.ndim(sigT) == 2 else np.atleast_1d(np.asarray(sigT, dtype=np.float64))
    b = np.diag(B_T) if np.ndim(B_T) == 2 else np.atleast_1d(np.asarray(B_T, dtype=np.float64))
    g = np.sqrt(t ** 2 * b ** 2 + sigH ** 2)
    Kw = t ** 2 - t ** 4 * b ** 2 / sigY ** 2 + t ** 4 * b ** 2 * g ** 2 / (sigY ** 2 * (g ** 2 + sigY ** 2))
    Kc = g ** 2 - t ** 4 * b ** 2 / sigX ** 2 + t ** 6 * b ** 2 / (sigX ** 2 * (t ** 2 + sigX ** 2))
    Kwc = (t ** 2 * b / (sigX ** 2 * sigY ** 2)
           - Kc * t ** 2 * b / (sigX ** 2 * sigY ** 2 * (Kc + sigY ** 2))
           - t ** 4 * b / (sigX ** 2 * sigY ** 2 * (t ** 2 + sigX ** 2))
           + Kc * t ** 4 * b / (sigX ** 2 * sigY ** 2 * (Kc + sigY ** 2) * (t ** 2 + sigX ** 2)))
    c1 = Kw / (sigX ** 2 * (Kw + sigX ** 2))
    c3 = Kc / (sigY ** 2 * (Kc + sigY ** 2))
    return dict(sig2T=t ** 2, c1=c1, c2=Kwc, c3=c3, Kc=Kc)


def logl_w(X, Y, W, C, B_T, sigX, sigY, sigH, sigT):
    """logl_W -- Package/PPLS/R/EM_W_multi.R:297-323 -> loglC_fast."""
    sigX = float(np.ravel(sigX)[0])
    sigY = float(np.ravel(sigY)[0])
    sigH = float(np.ravel(sigH)[0])
    cf = logl_coefficients(B_T, sigX, sigY, sigH, sigT)
    return loglc_fast(W, C, X, Y, sigX, sigY, cf["sig2T"], cf["c1"], cf["c2"], cf["c3"], cf["Kc"])


# ----------------------------------------------------------------------------- the loop

def canonicalize(W, C, B, sigT):
    """Sign/order canonicalisation -- EM_W_multi.R:773-778 and :794-799.

    signLoad = sign(diag(sigT B)); rotLoad = order(diag(sigT B diag(signLoad)), decreasing=TRUE)
    (R's order() is stable for ties, as is a stable argsort of the negated key).
    """
    a = W.shape[1]
    sB = np.diag(sigT) * np.diag(B)
    signLoad = np.sign(sB)
    key = np.diag(sigT @ B @ np.diag(signLoad))
    rot = np.argsort(-key, kind="stable")
    W2 = W[:, rot] @ np.diag(signLoad)
    C2 = C[:, rot] @ np.diag(signLoad)
    B2 = np.diag(np.diag(B @ np.diag(signLoad))[rot])
    T2 = np.diag(np.diag(sigT)[rot])
    return W2, C2, B2, T2


def ppls_simult(X, Y, a, EMsteps=10, atol=1e-4, type="SVD", theta0=None):
    """PPLS_simult -- Package/PPLS/R/EM_W_multi.R:758-807.

    The reference draws theta0 from a sequential PPLS(...,'random') fit with R's RNG
    (:762-771); here theta0 = dict(W, C, B, sigE, sigF, sigH, sigT) is passed explicitly and
    the rest of the function (canonicalisation :773-778, loop :780-793, final canonicalisation
    :794-799, Eout :802, return :803-806) is restated line by line.
    """
    X = np.asarray(X, dtype=np.float64)
    Y = np.asarray(Y, dtype=np.float64)
    W = np.asarray(theta0["W"], dtype=np.float64).reshape(X.shape[1], a)
    C = np.asarray(theta0["C"], dtype=np.float64).reshape(Y.shape[1], a)
    B = _diag(np.diag(theta0["B"]) if np.ndim(theta0["B"]) == 2 else np.broadcast_to(theta0["B"], (a,)))
    sigE = float(theta0["sigE"])
    sigF = float(theta0["sigF"])
    sigH = float(theta0["sigH"])
    sigT = _diag(np.diag(theta0["sigT"]) if np.ndim(theta0["sigT"]) == 2
                 else np.broadcast_to(theta0["sigT"], (a,)))
    W, C, B, sigT = canonicalize(W, C, B, sigT)                          # :773-778
    logl = []
    outp = None
    for i in range(1, EMsteps + 1):                                     # :781
        fit = expect_m(X, Y, W, C, B, sigE, sigF, sigH, sigT)
        outp = maximiz_m(fit, X, Y, type)                               # :782
        W, C, B = outp["W"], outp["C"], outp["B"]
        sigE, sigF, sigH, sigT = outp["sigE"], outp["sigF"], outp["sigH"], outp["sigT"]
        logl.append(logl_w(X, Y, W, C, B, sigE, sigF, sigH, sigT))      # :791
        if i > 1 and logl[i - 1] - logl[i - 2] < atol:                  # :792
            break
    est = dict(outp)
    est["W"], est["C"], est["B"], est["sigT"] = canonicalize(W, C, B, sigT)   # :794-799
    warn = bool(np.any(np.diff(logl) < 0))                              # :801
    Eout = expect_m(X, Y, W, C, B, sigE, sigF, sigH, sigT)              # :802 (un-canonicalised)
    return dict(Expectations=Eout, loglik=np.array(logl), estimates=est, warning_negative=warn)


# ----------------------------------------------------------------------------- sufficient statistics

def sweep_stats(X, Y, W, C, coef):
    """One-pass sufficient statistics of the build's sweep.

    Given mu_T = Xw diag(alpha) + Yc diag(beta), mu_U = Xw diag(gamma) + Yc diag(delta):
    returns S_X = X' mu_T (p x r), S_Y = Y' mu_U (q x r), G = [Xw Yc]'[Xw Yc] (2r x 2r).
    Used by the tests to check the device sweep and the sharded (gloo) reduction.
    """
    Xw = X @ W
    Yc = Y @ C
    mu_T = Xw * coef["alpha"] + Yc * coef["beta"]
    mu_U = Xw * coef["gamma"] + Yc * coef["delta"]
    Z = np.hstack([Xw, Yc])
    return dict(SX=X.T @ mu_T, SY=Y.T @ mu_U, G=Z.T @ Z, mu_T=mu_T, mu_U=mu_U)


def crossproducts(X, Y):
    """S = [X Y]'[X Y] ((p+q) x (p+q)): the cross-product form's one data pass."""
    Z = np.hstack([X, Y])
    return Z.T @ Z


def xprod_stats(S, p, W, C, coef):
    """sweep_stats from S instead of the rows: with B = blockdiag(W, C) and M = S B,
    X'mu_T = M[:p] (alpha | beta), Y'mu_U = M[p:] (gamma | delta) (EM_W_multi.R:691-694, :732-733)
    and Gram([Xw Yc]) = B' M (:696-712, loglC.cpp:334-335)."""
    r = W.shape[1]
    q = C.shape[0]
    B = np.zeros((p + q, 2 * r))
    B[:p, :r] = W
    B[p:, r:] = C
    M = S @ B
    SX = M[:p, :r] * coef["alpha"] + M[:p, r:] * coef["beta"]
    SY = M[p:, :r] * coef["gamma"] + M[p:, r:] * coef["delta"]
    return dict(SX=SX, SY=SY, G=B.T @ M)


def mu_coefficients(B, sigE, sigF, sigH, sigT):
    """alpha, beta, gamma, delta with mu_T[:,k] = alpha_k Xw_k + beta_k Yc_k and
    mu_U[:,k] = gamma_k Xw_k + delta_k Yc_k -- EM_W_multi.R:691-694 collected per column."""
    t = np.diag(sigT) if np.ndim(sigT) == 2 else np.asarray(sigT, dtype=np.float64)
    b = np.diag(B) if np.ndim(B) == 2 else np.asarray(B, dtype=np.float64)
    cf = coefficients(b, sigE, sigF, sigH, t)
    t2 = t * t
    v = t2 * b * b + sigH ** 2
    alpha = t2 / sigE ** 2 - cf["c1"] * t2 - cf["c2"] * t2 * b
    beta = t2 * b / sigF ** 2 - cf["c2"] * t2 - cf["c3"] * b * t2
    gamma = t2 * b / sigE ** 2 - cf["c1"] * t2 * b - cf["c2"] * v
    delta = v / sigF ** 2 - cf["c2"] * t2 * b - cf["c3"] * v
    return dict(alpha=alpha, beta=beta, gamma=gamma, delta=delta, **cf)


# ----------------------------------------------------------------------------- sequential init (PPLS)

def _rsqrt(v):
    """R's sqrt(): NaN (with a warning in R) for negative input."""
    with np.errstate(invalid="ignore"):
        return np.sqrt(np.asarray(v, dtype=np.float64))


def emstepc_fast(W, C, B, X, Y, sigX, sigY, sigH, sigT, c1, c2, c3):
    """EMstepC_fast -- Package/PPLS/src/loglC.cpp:340-397 (W, C vectors; scalars)."""
    sig2X, sig2Y, sig2H, sig2T = sigX * sigX, sigY * sigY, sigH * sigH, sigT * sigT
    N = X.shape[0]
    p, q = W.shape[0], C.shape[0]
    Xw = X @ W                                                                    # :353
    Yc = Y @ C
    mu_T = Xw * sig2T * (-c1 + -c2 * B + 1 / sig2X) + Yc * sig2T * (-c2 + -c3 * B + 1 / sig2Y * B)   # :356
    Cxt = X.T @ mu_T / N                                                          # :357
    Ctt = (sig2T - sig2T * sig2T * (-c1 - 2 * B * c2 - B * B * (c3 - 1 / sig2Y) + 1 / sig2X)
           + mu_T @ mu_T / N)                                                     # :358
    v = sig2T * B * B + sig2H
    mu_U = (Xw * (-sig2T * B * c1 + -c2 * v + 1 / sig2X * B * sig2T)
            + Yc * (-c2 * B * sig2T + -c3 * v + 1 / sig2Y * v))                    # :361
    Cyu = Y.T @ mu_U / N                                                          # :362
    Cuu = v - (-(c1 - 1 / sig2X) * sig2T * sig2T * B * B - 2 * sig2T * B * v * c2 - v ** 2 * (c3 - 1 / sig2Y)) \
        + mu_U @ mu_U / N                                                         # :363
    Cut = sig2T * B - (-sig2T * sig2T * B * (c1 - 1 / sig2X) - sig2T * sig2T * B * B * c2 - sig2T * v * c2
                       - v * sig2T * B * (c3 - 1 / sig2Y)) + mu_U @ mu_T / N       # :365
    xw2, yc2, xy = Xw @ Xw, Yc @ Yc, Xw @ Yc
    Ceetmp = (c1 * c1 * sig2X * sig2X * xw2 + ssq(X) + c2 * c2 * sig2X * sig2X * yc2 - 2 * c1 * sig2X * xw2
              + 2 * c1 * c2 * sig2X * sig2X * xy - 2 * c2 * sig2X * xy)           # :367-368
    Cee = sig2X - (-sig2X * sig2X * c1 + p * sig2X) / p + Ceetmp / N / p          # :369
    Cfftmp = (c3 * c3 * sig2Y * sig2Y * yc2 + ssq(Y) + c2 * c2 * sig2Y * sig2Y * xw2 - 2 * c3 * sig2Y * yc2
              + 2 * c3 * c2 * sig2Y * sig2Y * xy - 2 * c2 * sig2Y * xy)           # :371-372
    Cff = sig2Y - (-sig2Y * sig2Y * c3 + q * sig2Y) / q + Cfftmp / N / q          # :373
    mh = -c2 * sig2H * Xw - (c3 - 1 / sig2Y) * sig2H * Yc
    Chh = sig2H - (-sig2H * sig2H * (c3 - 1 / sig2Y)) + mh @ mh / N               # :375
    return dict(mu_T=mu_T, mu_U=mu_U, W=Cxt / np.linalg.norm(Cxt), C=Cyu / np.linalg.norm(Cyu),
                B=Cut / Ctt, sighat=_rsqrt(np.array([Cee, Cff])),
                siglathat=_rsqrt(np.array([Chh, Ctt])),
                Cut=Cut, Ctt=Ctt, Cuu=Cuu, Cee=Cee, Cff=Cff, Chh=Chh)            # :377-396


def emstep_w(X, Y, W, C, B_T, sigX, sigY, sigH, sigT):
    """EMstep_W -- Package/PPLS/R/EM_W_multi.R:51-73 (coefficients with g = t^2 b^2 + sigH^2)."""
    W = np.ravel(W)
    C = np.ravel(C)
    B_T, sigX, sigY, sigH, sigT = (float(np.ravel(v)[0]) for v in (B_T, sigX, sigY, sigH, sigT))
    g = sigT ** 2 * B_T ** 2 + sigH ** 2
    Kw = sigT ** 2 - sigT ** 4 * B_T ** 2 / sigY ** 2 + sigT ** 4 * B_T ** 2 * g / (sigY ** 2 * (g + sigY ** 2))
    Kc = g - sigT ** 4 * B_T ** 2 / sigX ** 2 + sigT ** 6 * B_T ** 2 / (sigX ** 2 * (sigT ** 2 + sigX ** 2))
    Kwc = (sigT ** 2 * B_T / (sigX ** 2 * sigY ** 2) - Kc * sigT ** 2 * B_T / (sigX ** 2 * sigY ** 2 * (Kc + sigY ** 2))
           - sigT ** 4 * B_T / (sigX ** 2 * sigY ** 2 * (sigT ** 2 + sigX ** 2))
           + Kc * sigT ** 4 * B_T / (sigX ** 2 * sigY ** 2 * (Kc + sigY ** 2) * (sigT ** 2 + sigX ** 2)))
    c1 = Kw / (sigX ** 2 * (Kw + sigX ** 2))
    c3 = Kc / (sigY ** 2 * (Kc + sigY ** 2))
    return emstepc_fast(W, C, B_T, X, Y, sigX, sigY, sigH, sigT, c1, Kwc, c3)


def initial_guess(p, q, kind="equal", rng=None):
    """PPLSi starting values -- EM_W_multi.R:126-140.  'equal' is deterministic; 'random' draws
    orth(runif(p)), orth(runif(q)), rchisq(1,1), rchisq(2,100)/100, rchisq(2,10)/100 in that order
    (:133) from ``rng``: an R stream (oracle/r_rng.RRNG: R's own values) or a numpy Generator."""
    if kind == "equal":
        return dict(W=np.ones(p) / math.sqrt(p), C=np.ones(q) / math.sqrt(q), B=1.0,
                    sigE=1.0 / p, sigF=1.0 / q, sigH=1.0, sigT=1.0)
    if kind == "random":
        rng = rng if rng is not None else np.random.default_rng()
        if hasattr(rng, "runif"):                       # R's stream (oracle/r_rng.RRNG), :133 order
            W, C = rng.runif(p), rng.runif(q)
            B = rng.rchisq(1, 1)[0]
            siglat = rng.rchisq(2, 100) / 100
            sig = rng.rchisq(2, 10) / 100
        else:
            W = rng.uniform(size=p)
            C = rng.uniform(size=q)
            B = rng.chisquare(1)
            siglat = rng.chisquare(100, size=2) / 100
            sig = rng.chisquare(10, size=2) / 100
        return dict(W=W / np.linalg.norm(W), C=C / np.linalg.norm(C), B=float(B), sigE=float(sig[0]),
                    sigF=float(sig[1]), sigH=float(siglat[0]), sigT=float(siglat[1]))
    raise ValueError(kind)


def o2m_1(X, Y):
    """OmicsPLS::o2m(X, Y, n = 1, nx = 0, ny = 0): the fields PPLSi reads (EM_W_multi.R:127-130).
    OmicsPLS is not vendored and its version is not pinned (DESCRIPTION Imports "OmicsPLS"); restated
    from the published O2PLS algorithm (el Bouhaddani et al.): with no orthogonal components nothing
    is filtered, the joint loadings W., C. are the first left / right singular vectors of X'Y, the
    scores Tt = X W., U = Y C., and the inner relation B_T. = (Tt'Tt)^-1 Tt'U.  (For p, q above its
    size thresholds OmicsPLS reaches the same pair by power iterations.)  The sign of the pair is
    LAPACK's (numpy's svd, the dgesdd R's svd calls; flipping both leaves B_T. and the fit's
    likelihood unchanged).  Parity unpinned: no file of the reference holds an o2m fit."""
    U_, _, Vt = np.linalg.svd(X.T @ Y, full_matrices=False)
    W, C = U_[:, 0], Vt[0]
    Tt, U = X @ W, Y @ C
    return dict(W=W, C=C, Tt=Tt, U=U, B_T=float(Tt @ U) / float(Tt @ Tt))


def initial_guess_o2m(X, Y):
    """PPLSi's 'o2m' starting values -- EM_W_multi.R:126-131 (meta_PPLSi :520-525): W., C., B_T.[1]
    of o2m(X, Y, 1, 0, 0), sig = sqrt(c((ssq(X) - ssq(Tt)) / N / p, (ssq(Y) - ssq(U)) / N / q)) and
    siglat = sqrt(c(ssq(U) - ssq(Tt B), ssq(Tt)) / N)."""
    N, p = X.shape
    q = Y.shape[1]
    sim = o2m_1(X, Y)
    B = sim["B_T"]
    Tt, U = sim["Tt"], sim["U"]
    return dict(W=sim["W"], C=sim["C"], B=B, sigE=math.sqrt((ssq(X) - ssq(Tt)) / N / p),
                sigF=math.sqrt((ssq(Y) - ssq(U)) / N / q), sigH=math.sqrt((ssq(U) - ssq(Tt * B)) / N),
                sigT=math.sqrt(ssq(Tt) / N))


def fconstraint(constraints=None):
    """fconstraint -- Package/PPLS/R/EM_W_multi.R:85-92: the 7 named constraints, None = free."""
    out = dict(W=None, C=None, B=None, sigE=None, sigF=None, sigH=None, sigT=None)
    for k, v in (constraints or {}).items():
        if k in out:
            out[k] = v
    return out


def _constrain(cs, W, C, B, sigE, sigF, sigH, sigT):
    """PPLSi's `with(constraints, if(is.numeric(.)) . else .)` -- EM_W_multi.R:141-145, :165-169."""
    if cs is None:
        return W, C, B, sigE, sigF, sigH, sigT
    f = lambda key, cur: cur if cs.get(key) is None else cs[key]   # noqa: E731
    W = np.ravel(np.asarray(f("W", W), dtype=np.float64))
    C = np.ravel(np.asarray(f("C", C), dtype=np.float64))
    return (W, C, float(np.ravel(f("B", B))[0]), float(np.ravel(f("sigE", sigE))[0]),
            float(np.ravel(f("sigF", sigF))[0]), float(np.ravel(f("sigH", sigH))[0]),
            float(np.ravel(f("sigT", sigT))[0]))


def pplsi(X, Y, EMsteps=100, atol=1e-4, theta0=None, constraints=None, critfunc=None):
    """PPLSi -- Package/PPLS/R/EM_W_multi.R:116-180; theta0 = initial_guess(...) (or a customGuess),
    constraints = fconstraint(...)-style dict (None = free), critfunc None = identity.  Returns the
    reference's list; NA fit -> W None."""
    crit = critfunc if critfunc is not None else (lambda x: x)
    W = np.ravel(np.asarray(theta0["W"], dtype=np.float64))
    C = np.ravel(np.asarray(theta0["C"], dtype=np.float64))
    B, sigE, sigF = float(theta0["B"]), float(theta0["sigE"]), float(theta0["sigF"])
    sigH, sigT = float(theta0["sigH"]), float(theta0["sigT"])
    W, C, B, sigE, sigF, sigH, sigT = _constrain(constraints, W, C, B, sigE, sigF, sigH, sigT)   # :141-145

    def ll(W, C, B, sigE, sigF, sigH, sigT):
        return logl_w(X, Y, W.reshape(-1, 1), C.reshape(-1, 1), np.array([[B]]), sigE, sigF, sigH,
                      np.array([[sigT]]))

    logvalue = [ll(W, C, B, sigE, sigF, sigH, sigT)]                               # :149
    i = 0
    for i in range(1, EMsteps + 1):                                                 # :151
        if sigE < 100 * np.finfo(float).eps or sigF < 100 * np.finfo(float).eps:   # :152-154
            return dict(W=None, C=None, B=None, sig=None, logvalue=None, Last_increment=None, Number_steps=i)
        fit = emstep_w(X, Y, W, C, B, sigE, sigF, sigH, sigT)                        # :156
        B, W, C = float(fit["B"]), fit["W"], fit["C"]
        sigE, sigF = fit["sighat"]
        sigH, sigT = fit["siglathat"]
        W, C, B, sigE, sigF, sigH, sigT = _constrain(constraints, W, C, B, sigE, sigF, sigH, sigT)  # :165-169
        logvalue.append(ll(W, C, B, sigE, sigF, sigH, sigT))                         # :172
        if crit(logvalue[i] - logvalue[i - 1]) < atol:                              # :173
            break
    last = logvalue[i] - logvalue[i - 1]                                            # :176
    return dict(W=W, C=C, B=B, sig=np.array([sigE, sigF, sigH, sigT]), logvalue=np.array(logvalue),
                Last_increment=last, Number_steps=i, not_monotone=bool(np.any(np.diff(logvalue) < 0)))


def ppls(X, Y, nr_comp=1, EMsteps=100, atol=1e-4, theta0s=None, constraints=None, critfunc=None):
    """PPLS -- Package/PPLS/R/EM_W_multi.R:229-279: nr_comp PPLSi fits on successively deflated
    X, Y (:270-271).  theta0s: one starting-value dict per component (initial_guess), or "o2m" for
    the o2m starting values of the deflated Xc, Yc that component sees (:126-131 inside PPLSi);
    constraints: one fconstraint dict per component (:230, :255) or None."""
    X = np.asarray(X, dtype=np.float64)
    Y = np.asarray(Y, dtype=np.float64)
    a = nr_comp
    p, q = X.shape[1], Y.shape[1]
    Wn, Cn = np.full((p, a), np.nan), np.full((q, a), np.nan)
    Bn, sig = np.full(a, np.nan), np.full((a, 4), np.nan)
    other = dict(Last_increment=[], Number_steps=[], Loglikelihoods=[], logvalue=[])
    Xc, Yc = X, Y
    done = 0
    for i in range(a):                                                              # :254
        th0 = initial_guess_o2m(Xc, Yc) if isinstance(theta0s[i], str) and theta0s[i] == "o2m" else theta0s[i]
        fit = pplsi(Xc, Yc, EMsteps, atol, th0, None if constraints is None else constraints[i],
                    critfunc)                                                       # :256-257
        if fit["B"] is None:                                                        # :258-263
            break
        Wn[:, i], Cn[:, i], Bn[i], sig[i] = fit["W"], fit["C"], fit["B"], fit["sig"]
        Xc = Xc - np.outer(Xc @ fit["W"], fit["W"])                                 # :270
        Yc = Yc - np.outer(Yc @ fit["C"], fit["C"])                                 # :271
        other["Last_increment"].append(fit["Last_increment"])
        other["Number_steps"].append(fit["Number_steps"])
        other["logvalue"].append(fit["logvalue"])
        other["Loglikelihoods"].append(logl_w(X, Y, Wn[:, :i + 1], Cn[:, :i + 1], np.diag(Bn[:i + 1]),
                                              sig[i, 0], sig[i, 1], sig[i, 2], np.diag(sig[:i + 1, 3])))  # :274
        done = i + 1
    return dict(W=Wn[:, :done], C=Cn[:, :done], B=Bn[:done], sig=sig[:done], Other_output=other)


def print_ppls(fit, perc=True, digits=3):
    """print.PPLS -- Package/PPLS/R/EM_W_multi.R:336-354: rows (LV, ssq(T)/ssq(X), ssq(U)/ssq(Y),
    sigH^2/ssq(U), log LR, #steps, last incr), rounded.  Note `sum(sig[1:i,4]^2*B[1:i]^2 +
    sig[i,3]^2)` adds sigH^2 once per component; `signif(last, 3)` before rounding."""
    p, q = fit["W"].shape[0], fit["C"].shape[0]
    sig, B, oo = np.asarray(fit["sig"]), np.asarray(fit["B"]), fit["Other_output"]
    dll = np.concatenate([[0.0], np.diff(np.asarray(oo["Loglikelihoods"], dtype=np.float64))])
    pc = 1.0 if perc else 0.0
    rows = []
    for i in range(sig.shape[0]):
        st = np.sum(sig[:i + 1, 3] ** 2)
        su = np.sum(sig[:i + 1, 3] ** 2 * B[:i + 1] ** 2 + sig[i, 2] ** 2)
        last = float(oo["Last_increment"][i])
        if last != 0:
            last = round(last, 2 - int(math.floor(math.log10(abs(last)))))
        rows.append([i + 1, st / (pc * (st + p * sig[i, 0] ** 2) + (1 - pc)),
                     su / (pc * (su + q * sig[i, 1] ** 2) + (1 - pc)), sig[i, 2] ** 2 / (pc * su + (1 - pc)),
                     dll[i], oo["Number_steps"][i], last])
    return np.round(np.array(rows, dtype=np.float64), digits)


def simult_theta0_from_ppls(f0):
    """PPLS_simult's use of the sequential fit -- EM_W_multi.R:764-770."""
    a = f0["W"].shape[1]
    return dict(W=f0["W"], C=f0["C"], B=np.diag(f0["B"]), sigE=f0["sig"][a - 1, 0],
                sigF=f0["sig"][a - 1, 1], sigH=f0["sig"][a - 1, 2], sigT=np.diag(f0["sig"][:, 3]))


# ----------------------------------------------------------------------------- outputs after the path

def scores_ppls(W, C, X, Y, subset=None):
    """scores.PPLS -- Package/PPLS/R/EM_W_multi.R:411-420 (subset: 1-based component indices)."""
    cols = list(range(W.shape[1])) if subset is None else [int(s) - 1 for s in np.atleast_1d(subset)]
    if len(cols) == 1:
        return np.concatenate([X @ W[:, cols[0]], Y @ C[:, cols[0]]])
    return np.vstack([X @ W[:, cols], Y @ C[:, cols]])


def ppls_to_o2m(X, Y, fit):
    """PPLS_to_o2m -- Package/PPLS/R/PPLS_to_o2m.R:28-80 (the numeric fields), literal."""
    W, C = np.asarray(fit["W"]), np.asarray(fit["C"])
    B_T = np.diag(np.ravel(fit["B"]))                                             # :33
    B_U = np.linalg.solve(B_T, np.eye(B_T.shape[0]))                               # :34
    Tt, U = X @ W, Y @ C                                                          # :35-36
    ssqX, ssqY = ssq(X), ssq(Y)                                                   # :44-45
    return dict(Tt=Tt, U=U, B_T_=B_T, B_U=B_U, H_UT=U - Tt @ B_T,
                R2Xcorr=ssq(Tt) / ssqX, R2Ycorr=ssq(U) / ssqY,                     # :47-48
                R2Xhat=ssq(U @ B_U @ W.T) / ssqX, R2Yhat=ssq(Tt @ B_T @ C.T) / ssqY,  # :51-52
                ssqX=ssqX, ssqY=ssqY, varXjoint=np.sum(Tt * Tt, axis=0), varYjoint=np.sum(U * U, axis=0))


def ppls_simult_to_o2m(X, Y, fit):
    """PPLS_simult_to_o2m -- Package/PPLS/R/PPLS_to_o2m.R:82-140 (the numeric fields)."""
    est, E = fit["estimates"], fit["Expectations"]
    W, C, B_T = est["W"], est["C"], est["B"]
    p, q, r = X.shape[1], Y.shape[1], W.shape[1]
    Tt, U = E["mu_T"], E["mu_U"]
    sT, B, sE, sF, sH = est["sigT"], est["B"], est["sigE"], est["sigF"], est["sigH"]
    R2Xcorr = ssq(sT @ sT) / (ssq(sT @ sT) + p * sE ** 2)                       # :109
    v = sT @ sT @ B @ B + np.diag(np.full(r, sH ** 2))
    R2Ycorr = ssq(v) / (ssq(v) + q * sF ** 2)                                    # :110
    R2Yhat = ssq(sT @ sT @ B) / (ssq(sT @ sT @ B @ B) + r * sH ** 2 + q * sF ** 2)   # :114
    return dict(Tt=Tt, U=U, W_=W, C_=C, B_T_=B_T, B_U=np.linalg.inv(B_T), H_UT=U - Tt @ B_T,
                R2X=R2Xcorr, R2Y=R2Ycorr, R2Xcorr=R2Xcorr, R2Ycorr=R2Ycorr, R2Yhat=R2Yhat,
                ssqX=ssq(X), ssqY=ssq(Y), varXjoint=np.sum(Tt * Tt, axis=0), varYjoint=np.sum(U * U, axis=0))


# ----------------------------------------------------------------------------- multi-population (meta_*)

def meta_estep(W, C, B, X, Y, sigX, sigY, sigH, sigT, c1, c2, c3):
    """meta_Estep -- Package/PPLS/src/loglC.cpp:399-448.  The same arithmetic as EMstepC_fast
    (:340-397) but Cxt, Cyu are returned un-normalised, with mu_T, mu_U, Vt, Vu."""
    e = emstepc_fast(W, C, B, X, Y, sigX, sigY, sigH, sigT, c1, c2, c3)
    N = X.shape[0]
    sig2X, sig2Y, sig2H, sig2T = sigX * sigX, sigY * sigY, sigH * sigH, sigT * sigT
    v = sig2T * B * B + sig2H
    return dict(Cxt=X.T @ e["mu_T"] / N, Cyu=Y.T @ e["mu_U"] / N, mu_T=e["mu_T"], mu_U=e["mu_U"],   # :416, :421
                Vt=sig2T - sig2T * sig2T * (-c1 - 2 * B * c2 - B * B * (c3 - 1 / sig2Y) + 1 / sig2X),   # :441
                Vu=v - (-(c1 - 1 / sig2X) * sig2T * sig2T * B * B - 2 * sig2T * B * v * c2
                        - v ** 2 * (c3 - 1 / sig2Y)),                                                    # :442
                Cut=e["Cut"], Ctt=e["Ctt"], Cee=e["Cee"], Cff=e["Cff"], Chh=e["Chh"])


def meta_mstep(e):
    """meta_Mstep -- Package/PPLS/src/loglC.cpp:452-474."""
    return dict(B=e["Cut"] / e["Ctt"], sighat=np.array([math.sqrt(e["Cee"]), math.sqrt(e["Cff"])]),
                siglathat=np.array([math.sqrt(e["Chh"]), math.sqrt(e["Ctt"])]), Cxt=e["Cxt"], Cyu=e["Cyu"])


def _vec_orth(v):
    """orth() of one column: v / ||v|| (Package/functions.R:252-260 semantics; OmicsPLS unpinned)."""
    return v / np.linalg.norm(v)


def meta_emstep(X, Y, W, C, pop_sizes, params):
    """meta_EMstep -- Package/PPLS/R/EM_W_multi.R:446-485.  pop_sizes = table(Ipopu) in level order;
    population j is the contiguous row block X[(1+Ni[j]):Ni[j+1], ] (:455-458).  params[j]: dict
    B_T, sigX, sigY, sigH, sigT.  Returns dict(pops=[meta_Mstep list per population], W, C)."""
    W, C = np.ravel(W), np.ravel(C)
    Ni = np.concatenate([[0], np.cumsum(pop_sizes)])
    ret = []
    for j in range(len(pop_sizes)):                                                  # :453
        Xj, Yj = X[Ni[j]:Ni[j + 1]], Y[Ni[j]:Ni[j + 1]]
        pp = params[j]
        B, sX, sY, sH, sT = (float(np.ravel(pp[k])[0]) for k in ("B_T", "sigX", "sigY", "sigH", "sigT"))
        g = sT ** 2 * B ** 2 + sH ** 2                                               # :466-474
        Kw = sT ** 2 - sT ** 4 * B ** 2 / sY ** 2 + sT ** 4 * B ** 2 * g / (sY ** 2 * (g + sY ** 2))
        Kc = g - sT ** 4 * B ** 2 / sX ** 2 + sT ** 6 * B ** 2 / (sX ** 2 * (sT ** 2 + sX ** 2))
        Kwc = (sT ** 2 * B / (sX ** 2 * sY ** 2) - Kc * sT ** 2 * B / (sX ** 2 * sY ** 2 * (Kc + sY ** 2))
               - sT ** 4 * B / (sX ** 2 * sY ** 2 * (sT ** 2 + sX ** 2))
               + Kc * sT ** 4 * B / (sX ** 2 * sY ** 2 * (Kc + sY ** 2) * (sT ** 2 + sX ** 2)))
        c1 = Kw / (sX ** 2 * (Kw + sX ** 2))
        c3 = Kc / (sY ** 2 * (Kc + sY ** 2))
        e = meta_estep(W, C, B, Xj, Yj, sX, sY, sH, sT, c1, Kwc, c3)                  # :475
        ret.append(meta_mstep(e))                                                     # :477
    sg = [float(np.sign(ret[0]["Cxt"] @ e["Cxt"])) for e in ret]
    Wn = _vec_orth(sum(s * e["Cxt"] for s, e in zip(sg, ret)))                        # :481
    Cn = _vec_orth(sum(s * e["Cyu"] for s, e in zip(sg, ret)))                        # :482
    return dict(pops=ret, W=Wn, C=Cn)


def meta_pplsi(X, Y, pop_sizes, EMsteps=100, atol=1e-4, theta0=None):
    """meta_PPLSi -- Package/PPLS/R/EM_W_multi.R:509-589 (critfunc = identity, no constraints).
    theta0: initial_guess(...)-style dict.  Returns dict(W, C, params, log = logvalue[1:i+1, ],
    logvalue = the whole trace incl. the initial row)."""
    W = np.ravel(np.asarray(theta0["W"], dtype=np.float64))
    C = np.ravel(np.asarray(theta0["C"], dtype=np.float64))
    B, sigE, sigF = float(theta0["B"]), float(theta0["sigE"]), float(theta0["sigF"])
    sigH, sigT = float(theta0["sigH"]), float(theta0["sigT"])
    K = len(pop_sizes)
    Ni = np.concatenate([[0], np.cumsum(pop_sizes)])

    def ll(Xd, Yd, W, C, pp):
        return logl_w(Xd, Yd, W.reshape(-1, 1), C.reshape(-1, 1), np.array([[pp["B_T"]]]), pp["sigX"],
                      pp["sigY"], pp["sigH"], np.array([[pp["sigT"]]]))

    params = [dict(B_T=B, sigX=sigE, sigY=sigF, sigH=sigH, sigT=sigT) for _ in range(K)]   # :545
    logvalue = [np.full(K, ll(X, Y, W, C, params[0]))]                                     # :544
    i = 0
    for i in range(1, EMsteps + 1):                                                         # :551
        fit = meta_emstep(X, Y, W, C, pop_sizes, params)                                    # :555
        params = [dict(B_T=float(e["B"]), sigX=float(e["sighat"][0]), sigY=float(e["sighat"][1]),
                       sigH=float(e["siglathat"][0]), sigT=float(e["siglathat"][1])) for e in fit["pops"]]
        W, C = fit["W"], fit["C"]                                                           # :556-570
        logvalue.append(np.array([ll(X[Ni[j]:Ni[j + 1]], Y[Ni[j]:Ni[j + 1]], W, C, params[j])
                                  for j in range(K)]))                                      # :571-573
        if np.sum(logvalue[i]) - np.sum(logvalue[i - 1]) < atol:                           # :575
            break
    lv = np.array(logvalue)
    return dict(W=W, C=C, params=params, log=lv[1:i + 1], logvalue=lv)


# ----------------------------------------------------------------------------- variances.PPLS_simult

def variances_ppls_simult(fit, data, XorY):
    """variances.PPLS_simult -- Package/PPLS/R/EM_W_multi.R:830-860 (dense, literal: the N x N
    diag(Ctt) product is written as Ctt * X'X, which is the same matrix).  fit: a ppls_simult() list.
    Note the reference uses fit$estimates$sigE for XorY = "Y" too (kept)."""
    X = np.asarray(data, dtype=np.float64)
    E = fit["Expectations"]
    mu_all = E["mu_T"] if XorY == "X" else E["mu_U"]                                  # :837
    Cm = E["Ctt"] if XorY == "X" else E["Cuu"]                                         # :836
    W = orth(X.T @ mu_all, type="SVD")                                                 # :831-832
    N, p = X.shape
    a = W.shape[1]
    sigE = float(np.ravel(fit["estimates"]["sigE"])[0])
    XtX = X.T @ X
    outp = []
    for i in range(a):                                                                 # :838
        w = W[:, [i]]
        Ctt = N * Cm[i, i]
        mu = mu_all[:, i]
        mu2 = float(mu @ mu)
        Vt = Ctt - mu2                                                                 # :842
        Cxt = (X.T @ mu)[:, None]                                                      # :843
        B_star = Ctt / sigE ** 2 * np.eye(p) / N                                       # :844
        SSt_expec = (Ctt * XtX - Cxt * (Ctt + 2 * Vt) @ w.T - w * (Ctt + 2 * Vt) @ Cxt.T
                     + w * (Ctt ** 2 + 4 * mu2 * Vt + 2 * Vt * Vt) @ w.T)               # :846-847
        SSt_expec = SSt_expec / sigE ** 4 / N                                          # :848
        d = Cxt - w * Ctt
        SSt_star = (d @ d.T) / sigE ** 4                                               # :850-851
        outp.append(dict(B_exp=B_star, SSt_exp=SSt_expec, SSt_star=SSt_star))
    varMatrix = [-np.linalg.solve(e["B_exp"] - e["SSt_exp"], np.eye(p)) for e in outp]   # :856
    seLoad = np.stack([np.sqrt(np.diag(v)) for v in varMatrix], 1)                     # :857
    return dict(components=outp, varMatrix=varMatrix, seLoad=seLoad, W=W)
