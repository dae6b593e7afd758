"""ctypes binding of libppls_amd.so (include/ppls.h).

The native library is the product: if it is missing this module raises at import time --
there is no Python or CPU fallback for the hot path.
"""
from __future__ import annotations

import ctypes as ct
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libppls_amd.so")

PPLS_OK = 0
PPLS_ORTH_SVD = 0
PPLS_ORTH_QR = 1
PPLS_LAYOUT_COLMAJOR = 0
PPLS_LAYOUT_ROWMAJOR = 1

_dp = ct.POINTER(ct.c_double)


class PplsTheta(ct.Structure):
    _fields_ = [("W", _dp), ("C", _dp), ("B", _dp), ("sigT", _dp),
                ("sigE", ct.c_double), ("sigF", ct.c_double), ("sigH", ct.c_double)]


class PplsExpect(ct.Structure):
    _fields_ = [("mu_T", _dp), ("mu_U", _dp), ("Ctt", _dp), ("Cuu", _dp), ("Cut", _dp),
                ("Cee", ct.c_double), ("Cff", ct.c_double), ("Chh", _dp)]


class PplsSeqFit(ct.Structure):
    _fields_ = [("W", _dp), ("C", _dp), ("B", _dp), ("sig", _dp), ("logvalue", _dp),
                ("last_increment", _dp), ("number_steps", ct.POINTER(ct.c_int)),
                ("loglikelihoods", _dp), ("ncomp", ct.c_int), ("not_monotone", ct.c_int)]


class PplsConstraint(ct.Structure):
    _fields_ = [("W", _dp), ("C", _dp), ("B", _dp), ("sigE", _dp), ("sigF", _dp), ("sigH", _dp),
                ("sigT", _dp)]


class PplsMetaFit(ct.Structure):
    _fields_ = [("W", _dp), ("C", _dp), ("params", _dp), ("log", _dp), ("steps", ct.c_int)]


_i64p = ct.POINTER(ct.c_int64)

# typedef int (*ppls_reduce_fn)(void* user, double* buf, int64_t count)
REDUCE_FN = ct.CFUNCTYPE(ct.c_int, ct.c_void_p, _dp, ct.c_int64)

# name -> (restype, argtypes); every symbol declared in include/ppls.h
SIGNATURES = {
    "ppls_version": (ct.c_int, []),
    "ppls_strerror": (ct.c_char_p, [ct.c_int]),
    "ppls_ctx_create": (ct.c_int, [ct.c_int, ct.POINTER(ct.c_void_p)]),
    "ppls_ctx_destroy": (None, [ct.c_void_p]),
    "ppls_last_error": (ct.c_char_p, [ct.c_void_p]),
    "ppls_set_option": (ct.c_int, [ct.c_void_p, ct.c_char_p, ct.c_int64]),
    "ppls_shard_range": (None, [ct.c_int64, ct.c_int, ct.c_int, ct.POINTER(ct.c_int64),
                                ct.POINTER(ct.c_int64)]),
    "ppls_comm_unique_id": (ct.c_int, [ct.c_char_p]),
    "ppls_comm_init": (ct.c_int, [ct.c_void_p, ct.c_int, ct.c_int, ct.c_char_p]),
    "ppls_set_reducer": (ct.c_int, [ct.c_void_p, ct.c_void_p, ct.c_void_p]),
    "ppls_set_data": (ct.c_int, [ct.c_void_p, _dp, _dp, ct.c_int64, ct.c_int, ct.c_int, ct.c_int,
                                 ct.c_int64]),
    "ppls_generate_synthetic": (ct.c_int, [ct.c_void_p, ct.c_int64, ct.c_int64, ct.c_int64, ct.c_int,
                                           ct.c_int, ct.c_int, ct.POINTER(PplsTheta), ct.c_uint64]),
    "ppls_get_data": (ct.c_int, [ct.c_void_p, _dp, _dp, ct.c_int64, ct.c_int64]),
    "ppls_get_data_rows": (ct.c_int, [ct.c_void_p, _dp, _dp, ct.c_int64, ct.c_int64]),
    "ppls_philox4x32_10": (ct.c_int, [ct.c_void_p, ct.POINTER(ct.c_uint32), ct.c_int64, ct.c_uint64,
                                      ct.POINTER(ct.c_uint32)]),
    "ppls_data_ssq": (ct.c_int, [ct.c_void_p, _dp, _dp]),
    "ppls_estep": (ct.c_int, [ct.c_void_p, ct.POINTER(PplsTheta), ct.c_int, ct.POINTER(PplsExpect)]),
    "ppls_mstep": (ct.c_int, [ct.c_void_p, ct.POINTER(PplsExpect), ct.c_int, ct.c_int,
                              ct.POINTER(PplsTheta)]),
    "ppls_em_step": (ct.c_int, [ct.c_void_p, ct.POINTER(PplsTheta), ct.c_int, ct.c_int,
                                ct.POINTER(PplsTheta), ct.POINTER(PplsExpect)]),
    "ppls_loglik": (ct.c_int, [ct.c_void_p, ct.POINTER(PplsTheta), ct.c_int, _dp]),
    "ppls_em_run": (ct.c_int, [ct.c_void_p, ct.POINTER(PplsTheta), ct.c_int, ct.c_int, ct.c_double,
                               ct.c_int, _dp, ct.POINTER(ct.c_int), ct.POINTER(ct.c_int),
                               ct.POINTER(PplsExpect)]),
    "ppls_loglC_fast": (ct.c_int, [ct.c_void_p, _dp, _dp, _dp, _dp, ct.c_int64, ct.c_int, ct.c_int,
                                   ct.c_int, ct.c_double, ct.c_double, _dp, _dp, _dp, _dp, _dp, _dp]),
    "ppls_em_begin": (ct.c_int, [ct.c_void_p, ct.POINTER(PplsTheta), ct.c_int]),
    "ppls_em_iterate": (ct.c_int, [ct.c_void_p, ct.c_int, ct.c_int]),
    "ppls_em_state": (ct.c_int, [ct.c_void_p, ct.POINTER(PplsTheta), _dp, ct.c_int, ct.POINTER(ct.c_int)]),
    "ppls_synchronize": (ct.c_int, [ct.c_void_p]),
    "ppls_scores": (ct.c_int, [ct.c_void_p, _dp, _dp, ct.c_int, _dp, _dp]),
    "ppls_ppls": (ct.c_int, [ct.c_void_p, ct.c_int, ct.c_int, ct.c_double, ct.POINTER(PplsTheta),
                             ct.POINTER(PplsSeqFit)]),
    "ppls_ppls_ex": (ct.c_int, [ct.c_void_p, ct.c_int, ct.c_int, ct.c_double, ct.c_int, ct.POINTER(PplsTheta),
                                ct.POINTER(PplsConstraint), ct.POINTER(PplsSeqFit)]),
    "ppls_meta_emstep": (ct.c_int, [ct.c_void_p, ct.c_int, _i64p, _i64p, _dp, _dp, _dp, _dp, _dp, _dp,
                                    _dp, _dp]),
    "ppls_meta_ppls": (ct.c_int, [ct.c_void_p, ct.c_int, _i64p, _i64p, ct.c_int, ct.c_double, ct.c_int,
                                  ct.POINTER(PplsTheta), ct.POINTER(PplsMetaFit)]),
    "ppls_variances": (ct.c_int, [ct.c_void_p, _dp, _dp, ct.c_double, ct.c_int, ct.c_int, _dp, _dp, _dp, _dp,
                                  _dp, _dp]),
    "ppls_gram": (ct.c_int, [ct.c_void_p, ct.c_int, ct.c_int, _dp, _dp]),
    "ppls_spd_inverse": (ct.c_int, [ct.c_void_p, _dp, ct.c_int, ct.c_int, ct.c_int, _dp, ct.POINTER(ct.c_int), _dp]),
    "ppls_xprod_prepare": (ct.c_int, [ct.c_void_p, _dp, _dp]),
    "ppls_xprod_release": (ct.c_int, [ct.c_void_p]),
    "ppls_xprod_setup_times": (ct.c_int, [ct.c_void_p, _dp, _dp, _dp]),
    "ppls_xprod_tile_timing": (ct.c_int, [ct.c_void_p, ct.c_int, _dp]),
    "ppls_xprod_stats": (ct.c_int, [ct.c_void_p, ct.POINTER(PplsTheta), ct.c_int, _dp]),
    "ppls_xprod_info": (ct.c_int, [ct.c_void_p, ct.c_int, ct.POINTER(ct.c_int), ct.POINTER(ct.c_int64), _dp,
                                   ct.POINTER(ct.c_int)]),
    "ppls_sweep_timing": (ct.c_int, [ct.c_void_p, _dp, ct.POINTER(ct.c_int64), ct.c_int]),
    "ppls_sweep_balance": (ct.c_int, [ct.c_void_p, _dp, ct.POINTER(ct.c_int64), ct.c_int, ct.POINTER(ct.c_int)]),
    "ppls_comm_info": (ct.c_int, [ct.c_void_p, ct.POINTER(ct.c_int), ct.POINTER(ct.c_int), _dp,
                                  ct.POINTER(ct.c_int64), ct.c_int]),
    "ppls_finalize_trace": (ct.c_int, [ct.c_void_p, ct.POINTER(ct.c_int64), _dp]),
    "ppls_sweep_trace": (ct.c_int, [ct.c_void_p, ct.POINTER(ct.c_int64), ct.c_int, ct.POINTER(ct.c_int), _dp]),
    "ppls_sweep_info": (ct.c_int, [ct.c_void_p, ct.c_int, ct.POINTER(ct.c_int64), ct.POINTER(ct.c_int),
                                   ct.POINTER(ct.c_int)]),
    "ppls_sweep_kernel": (ct.c_int, [ct.c_void_p, ct.c_int, ct.c_char_p, ct.c_int]),
    "ppls_meta_info": (ct.c_int, [ct.c_void_p, ct.POINTER(ct.c_int)]),
    "ppls_gram_int8": (ct.c_int, [ct.c_void_p, ct.c_int, _dp, ct.POINTER(ct.c_int), ct.POINTER(ct.c_int), _dp]),
    "ppls_oz_residue_host": (ct.c_int, [ct.c_double, ct.c_int, ct.c_int, ct.POINTER(ct.c_int)]),
    "ppls_oz_crt_host": (ct.c_int, [ct.POINTER(ct.c_int), ct.c_int, _dp]),
    "ppls_oz_modulus": (ct.c_int, [ct.c_int]),
    "ppls_gram_info": (ct.c_int, [ct.c_void_p, ct.POINTER(ct.c_int), ct.POINTER(ct.c_int), ct.POINTER(ct.c_int),
                                  _dp]),
    "ppls_gram_shifts": (ct.c_int, [ct.c_void_p, ct.POINTER(ct.c_int), ct.c_int, ct.POINTER(ct.c_int)]),
    "ppls_finalize_host": (ct.c_int, [_dp, _dp, _dp, ct.c_double, ct.c_double, ct.c_double, ct.c_int,
                                      ct.c_int, ct.c_int, ct.POINTER(PplsTheta), ct.c_int,
                                      ct.POINTER(PplsTheta), ct.POINTER(PplsExpect), _dp]),
    "ppls_mu_coefficients": (ct.c_int, [ct.POINTER(PplsTheta), ct.c_int, _dp]),
}


def load(path: str = LIB_PATH) -> ct.CDLL:
    if not os.path.exists(path):
        raise ImportError(
            f"libppls_amd.so not found at {path}: build it with `python -m ppls_amd.build` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback for the PPLS hot path.")
    lib = ct.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_LIB = None


def lib() -> ct.CDLL:
    global _LIB
    if _LIB is None:
        _LIB = load()
    return _LIB


class PplsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"PPLS error {code}: {msg}")
        self.code = code


def dptr(a: np.ndarray):
    if a is None:
        return None
    assert a.dtype == np.float64 and (a.flags.c_contiguous or a.flags.f_contiguous)
    return a.ctypes.data_as(_dp)


class Theta:
    """Host-side theta in the reference's column-major convention (owned numpy buffers)."""

    def __init__(self, W, C, B, sigE, sigF, sigH, sigT):
        self.W = np.asfortranarray(np.array(W, dtype=np.float64, ndmin=2))
        self.C = np.asfortranarray(np.array(C, dtype=np.float64, ndmin=2))
        r = self.W.shape[1]
        self.B = np.ascontiguousarray(np.diag(B) if np.ndim(B) == 2 else np.broadcast_to(B, (r,)),
                                      dtype=np.float64).copy()
        self.sigT = np.ascontiguousarray(np.diag(sigT) if np.ndim(sigT) == 2
                                         else np.broadcast_to(sigT, (r,)), dtype=np.float64).copy()
        self.sigE = float(np.ravel(sigE)[0])
        self.sigF = float(np.ravel(sigF)[0])
        self.sigH = float(np.ravel(sigH)[0])

    @property
    def r(self):
        return self.W.shape[1]

    def struct(self) -> PplsTheta:
        return PplsTheta(dptr(self.W), dptr(self.C), dptr(self.B), dptr(self.sigT),
                         self.sigE, self.sigF, self.sigH)

    def pull(self, s: PplsTheta):
        self.sigE, self.sigF, self.sigH = s.sigE, s.sigF, s.sigH

    @classmethod
    def empty(cls, p, q, r):
        return cls(np.zeros((p, r)), np.zeros((q, r)), np.zeros(r), 1.0, 1.0, 1.0, np.zeros(r))

    def as_dict(self):
        r = self.r
        return dict(W=self.W.copy(), C=self.C.copy(), B=np.diag(self.B), sigE=self.sigE,
                    sigF=self.sigF, sigH=self.sigH, sigT=np.diag(self.sigT))


class Expect:
    """Host buffers for Expect_M's return list."""

    def __init__(self, r, n_local=0, want_mu=False):
        self.r = r
        self.mu_T = np.zeros((n_local, r), order="F") if want_mu else None
        self.mu_U = np.zeros((n_local, r), order="F") if want_mu else None
        self.Ctt = np.zeros(r)
        self.Cuu = np.zeros(r)
        self.Cut = np.zeros(r)
        self.Chh = np.zeros((r, r), order="F")
        self.Cee = 0.0
        self.Cff = 0.0

    def struct(self) -> PplsExpect:
        return PplsExpect(dptr(self.mu_T), dptr(self.mu_U), dptr(self.Ctt), dptr(self.Cuu),
                          dptr(self.Cut), self.Cee, self.Cff, dptr(self.Chh))

    def pull(self, s: PplsExpect):
        self.Cee, self.Cff = s.Cee, s.Cff

    def as_dict(self):
        """The reference's list (EM_W_multi.R:715-716): Ctt, Cuu, Cut as diagonal r x r."""
        return dict(mu_T=self.mu_T, mu_U=self.mu_U, Ctt=np.diag(self.Ctt), Cuu=np.diag(self.Cuu),
                    Cut=np.diag(self.Cut), Cee=np.array([[self.Cee]]), Cff=np.array([[self.Cff]]),
                    Chh=np.array(self.Chh))
