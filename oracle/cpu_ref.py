"""ctypes wrapper of oracle/libcpu_ref.so -- TEST INFRASTRUCTURE ONLY (CPU baseline / oracle)."""
import ctypes as ct
import os
import subprocess

import numpy as np

import hashlib

HERE = os.path.dirname(os.path.abspath(__file__))
_dp = ct.POINTER(ct.c_double)


def _cpu_tag():
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln for ln in f if ln.startswith("model name")), "unknown")
    except OSError:
        model = "unknown"
    return hashlib.sha1(model.encode()).hexdigest()[:10]


def lib_path():
    return os.path.join(HERE, "_build", f"libcpu_ref_{_cpu_tag()}.so")


def build():
    out = lib_path()
    os.makedirs(os.path.dirname(out), exist_ok=True)
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(os.path.join(HERE, "cpu_ref.c")):
        subprocess.run(["make", "-s", "-C", HERE, f"OUT={out}"], check=True)
    return out


def load():
    lib = ct.CDLL(build())
    lib.cpu_ref_em_step.restype = ct.c_int
    lib.cpu_ref_em_step.argtypes = [_dp, _dp, ct.c_int64, ct.c_int, ct.c_int, ct.c_int, _dp, _dp, _dp, _dp,
                                    _dp, _dp, ct.c_int]
    lib.cpu_ref_max_threads.restype = ct.c_int
    return lib


def em_steps(X, Y, theta, steps, nthreads=0):
    """Run `steps` EM iterations on row-major X, Y; returns (theta dict, loglik array)."""
    lib = load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    n, p = X.shape
    q = Y.shape[1]
    W = np.asfortranarray(theta["W"], dtype=np.float64).copy(order="F")
    C = np.asfortranarray(theta["C"], dtype=np.float64).copy(order="F")
    r = W.shape[1]
    b = np.array(np.diag(theta["B"]) if np.ndim(theta["B"]) == 2 else theta["B"], dtype=np.float64)
    t = np.array(np.diag(theta["sigT"]) if np.ndim(theta["sigT"]) == 2 else theta["sigT"], dtype=np.float64)
    sig = np.array([theta["sigE"], theta["sigF"], theta["sigH"]], dtype=np.float64)
    ll = np.zeros(steps)
    P = lambda a: a.ctypes.data_as(_dp)  # noqa: E731
    for s in range(steps):
        out = ct.c_double()
        rc = lib.cpu_ref_em_step(P(X), P(Y), n, p, q, r, P(W), P(C), P(b), P(t), P(sig), ct.byref(out), nthreads)
        if rc != 0:
            raise RuntimeError("cpu_ref_em_step failed")
        ll[s] = out.value
    return dict(W=W, C=C, B=np.diag(b), sigT=np.diag(t), sigE=sig[0], sigF=sig[1], sigH=sig[2]), ll
