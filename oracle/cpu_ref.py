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
    _ip = ct.POINTER(ct.c_int)
    lib.cpu_ref_ppls_simult.restype = ct.c_int
    lib.cpu_ref_ppls_simult.argtypes = [_dp, _dp, ct.c_int64, ct.c_int, ct.c_int, ct.c_int, _dp, _dp, _dp, ct.c_int,
                                        ct.c_double, ct.c_int, ct.c_double, _dp, _dp, _dp, _dp, _dp, _dp, _ip, _ip,
                                        _dp, ct.c_int]
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


def ppls_simult_call(X, Y, a, inits, EMsteps=10, atol=1e-4, init_steps=20, init_atol=1e-4, nthreads=0):
    """The whole PPLS_simult(X, Y, a, EMsteps, atol) call (EM_W_multi.R:758-807) on row-major X, Y:
    the initialiser PPLS(X, Y, a, init_steps, init_atol) from the starting values ``inits`` (one
    dict per component: W, C, B, sigE, sigF, sigH, sigT -- PPLSi's 'random' draws), the EM loop and
    Eout.  Returns (estimates dict, loglik, component steps, {init, loop, eout} seconds)."""
    lib = load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    n, p = X.shape
    q = Y.shape[1]
    iw = np.asfortranarray(np.column_stack([np.ravel(t["W"]) for t in inits]), dtype=np.float64)
    ic = np.asfortranarray(np.column_stack([np.ravel(t["C"]) for t in inits]), dtype=np.float64)
    th = np.ascontiguousarray([[float(np.ravel(t[k])[0]) for k in ("B", "sigE", "sigF", "sigH", "sigT")]
                               for t in inits], dtype=np.float64)
    W = np.zeros((p, a), order="F")
    C = np.zeros((q, a), order="F")
    b, t, sig = np.zeros(a), np.zeros(a), np.zeros(3)
    ll = np.zeros(EMsteps)
    steps = ct.c_int()
    cs = np.zeros(a, dtype=np.int32)
    secs = np.zeros(3)
    P = lambda v: v.ctypes.data_as(_dp)  # noqa: E731
    rc = lib.cpu_ref_ppls_simult(P(X), P(Y), n, p, q, a, P(th), P(iw), P(ic), int(init_steps), float(init_atol),
                                 int(EMsteps), float(atol), P(W), P(C), P(b), P(t), P(sig), P(ll), ct.byref(steps),
                                 cs.ctypes.data_as(ct.POINTER(ct.c_int)), P(secs), int(nthreads))
    if rc != 0:
        raise RuntimeError(f"cpu_ref_ppls_simult failed ({rc})")
    est = dict(W=W, C=C, B=np.diag(b), sigT=np.diag(t), sigE=sig[0], sigF=sig[1], sigH=sig[2])
    return est, ll[: steps.value].copy(), cs.copy(), dict(init=secs[0], loop=secs[1], eout=secs[2])
