"""Host-side mirror of the reference's R interface for the PPLS_simult hot path.

Same names, argument meaning, return structure and error behaviour as the R functions
(paths relative to /root/reference):

* ``PPLS_simult``  Package/PPLS/R/EM_W_multi.R:758-807
* ``Expect_M``     Package/PPLS/R/EM_W_multi.R:637-717
* ``Maximiz_M``    Package/PPLS/R/EM_W_multi.R:729-742
* ``logl_W``       Package/PPLS/R/EM_W_multi.R:297-323
* ``loglC_fast``   Package/PPLS/src/loglC.cpp:318-338 (via RcppExports.R:32-34)
* ``meta_EMstep``  Package/PPLS/R/EM_W_multi.R:446-485 (meta_Estep/meta_Mstep, src/loglC.cpp:399-474)
* ``meta_PPLSi``   Package/PPLS/R/EM_W_multi.R:509-589
* ``PPLS_to_o2m``  Package/PPLS/R/PPLS_to_o2m.R:28-80
* ``variances_PPLS_simult``  Package/PPLS/R/EM_W_multi.R:830-860 (variances.PPLS_simult)

Every call goes through the C ABI (include/ppls.h) into the HIP kernels on the GPU; matrices
are numpy arrays, R lists are dicts.  Passing ``X=None, Y=None`` uses the data already resident
in the context (no copy), which is how multi-GPU shards and large synthetic problems are driven.
"""
from __future__ import annotations

import ctypes as ct
import math
import time
import warnings

import numpy as np

from . import _lib
from ._lib import Expect, PplsError, Theta, dptr


def pop_rows(pop_sizes, row0, n_local):
    """(local, total) rows per population for the shard [row0, row0 + n_local): population j is the
    global row block [N_1 + .. + N_{j-1}, N_1 + .. + N_j) (EM_W_multi.R:451-458, :537-541)."""
    sizes = np.asarray(pop_sizes, dtype=np.int64)
    ends = np.cumsum(sizes)
    begins = ends - sizes
    lo, hi = int(row0), int(row0) + int(n_local)
    local = np.clip(np.minimum(ends, hi) - np.maximum(begins, lo), 0, None).astype(np.int64)
    return np.ascontiguousarray(local), np.ascontiguousarray(sizes)


class Context:
    """One GPU, one HIP stream, resident X/Y (``ppls_ctx``)."""

    def __init__(self, device: int = 0):
        self._L = _lib.lib()
        h = ct.c_void_p()
        rc = self._L.ppls_ctx_create(int(device), ct.byref(h))
        if rc != 0:
            raise PplsError(rc, f"ppls_ctx_create(device={device}) failed: "
                                f"{self._L.ppls_strerror(rc).decode()} (is a GPU visible?)")
        self.h = h
        self.p = self.q = None
        self.n_local = self.n_total = None
        self.row0 = 0

    # -- plumbing
    def _chk(self, rc):
        if rc != 0:
            raise PplsError(rc, self._L.ppls_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            self._L.ppls_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_option(self, key: str, value: int):
        self._chk(self._L.ppls_set_option(self.h, key.encode(), int(value)))

    # -- multi-GPU
    @staticmethod
    def shard_range(n_total, nranks, rank):
        L = _lib.lib()
        r0, nl = ct.c_int64(), ct.c_int64()
        L.ppls_shard_range(int(n_total), int(nranks), int(rank), ct.byref(r0), ct.byref(nl))
        return r0.value, nl.value

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = ct.create_string_buffer(128)
        rc = _lib.lib().ppls_comm_unique_id(buf)
        if rc != 0:
            raise PplsError(rc, "ncclGetUniqueId failed")
        return buf.raw

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        assert len(uid) == 128
        self._chk(self._L.ppls_comm_init(self.h, int(nranks), int(rank), uid))

    def set_reducer(self, fn):
        """Host-side reduction in place of RCCL (ppls_set_reducer): ``fn(buf)`` receives a float64
        numpy view of the buffer and must overwrite it in place with its sum over all ranks (e.g.
        ``torch.distributed.all_reduce`` on gloo).  ``None`` restores RCCL.  Collective when data
        is resident."""
        if fn is None:
            self._reducer_cb = None
            self._chk(self._L.ppls_set_reducer(self.h, None, None))
            return

        def _cb(_user, buf, count):
            try:
                fn(np.ctypeslib.as_array(buf, shape=(int(count),)))
                return 0
            except Exception:   # noqa: BLE001 -- reported to the library as a reduction failure
                import traceback
                traceback.print_exc()
                return 1

        self._reducer_cb = _lib.REDUCE_FN(_cb)   # kept alive as long as the context
        self._chk(self._L.ppls_set_reducer(self.h, ct.cast(self._reducer_cb, ct.c_void_p), None))

    # -- data
    def set_data(self, X, Y, n_total=None):
        X = np.asarray(X, dtype=np.float64)
        Y = np.asarray(Y, dtype=np.float64)
        if X.ndim != 2 or Y.ndim != 2 or X.shape[0] != Y.shape[0]:
            raise ValueError("X and Y must be matrices with the same number of rows")
        if X.flags.f_contiguous and Y.flags.f_contiguous and not (X.flags.c_contiguous and Y.flags.c_contiguous):
            layout = _lib.PPLS_LAYOUT_COLMAJOR
        else:
            X = np.ascontiguousarray(X)
            Y = np.ascontiguousarray(Y)
            layout = _lib.PPLS_LAYOUT_ROWMAJOR
        n, p = X.shape
        q = Y.shape[1]
        nt = n if n_total is None else int(n_total)
        self._chk(self._L.ppls_set_data(self.h, dptr(X), dptr(Y), n, p, q, layout, nt))
        self.p, self.q, self.n_local, self.n_total = p, q, n, nt

    def generate_synthetic(self, n_total, p, q, truth: Theta, seed: int, row0=0, n_local=None):
        nl = n_total - row0 if n_local is None else int(n_local)
        t = truth.struct()
        self._chk(self._L.ppls_generate_synthetic(self.h, int(n_total), int(row0), nl, int(p), int(q),
                                                  truth.r, ct.byref(t), ct.c_uint64(int(seed))))
        self.p, self.q, self.n_local, self.n_total, self.row0 = p, q, nl, int(n_total), int(row0)

    def get_data(self, row_begin=0, nrows=None):
        nrows = self.n_local - row_begin if nrows is None else nrows
        X = np.zeros((nrows, self.p), order="F")
        Y = np.zeros((nrows, self.q), order="F")
        self._chk(self._L.ppls_get_data(self.h, dptr(X), dptr(Y), int(row_begin), int(nrows)))
        return X, Y

    def get_data_rows(self, row_begin=0, nrows=None):
        """Rows [row_begin, row_begin + nrows) of X, Y as C-ordered (row-major) float64 arrays."""
        nrows = self.n_local - row_begin if nrows is None else nrows
        X = np.empty((nrows, self.p))
        Y = np.empty((nrows, self.q))
        self._chk(self._L.ppls_get_data_rows(self.h, dptr(X), dptr(Y), int(row_begin), int(nrows)))
        return X, Y

    def philox4x32_10(self, ctr, key: int):
        """Device Philox4x32-10 block function (the generator's): ctr (count, 4) uint32 -> (count, 4)."""
        c = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
        out = np.empty_like(c)
        u32p = ct.POINTER(ct.c_uint32)
        self._chk(self._L.ppls_philox4x32_10(self.h, c.ctypes.data_as(u32p), c.shape[0], ct.c_uint64(int(key)),
                                             out.ctypes.data_as(u32p)))
        return out

    def ssq(self):
        a, b = ct.c_double(), ct.c_double()
        self._chk(self._L.ppls_data_ssq(self.h, ct.byref(a), ct.byref(b)))
        return a.value, b.value

    # -- hot path
    def estep(self, th: Theta, want_mu=True) -> Expect:
        e = Expect(th.r, self.n_local, want_mu)
        s = e.struct()
        t = th.struct()
        self._chk(self._L.ppls_estep(self.h, ct.byref(t), th.r, ct.byref(s)))
        e.pull(s)
        return e

    def mstep(self, fit: Expect, type_: int = _lib.PPLS_ORTH_SVD) -> Theta:
        out = Theta.empty(self.p, self.q, fit.r)
        s = fit.struct()
        o = out.struct()
        self._chk(self._L.ppls_mstep(self.h, ct.byref(s), fit.r, int(type_), ct.byref(o)))
        out.pull(o)
        return out

    def em_step(self, th: Theta, type_: int = _lib.PPLS_ORTH_SVD, want_fit=False):
        out = Theta.empty(self.p, self.q, th.r)
        fit = Expect(th.r, self.n_local, want_fit) if want_fit else None
        t, o = th.struct(), out.struct()
        fs = fit.struct() if fit is not None else None
        self._chk(self._L.ppls_em_step(self.h, ct.byref(t), th.r, int(type_), ct.byref(o),
                                       ct.byref(fs) if fs is not None else None))
        out.pull(o)
        if fit is not None:
            fit.pull(fs)
        return out, fit

    def loglik(self, th: Theta) -> float:
        out = ct.c_double()
        t = th.struct()
        self._chk(self._L.ppls_loglik(self.h, ct.byref(t), th.r, ct.byref(out)))
        return out.value

    def em_run(self, th: Theta, max_steps=10, atol=1e-4, type_=_lib.PPLS_ORTH_SVD, want_eout=True,
               want_mu=True):
        """PPLS_simult's loop from theta0 = th (copied); returns (estimates, loglik, eout, warn)."""
        est = Theta(th.W, th.C, th.B, th.sigE, th.sigF, th.sigH, th.sigT)
        ll = np.zeros(max_steps)
        steps = ct.c_int()
        neg = ct.c_int()
        eout = Expect(th.r, self.n_local, want_mu) if want_eout else None
        t = est.struct()
        es = eout.struct() if eout is not None else None
        self._chk(self._L.ppls_em_run(self.h, ct.byref(t), th.r, int(max_steps), float(atol), int(type_),
                                      dptr(ll), ct.byref(steps), ct.byref(neg),
                                      ct.byref(es) if es is not None else None))
        est.pull(t)
        if eout is not None:
            eout.pull(es)
        return est, ll[: steps.value].copy(), eout, bool(neg.value)

    def em_begin(self, th: Theta):
        t = th.struct()
        self._chk(self._L.ppls_em_begin(self.h, ct.byref(t), th.r))
        self._em_r = th.r

    def em_iterate(self, nsteps: int, type_: int = _lib.PPLS_ORTH_SVD):
        self._chk(self._L.ppls_em_iterate(self.h, int(nsteps), int(type_)))

    def em_state(self):
        out = Theta.empty(self.p, self.q, self._em_r)
        cap = 1 << 16
        ll = np.zeros(cap)
        n = ct.c_int()
        o = out.struct()
        self._chk(self._L.ppls_em_state(self.h, ct.byref(o), dptr(ll), cap, ct.byref(n)))
        out.pull(o)
        return out, ll[: n.value].copy()

    def ppls(self, a: int, max_steps: int, atol: float, inits, constraints=None, crit_abs=False):
        """Sequential PPLS fit (EM_W_multi.R:229-279) from a list of ``a`` rank-1 starting values
        (dicts W, C, B, sigE, sigF, sigH, sigT); ``constraints``: None or one fconstraint dict per
        component (fixed values, EM_W_multi.R:85-92); ``crit_abs``: critfunc = abs.  Returns the
        reference's list (W, C, B, sig, Other_output) plus the per-component logvalue traces."""
        p, q = self.p, self.q
        ths = [Theta(np.reshape(t["W"], (p, 1)), np.reshape(t["C"], (q, 1)), float(np.ravel(t["B"])[0]),
                     t["sigE"], t["sigF"], t["sigH"], float(np.ravel(t["sigT"])[0])) for t in inits]
        if len(ths) != a:
            raise ValueError(f"{len(ths)} starting values for nr_comp = {a}")
        arr = (_lib.PplsTheta * a)(*[t.struct() for t in ths])
        W = np.zeros((p, a), order="F")
        C = np.zeros((q, a), order="F")
        B = np.zeros(a)
        sig = np.zeros((a, 4), order="F")
        lv = np.full((a, max_steps + 1), np.nan)
        last = np.zeros(a)
        nst = np.zeros(a, dtype=np.int32)
        lls = np.zeros(a)
        fit = _lib.PplsSeqFit(dptr(W), dptr(C), dptr(B), dptr(sig), dptr(lv), dptr(last),
                              nst.ctypes.data_as(ct.POINTER(ct.c_int)), dptr(lls), 0, 0)
        cons = None
        keep = []
        if constraints is not None:
            if len(constraints) != a:
                raise ValueError("There should be a list of constraints for each component, see ?PPLS.")
            cons = (_lib.PplsConstraint * a)()
            for k, cdict in enumerate(constraints):
                for key, size in (("W", p), ("C", q), ("B", 1), ("sigE", 1), ("sigF", 1), ("sigH", 1), ("sigT", 1)):
                    v = (cdict or {}).get(key)
                    if v is None:
                        continue
                    arrv = np.ascontiguousarray(np.ravel(np.asarray(v, dtype=np.float64)))
                    if arrv.shape[0] != size:
                        raise ValueError(f"constraint {key} of component {k + 1} has {arrv.shape[0]} values, not {size}")
                    keep.append(arrv)
                    setattr(cons[k], key, dptr(arrv))
        self._chk(self._L.ppls_ppls_ex(self.h, int(a), int(max_steps), float(atol), int(bool(crit_abs)), arr,
                                       cons, ct.byref(fit)))
        del keep
        k = fit.ncomp
        return dict(W=W[:, :k].copy(), C=C[:, :k].copy(), B=B[:k].copy(), sig=sig[:k].copy(),
                    Other_output=dict(Last_increment=last[:k].copy(), Number_steps=nst[:k].copy(),
                                      Loglikelihoods=lls[:k].copy(),
                                      logvalue=[lv[i, :nst[i] + 1].copy() for i in range(k)]),
                    not_monotone=[bool(fit.not_monotone >> i & 1) for i in range(k)], ncomp=k)

    def pop_rows(self, pop_sizes):
        return pop_rows(pop_sizes, self.row0, self.n_local)

    def meta_emstep(self, W, C, pop_sizes, params):
        """meta_EMstep (EM_W_multi.R:446-485) on the resident rows: per-population E- and M-step
        (meta_Estep / meta_Mstep, src/loglC.cpp:399-474) and the shared W., C.  params: npop x 5
        (B_T, sigX, sigY, sigH, sigT).  Returns (W, C, params_out, Cxt p x npop, Cyu q x npop)."""
        loc, tot = self.pop_rows(pop_sizes)
        npop = len(tot)
        W = np.ascontiguousarray(np.ravel(W), dtype=np.float64)
        C = np.ascontiguousarray(np.ravel(C), dtype=np.float64)
        pin = np.asfortranarray(np.asarray(params, dtype=np.float64).reshape(npop, 5))
        Wo, Co = np.zeros(self.p), np.zeros(self.q)
        po = np.zeros((npop, 5), order="F")
        cxt, cyu = np.zeros((self.p, npop), order="F"), np.zeros((self.q, npop), order="F")
        i64 = ct.POINTER(ct.c_int64)
        self._chk(self._L.ppls_meta_emstep(self.h, npop, loc.ctypes.data_as(i64), tot.ctypes.data_as(i64),
                                           dptr(W), dptr(C), dptr(pin), dptr(Wo), dptr(Co), dptr(po),
                                           dptr(cxt), dptr(cyu)))
        return Wo, Co, po, cxt, cyu

    def meta_ppls(self, pop_sizes, max_steps, atol, init, crit_abs=False):
        """meta_PPLSi's loop (EM_W_multi.R:544-578) from the starting values ``init`` (dict W, C, B,
        sigE, sigF, sigH, sigT, r = 1).  Returns (W, C, params npop x 5, logvalue (steps+1) x npop)."""
        loc, tot = self.pop_rows(pop_sizes)
        npop = len(tot)
        th = Theta(np.reshape(init["W"], (self.p, 1)), np.reshape(init["C"], (self.q, 1)),
                   float(np.ravel(init["B"])[0]), init["sigE"], init["sigF"], init["sigH"],
                   float(np.ravel(init["sigT"])[0]))
        t = th.struct()
        Wo, Co = np.zeros(self.p), np.zeros(self.q)
        po = np.zeros((npop, 5), order="F")
        lg = np.full((max_steps + 1, npop), np.nan, order="F")
        fit = _lib.PplsMetaFit(dptr(Wo), dptr(Co), dptr(po), dptr(lg), 0)
        i64 = ct.POINTER(ct.c_int64)
        self._chk(self._L.ppls_meta_ppls(self.h, npop, loc.ctypes.data_as(i64), tot.ctypes.data_as(i64),
                                         int(max_steps), float(atol), int(bool(crit_abs)), ct.byref(t),
                                         ct.byref(fit)))
        return Wo, Co, po, lg[: fit.steps + 1].copy()

    def variances(self, mu, Cdiag, sigE, xory, full=True):
        """variances.PPLS_simult (EM_W_multi.R:830-860) on the resident X (xory 0) or Y (xory 1):
        mu = this rank's rows of Expectations$mu_T / mu_U (n_local x a), Cdiag = diag(Ctt / Cuu).
        Returns (W, B_exp scalars, varMatrix a x p x p, seLoad p x a, SSt_exp, SSt_star) -- the
        last two (a x p x p) only with full=True."""
        # no copy when mu is already a column-major float64 n_local x a array (the fits' Expectations are)
        mu = np.asfortranarray(np.asarray(mu, dtype=np.float64).reshape(self.n_local, -1))
        a = mu.shape[1]
        p = self.q if xory else self.p
        Cd = np.ascontiguousarray(np.ravel(Cdiag), dtype=np.float64)
        if Cd.shape[0] != a:
            raise ValueError(f"{Cd.shape[0]} variances for {a} components")
        W = np.zeros((p, a), order="F")
        Bx = np.zeros(a)
        V = np.zeros((a, p, p))            # component i: V[i] holds the column-major p x p as its transpose
        se = np.zeros((p, a), order="F")
        SE = np.zeros((a, p, p)) if full else None
        SS = np.zeros((a, p, p)) if full else None
        self._chk(self._L.ppls_variances(self.h, dptr(mu), dptr(Cd), float(sigE), int(a), int(xory), dptr(W),
                                         dptr(Bx), dptr(V), dptr(SE), dptr(SS), dptr(se)))
        # buffers hold consecutive column-major matrices: each is returned as its transposed view (no
        # copy -- a contiguous transpose of a x p x p doubles cost ~30 ms of host time at C3)
        tr = (lambda A: None if A is None else np.transpose(A, (0, 2, 1)))
        return W, Bx, tr(V), se, tr(SE), tr(SS)

    def gram(self, xory=0, nsplit=0, want=True):
        """D'D (D = X, Y, or xory = 2 the joint [X Y], (p + q) x (p + q)) on the fp64 MFMA Gram kernel
        alone, this rank's rows -> (G or None, kernel ms)."""
        p = self.p + self.q if xory == 2 else self.q if xory else self.p
        G = np.zeros((p, p), order="F") if want else None
        ms = ct.c_double()
        self._chk(self._L.ppls_gram(self.h, int(xory), int(nsplit), dptr(G), ct.byref(ms)))
        return G, ms.value

    def gram_int8(self, which=2, want=True):
        """The Gram by the int8-MFMA Chinese-remainder form alone (which: 0 X'X, 1 Y'Y, 2 the joint
        [X Y]'[X Y] over the padded columns) -> (G or None, dict(nmod, L, ms = [stats + residues, SYRK,
        CRT, total], shift = the per-column scalings))."""
        P = self.p if which == 0 else self.q if which == 1 else int(round(np.sqrt(self.xprod_info()["bytes_per_pass"] / 8)))
        G = np.zeros((P, P), order="F") if want else None
        nm, L, ms = ct.c_int(), ct.c_int(), np.zeros(4)
        self._chk(self._L.ppls_gram_int8(self.h, int(which), dptr(G), ct.byref(nm), ct.byref(L), dptr(ms)))
        return G, dict(nmod=nm.value, L=L.value, ms=ms.tolist(), shift=self.gram_shifts())

    def gram_shifts(self):
        """The last int8 Gram's per-column scalings: x'_kj = rint(D_kj 2^shift[j]) (int array)."""
        k = ct.c_int()
        self._chk(self._L.ppls_gram_shifts(self.h, None, 0, ct.byref(k)))
        out = (ct.c_int * max(k.value, 1))()
        self._chk(self._L.ppls_gram_shifts(self.h, out, k.value, ct.byref(k)))
        return np.array(out[:k.value], dtype=np.int64)

    def gram_info(self):
        """Which Gram ran last (forming S, or variances' X'X / Y'Y): dict(int8 (bool), nmod, L, ms =
        [stats + residues, SYRK, CRT, total])."""
        u, nm, L, ms = ct.c_int(), ct.c_int(), ct.c_int(), np.zeros(4)
        self._chk(self._L.ppls_gram_info(self.h, ct.byref(u), ct.byref(nm), ct.byref(L), dptr(ms)))
        return dict(int8=bool(u.value), nmod=nm.value, L=L.value, ms=ms.tolist())

    def spd_inverse(self, A, method=1):
        """Inverses of symmetric positive definite matrices A (a x p x p or p x p) on the device as
        variances.PPLS_simult computes them (method 1 hand-written blocked Cholesky, 2 rocSOLVER)
        -> (inverses, info per matrix: 0 or the 1-based column of the first bad pivot, device ms)."""
        A = np.asarray(A, dtype=np.float64)
        one = A.ndim == 2
        A3 = A[None] if one else A
        a, p = A3.shape[0], A3.shape[1]
        Af = np.ascontiguousarray(np.transpose(A3, (0, 2, 1)))   # column-major per matrix
        out = np.empty_like(Af)
        info = (ct.c_int * a)()
        ms = ct.c_double()
        self._chk(self._L.ppls_spd_inverse(self.h, dptr(Af), int(p), int(a), int(method), dptr(out), info,
                                            ct.byref(ms)))
        inv = np.transpose(out, (0, 2, 1))
        return (inv[0] if one else inv), np.array(list(info)), ms.value

    def xprod_prepare(self):
        """Form the cross-products S = [X Y]'[X Y] now (option "xprod") -> (Gram kernel ms, total ms);
        (0, 0) when S is already formed for the current data."""
        ms, tot = ct.c_double(), ct.c_double()
        self._chk(self._L.ppls_xprod_prepare(self.h, ct.byref(ms), ct.byref(tot)))
        return ms.value, tot.value

    def xprod_release(self):
        """Free the cross-products S now (ppls_xprod_release; 8 (p+q)^2 bytes of HBM); the next run
        that reads S forms it again."""
        self._chk(self._L.ppls_xprod_release(self.h))

    def xprod_tile_timing(self, reps=200):
        """Average ms of the cross-product tile kernel over reps back-to-back launches (HIP events
        around the batch) for the current em_begin session's theta."""
        ms = ct.c_double()
        self._chk(self._L.ppls_xprod_tile_timing(self.h, int(reps), ct.byref(ms)))
        return ms.value

    def xprod_setup_times(self):
        """(Gram kernel ms, all-reduce of S ms, whole setup ms) of the last formation of S."""
        g, a, t = ct.c_double(), ct.c_double(), ct.c_double()
        self._chk(self._L.ppls_xprod_setup_times(self.h, ct.byref(g), ct.byref(a), ct.byref(t)))
        return g.value, a.value, t.value

    def xprod_stats(self, th: Theta):
        """One statistics step from S for theta: (X'mu_T p x r, Y'mu_U q x r, Gram 2r x 2r)."""
        r = th.r
        out = np.zeros(r * (self.p + self.q) + 4 * r * r)
        t = th.struct()
        self._chk(self._L.ppls_xprod_stats(self.h, ct.byref(t), r, dptr(out)))
        SX = out[: self.p * r].reshape(r, self.p).T
        SY = out[self.p * r: (self.p + self.q) * r].reshape(r, self.q).T
        G = out[(self.p + self.q) * r:].reshape(2 * r, 2 * r).T
        return SX, SY, G

    def xprod_info(self, r=1):
        """{ready, bytes_per_pass (8 P^2), gram_flops (as computed), rows_per_wave} of the cross-product form."""
        rd, b, f, rw = ct.c_int(), ct.c_int64(), ct.c_double(), ct.c_int()
        self._chk(self._L.ppls_xprod_info(self.h, int(r), ct.byref(rd), ct.byref(b), ct.byref(f), ct.byref(rw)))
        return dict(ready=bool(rd.value), bytes_per_pass=b.value, gram_flops=f.value, rows_per_wave=rw.value)

    def scores(self, W, C):
        """scores.PPLS (EM_W_multi.R:411-420) on the resident rows: (X W, Y C), n_local x k each."""
        W = np.asfortranarray(np.array(W, dtype=np.float64, ndmin=2).reshape(self.p, -1))
        C = np.asfortranarray(np.array(C, dtype=np.float64, ndmin=2).reshape(self.q, -1))
        k = W.shape[1]
        if C.shape[1] != k:
            raise ValueError("W and C need the same number of components")
        T = np.zeros((self.n_local, k), order="F")
        U = np.zeros((self.n_local, k), order="F")
        self._chk(self._L.ppls_scores(self.h, dptr(W), dptr(C), int(k), dptr(T), dptr(U)))
        return T, U

    def synchronize(self):
        self._chk(self._L.ppls_synchronize(self.h))

    def loglC_fast(self, W, C, X, Y, sigX, sigY, sig2T, c1, c2, c3, Kc) -> float:
        W = np.asfortranarray(W, dtype=np.float64)
        C = np.asfortranarray(C, dtype=np.float64)
        a = W.shape[1] if W.ndim == 2 else 1
        vec = [np.ascontiguousarray(np.ravel(v), dtype=np.float64) for v in (sig2T, c1, c2, c3, Kc)]
        out = ct.c_double()
        if X is None:
            n, p, q = self.n_total, self.p, self.q
            xp = yp = None
        else:
            X = np.asfortranarray(X, dtype=np.float64)
            Y = np.asfortranarray(Y, dtype=np.float64)
            n, p = X.shape
            q = Y.shape[1]
            xp, yp = dptr(X), dptr(Y)
            self.p, self.q, self.n_local, self.n_total = p, q, n, n
        self._chk(self._L.ppls_loglC_fast(self.h, dptr(W), dptr(C), xp, yp, int(n), int(p), int(q), int(a),
                                          float(sigX), float(sigY), *[dptr(v) for v in vec],
                                          ct.byref(out)))
        return out.value

    # -- measurement
    def sweep_timing(self, reset=True):
        ms, n = ct.c_double(), ct.c_int64()
        self._chk(self._L.ppls_sweep_timing(self.h, ct.byref(ms), ct.byref(n), int(reset)))
        return ms.value, n.value

    def sweep_balance(self):
        """(weights per XCD class g % 8, row boundaries per workgroup or None) of the split sweep's
        calibrated row partition (option "balance")."""
        w = np.ones(8)
        cap = 4097
        b = np.zeros(cap, dtype=np.int64)
        nb = ct.c_int()
        self._chk(self._L.ppls_sweep_balance(self.h, dptr(w), b.ctypes.data_as(ct.POINTER(ct.c_int64)), cap,
                                             ct.byref(nb)))
        return w, (b[: nb.value].copy() if nb.value else None)

    def comm_info(self, reset=True):
        """(nranks, rank) as RCCL's communicator reports them (ncclCommCount / ncclCommUserRank; the
        context's own values without RCCL) and (total ms, calls) of the timed all-reduces."""
        nr, rk, ms, n = ct.c_int(), ct.c_int(), ct.c_double(), ct.c_int64()
        self._chk(self._L.ppls_comm_info(self.h, ct.byref(nr), ct.byref(rk), ct.byref(ms), ct.byref(n), int(reset)))
        return nr.value, rk.value, ms.value, n.value

    def sweep_trace(self, grid):
        """Per-workgroup wall-clock stamps (us, relative to the earliest entry) of the last split
        sweep: (grid, 4) = entry, ring prologue done, row loop done, partials written."""
        buf = (ct.c_int64 * (4 * grid))()
        n, tick = ct.c_int(), ct.c_double()
        self._chk(self._L.ppls_sweep_trace(self.h, buf, int(grid), ct.byref(n), ct.byref(tick)))
        a = np.array(buf[:4 * n.value], dtype=np.int64).reshape(n.value, 4)
        return (a - a[:, 0].min()) * tick.value / 1e3

    def finalize_trace(self):
        """Phase stamps of the last finalize (set_option('ftrace', 1) first): {block: [us since the
        block's first stamp, ...]} for the slots that were reached."""
        buf = (ct.c_int64 * 48)()
        tick = ct.c_double()
        self._chk(self._L.ppls_finalize_trace(self.h, buf, ct.byref(tick)))
        out = {}
        for b in range(3):
            s = [buf[16 * b + i] for i in range(16)]
            if s[0]:
                us = [round((v - s[0]) * tick.value * 1e-3, 3) if v else None for v in s]
                # 10-12 raw (Jacobi sweeps, core clock stamps); a polar team's member 0 stamps its
                # first barrier in 9 (arrived) and 10 (all arrived)
                out[b] = us[:10] + ([us[10]] if s[10] > 1000 else [s[10]]) + s[11:13] + us[13:]
        return out

    def sweep_info(self, r):
        b, v, g = ct.c_int64(), ct.c_int(), ct.c_int()
        self._chk(self._L.ppls_sweep_info(self.h, int(r), ct.byref(b), ct.byref(v), ct.byref(g)))
        return dict(bytes_per_sweep=b.value, variant={4: "split512", 5: "panel"}[v.value], grid=g.value)

    def meta_info(self):
        """The path the last meta_ppls took: "none", "host", "device_split" or "device_panel"."""
        v = ct.c_int()
        self._chk(self._L.ppls_meta_info(self.h, ct.byref(v)))
        return ("none", "host", "device_split", "device_panel")[v.value]

    def sweep_kernel(self, r):
        """The sweep kernel instantiation an EM iteration with r components launches (text)."""
        buf = ct.create_string_buffer(256)
        self._chk(self._L.ppls_sweep_kernel(self.h, int(r), buf, 256))
        return buf.value.decode()


# ================================================================================ R mirror
_DEFAULT_CTX = None


def default_context() -> Context:
    """The context the R-named functions use when no ``ctx`` is given: GPU 0, with the statistics
    path chosen per run by the cost model (option "xprod" = -1, as the R shim in INTEGRATION.md
    sets it: the cross-product form once a run is long enough to repay forming S).  A formed S
    stays resident for the data (8 (p+q)^2 bytes of HBM: 128 MB at p = q = 2000, 0.9 GB at
    p + q = 10,500) until new data are loaded, ``xprod`` is set to 0, or
    ``default_context().xprod_release()`` frees it."""
    global _DEFAULT_CTX
    if _DEFAULT_CTX is None:
        _DEFAULT_CTX = Context(0)
        _DEFAULT_CTX.set_option("xprod", -1)
    return _DEFAULT_CTX


def _orth_type(type):
    if isinstance(type, (list, tuple)):
        type = type[0]            # match.arg(type) picks the first choice, EM_W_multi.R:761
    if type not in ("SVD", "QR"):
        raise ValueError("'arg' should be one of \"SVD\", \"QR\"")
    return _lib.PPLS_ORTH_SVD if type == "SVD" else _lib.PPLS_ORTH_QR


def _ctx_with(X, Y, ctx):
    ctx = ctx or default_context()
    if X is not None:
        ctx.set_data(X, Y)
    elif ctx.n_local is None:
        raise ValueError("no data: pass X and Y or a context with resident data")
    return ctx


def Expect_M(X, Y, W, C, B, sigE, sigF, sigH, sigT, debug=False, ctx=None):
    """Expect_M (EM_W_multi.R:637-717): posterior first and second moments."""
    if debug:
        raise NotImplementedError("debug=TRUE (dense Sigma^-1, EM_W_multi.R:643-667) is an O(n(p+q)^2) "
                                  "cross-check; it lives in the test oracle, not on the GPU path")
    ctx = _ctx_with(X, Y, ctx)
    th = Theta(W, C, B, sigE, sigF, sigH, sigT)
    return ctx.estep(th, want_mu=True).as_dict()


def Maximiz_M(fit, X, Y, type=("SVD", "QR"), ctx=None):
    """Maximiz_M (EM_W_multi.R:729-742): W = orth(X'mu_T), C = orth(Y'mu_U), scalar updates."""
    ctx = _ctx_with(X, Y, ctx)
    r = np.asarray(fit["Ctt"]).shape[0]
    e = Expect(r, ctx.n_local, True)
    e.mu_T[:] = np.asarray(fit["mu_T"])
    e.mu_U[:] = np.asarray(fit["mu_U"])
    e.Ctt[:] = np.diag(np.asarray(fit["Ctt"]))
    e.Cuu[:] = np.diag(np.asarray(fit["Cuu"]))
    e.Cut[:] = np.diag(np.asarray(fit["Cut"]))
    e.Cee = float(np.trace(np.atleast_2d(fit["Cee"])) / np.atleast_2d(fit["Cee"]).shape[1])
    e.Cff = float(np.trace(np.atleast_2d(fit["Cff"])) / np.atleast_2d(fit["Cff"]).shape[1])
    e.Chh[:] = np.asarray(fit["Chh"])
    th = ctx.mstep(e, _orth_type(type))
    d = th.as_dict()
    return dict(W=d["W"], C=d["C"], B=d["B"], sigE=d["sigE"], sigF=d["sigF"], sigH=d["sigH"], sigT=d["sigT"])


def logl_W(X, Y, W, C, B_T, sigX, sigY, sigH, sigT, ctx=None):
    """logl_W (EM_W_multi.R:297-323)."""
    ctx = _ctx_with(X, Y, ctx)
    W = np.array(W, dtype=np.float64, ndmin=2)
    if W.shape[0] == 1 and ctx.p != 1:
        W = W.T
    C = np.array(C, dtype=np.float64, ndmin=2)
    if C.shape[0] == 1 and ctx.q != 1:
        C = C.T
    return ctx.loglik(Theta(W, C, B_T, sigX, sigY, sigH, sigT))


def loglC_fast(W, C, X, Y, sigX, sigY, sig2T, c1, c2, c3, Kc, ctx=None):
    """loglC_fast (src/loglC.cpp:318-338) -- the drop-in of .Call('PPLS_loglC_fast', ...)."""
    ctx = ctx or default_context()
    return ctx.loglC_fast(W, C, X, Y, sigX, sigY, sig2T, c1, c2, c3, Kc)


def random_theta0(p, q, a, seed=0):
    """Deterministic synthetic theta0: W0 = orth(N(0,1)), C0 = orth(N(0,1)), B0 = I, sigT0 = I,
    sigmas = 1 (the benchmark's starting point).  PPLS_simult's own default theta0 is
    the sequential fit PPLS(X, Y, a, 20, 1e-4, 'random') (EM_W_multi.R:762-771), which
    ``PPLS_simult`` below runs on the device."""
    rng = np.random.default_rng(seed)

    def polar(M):
        U, _, Vt = np.linalg.svd(M, full_matrices=False)
        return U @ Vt

    return dict(W=polar(rng.standard_normal((p, a))), C=polar(rng.standard_normal((q, a))),
                B=np.eye(a), sigE=1.0, sigF=1.0, sigH=1.0, sigT=np.eye(a))


def initial_guess(p, q, kind="equal", rng=None):
    """PPLSi's starting values (EM_W_multi.R:126-140): 'equal' (deterministic) or 'random' --
    orth(runif(p)), orth(runif(q)), rchisq(1,1), rchisq(2,100)/100 (sigH, sigT), rchisq(2,10)/100
    (sigE, sigF), drawn in that order (:133).

    ``rng``: an R-compatible stream (any object with R's ``runif(n)`` and ``rchisq(n, df)``, e.g. a
    restatement of R's Mersenne-Twister/Inversion defaults) reproduces R's draws after the same
    ``set.seed``; a numpy ``Generator`` draws from the same distributions.  ``orth`` of a positive
    vector is taken as v/||v|| (the QR form's -v/||v|| gives the mirrored, equivalent fit).
    'o2m' depends on the data: PPLS / PPLSi / meta_PPLSi compute it (o2m_guess_from_gram)."""
    if kind == "equal":
        return dict(W=np.ones(p) / np.sqrt(p), C=np.ones(q) / np.sqrt(q), B=1.0, sigE=1.0 / p,
                    sigF=1.0 / q, sigH=1.0, sigT=1.0)
    if kind == "random":
        rng = rng if rng is not None else np.random.default_rng()
        if hasattr(rng, "runif") and hasattr(rng, "rchisq"):      # R's own stream
            W = np.asarray(rng.runif(p), dtype=np.float64)
            C = np.asarray(rng.runif(q), dtype=np.float64)
            B = float(np.ravel(rng.rchisq(1, 1))[0])
            siglat = np.asarray(rng.rchisq(2, 100), dtype=np.float64) / 100
            sig = np.asarray(rng.rchisq(2, 10), dtype=np.float64) / 100
        else:
            W = rng.uniform(size=p)
            C = rng.uniform(size=q)
            B = rng.chisquare(1)
            siglat = rng.chisquare(100, size=2) / 100
            sig = rng.chisquare(10, size=2) / 100
        return dict(W=W / np.linalg.norm(W), C=C / np.linalg.norm(C), B=float(B), sigE=float(sig[0]),
                    sigF=float(sig[1]), sigH=float(siglat[0]), sigT=float(siglat[1]))
    if kind == "o2m":
        raise ValueError("initialGuess='o2m' depends on the data: PPLS / PPLSi / meta_PPLSi compute it "
                         "(o2m_guess_from_gram)")
    raise ValueError(f"unknown initialGuess {kind!r}")


def o2m_guess_from_gram(G, N, p, q, Wprev=None, Cprev=None):
    """PPLSi's 'o2m' starting values (EM_W_multi.R:126-131; meta_PPLSi :520-525) from the joint Gram
    G = [X Y]'[X Y] ((p + q) x (p + q), Context.gram(2)) of N rows, for the data PPLS deflated by the
    earlier components' loadings Wprev (p x k), Cprev (q x k): Xc = X P_1 ... P_k, P_j = I - w_j w_j'
    (:270-271, sequentially, as the reference does).  o2m(Xc, Yc, 1, 0, 0) of OmicsPLS (not vendored,
    no version pinned) with no orthogonal parts: W., C. = the first singular pair of Xc'Yc (LAPACK on
    the host, p x q: _top_singular_pair), Tt = Xc W., U = Yc C., B = Tt'U / Tt'Tt -- every sum of squares
    and product read off G (ssq(Tt) = z'X'Xz with z = P_1 ... P_k W.), so no pass over the rows.
    Returns the starting-value dict (W, C, B, sigE, sigF, sigH, sigT).  Parity unpinned against R
    (no reference file holds an o2m fit); checked against the oracle's restatement on the explicit
    deflated data (tests/test_o2m_host.py, tests/test_gpu_o2m.py)."""
    G = np.asarray(G, dtype=np.float64)
    Gxx, Gyy, Gxy = G[:p, :p], G[p:, p:], G[:p, p:]
    Wp = np.zeros((p, 0)) if Wprev is None else np.asarray(Wprev, dtype=np.float64).reshape(p, -1)
    Cp = np.zeros((q, 0)) if Cprev is None else np.asarray(Cprev, dtype=np.float64).reshape(q, -1)
    M = Gxy.copy()                          # Xc'Yc = P_k ... P_1 X'Y Q_1 ... Q_k
    for j in range(Wp.shape[1]):
        M -= np.outer(Wp[:, j], Wp[:, j] @ M)
    for j in range(Cp.shape[1]):
        M -= np.outer(M @ Cp[:, j], Cp[:, j])

    def chain(Vp, v):                       # P_1 ... P_k v
        for j in reversed(range(Vp.shape[1])):
            v = v - Vp[:, j] * (Vp[:, j] @ v)
        return v

    def ssq_deflated(Gd, Vp):               # ssq(D P_1 ... P_k): ssq(A P) = ssq(A) - (2 - w'w) ||A w||^2
        t = float(np.trace(Gd))
        for j in range(Vp.shape[1]):
            z = chain(Vp[:, :j], Vp[:, j])  # A_{j-1} w_j = D z
            t -= (2.0 - float(Vp[:, j] @ Vp[:, j])) * float(z @ Gd @ z)
        return t

    w, c = _top_singular_pair(M)
    zx, zy = chain(Wp, w), chain(Cp, c)
    sst, ssu, tu = float(zx @ Gxx @ zx), float(zy @ Gyy @ zy), float(zx @ Gxy @ zy)
    B = tu / sst
    ssx, ssy = ssq_deflated(Gxx, Wp), ssq_deflated(Gyy, Cp)
    return dict(W=w, C=c, B=B, sigE=float(np.sqrt((ssx - sst) / N / p)), sigF=float(np.sqrt((ssy - ssu) / N / q)),
                sigH=float(np.sqrt((ssu - B * B * sst) / N)), sigT=float(np.sqrt(sst / N)))


def _top_singular_pair(M):
    """The first singular pair of M (p x q) from the top eigenvector of the smaller of M'M, MM'
    (LAPACK's MRRR for that one pair: 0.3 s at 2000 x 2000 against 2.5 s for a whole svd), the
    other side as M v / ||M v||.  Its sign is LAPACK's, as the reference's svd's is."""
    import scipy.linalg
    p, q = M.shape
    if q <= p:
        _, v = scipy.linalg.eigh(M.T @ M, subset_by_index=[q - 1, q - 1])
        c = v[:, 0]
        w = M @ c
        return w / np.linalg.norm(w), c
    _, v = scipy.linalg.eigh(M @ M.T, subset_by_index=[p - 1, p - 1])
    w = v[:, 0]
    c = M.T @ w
    return w, c / np.linalg.norm(c)


def _ppls_o2m(ctx, a, steps, atol, constraints, crit_abs):
    """PPLS with 'o2m' starting values: component i starts from o2m of the data deflated by the
    fitted components 1 .. i-1 (:256-257 with :126-131), read off the joint Gram.  The device learns
    component i in a fit of i components whose first i - 1 are fixed (fconstraint, all seven values)
    to their fitted values -- the same deflation, each fixed component one EM step (its increment is
    exactly 0) -- and the result is assembled from those fits (ctx.ppls's dict)."""
    G = _joint_gram(ctx)
    p, q = ctx.p, ctx.q
    keys = ("W", "C", "B", "sig", "not_monotone")
    acc = {k: [] for k in keys}
    oo = {k: [] for k in ("Last_increment", "Number_steps", "Loglikelihoods", "logvalue")}
    inits, fixed = [], []
    Wp = Cp = None
    for i in range(a):
        inits.append(o2m_guess_from_gram(G, ctx.n_total, p, q, Wp, Cp))
        cons = fixed + [None if constraints is None else constraints[i]]
        f = ctx.ppls(i + 1, steps, atol, inits, cons, crit_abs)
        if f["ncomp"] < i + 1:   # :258-263: the fit stops at this component
            break
        for k in ("W", "C"):
            acc[k].append(f[k][:, i].copy())
        acc["B"].append(f["B"][i])
        acc["sig"].append(f["sig"][i].copy())
        acc["not_monotone"].append(f["not_monotone"][i])
        for k in ("Last_increment", "Number_steps", "Loglikelihoods"):
            oo[k].append(f["Other_output"][k][i])
        oo["logvalue"].append(f["Other_output"]["logvalue"][i])
        s = f["sig"][i]
        fixed.append(dict(W=f["W"][:, i].copy(), C=f["C"][:, i].copy(), B=f["B"][i], sigE=s[0], sigF=s[1],
                          sigH=s[2], sigT=s[3]))
        inits[i] = dict(fixed[i])
        Wp, Cp = f["W"], f["C"]
    k = len(acc["B"])
    return dict(W=np.array(acc["W"]).T.reshape(p, k), C=np.array(acc["C"]).T.reshape(q, k), B=np.array(acc["B"]),
                sig=np.array(acc["sig"]).reshape(k, 4),
                Other_output=dict(Last_increment=np.array(oo["Last_increment"]),
                                  Number_steps=np.array(oo["Number_steps"], dtype=np.int32),
                                  Loglikelihoods=np.array(oo["Loglikelihoods"]), logvalue=oo["logvalue"]),
                not_monotone=acc["not_monotone"], ncomp=k)


def _joint_gram(ctx):
    if ctx.n_local != ctx.n_total:
        raise NotImplementedError("initialGuess='o2m' on row shards: all-reduce the ranks' Context.gram(2) "
                                  "and call o2m_guess_from_gram")
    G, _ = ctx.gram(2)
    return G


def fconstraint(constraints=None):
    """fconstraint (EM_W_multi.R:85-92): the seven named constraints W, C, B, sigE, sigF, sigH, sigT;
    None = estimated, a number (or vector for W, C) = fixed."""
    out = dict(W=None, C=None, B=None, sigE=None, sigF=None, sigH=None, sigT=None)
    for k, v in (constraints or {}).items():
        if k in out:
            out[k] = v
    return out


def _crit_abs(critfunc):
    if critfunc is None or getattr(critfunc, "__name__", "") == "identity":
        return False
    if critfunc in (abs, np.abs, np.fabs):
        return True
    raise NotImplementedError("critfunc must be the identity (default) or abs")


def PPLS(X, Y, nr_comp=1, EMsteps=100, atol=1e-4, initialGuess=("equal", "o2m", "random", "custom"),
         customGuess=None, critfunc=None, constraints=None, rng=None, ctx=None):
    """PPLS (EM_W_multi.R:229-279) on the GPU: nr_comp sequential rank-1 EM fits on deflated data.
    Same return list (W, C, B, sig, Other_output); class "PPLS".  customGuess: one dict (used for
    every component, as in R) or a list of per-component dicts; critfunc: identity (default) or abs;
    constraints: None or a list of nr_comp fconstraint(...) dicts (:230, :255)."""
    ctx = _ctx_with(X, Y, ctx)
    kind = initialGuess if isinstance(initialGuess, str) else initialGuess[0]
    if customGuess is not None:
        kind = "custom"
    if constraints is not None and len(constraints) != nr_comp:
        raise ValueError("There should be a list of constraints for each component, see ?PPLS.")   # :240
    if kind == "custom":
        inits = list(customGuess) if isinstance(customGuess, (list, tuple)) else [customGuess] * nr_comp
    elif kind == "o2m":
        out = _ppls_o2m(ctx, int(nr_comp), int(EMsteps), float(atol), constraints, _crit_abs(critfunc))
        return _ppls_finish(out, nr_comp)
    else:
        rng = rng if rng is not None else np.random.default_rng()
        inits = [initial_guess(ctx.p, ctx.q, kind, rng) for _ in range(nr_comp)]
    return _ppls_finish(ctx.ppls(int(nr_comp), int(EMsteps), float(atol), inits, constraints, _crit_abs(critfunc)),
                        nr_comp)


def _ppls_finish(out, nr_comp):
    if out["ncomp"] < nr_comp:
        warnings.warn(f"From component {out['ncomp'] + 1} on the residuals are of rank < 1e-14 and "
                      "calculations are stopped.")
    for k, bad in enumerate(out.pop("not_monotone")):
        if bad:
            warnings.warn(f"Not monotone (component {k + 1})")
    out.pop("ncomp")
    out["class"] = "PPLS"
    return out


def PPLSi(X, Y, EMsteps=100, atol=1e-4, initialGuess=("equal", "o2m", "random", "custom"),
          customGuess=None, critfunc=None, constraints=None, rng=None, ctx=None):
    """PPLSi (EM_W_multi.R:116-180): one direction; returns W, C, B, sig, logvalue, Last_increment,
    Number_steps (W = NA when sigE or sigF collapse, :152-154).  constraints: one fconstraint dict."""
    fit = PPLS(X, Y, 1, EMsteps, atol, initialGuess, customGuess, critfunc,
               None if constraints is None else [constraints], rng, ctx)
    if len(fit["B"]) == 0:
        return dict(W=None, C=None, B=None, sig=None, logvalue=None, Last_increment=None, Number_steps=None)
    oo = fit["Other_output"]
    return dict(W=fit["W"][:, 0], C=fit["C"][:, 0], B=fit["B"][0], sig=fit["sig"][0],
                logvalue=oo["logvalue"][0], Last_increment=oo["Last_increment"][0],
                Number_steps=int(oo["Number_steps"][0]))


def _signif(x, digits):
    if x == 0 or not np.isfinite(x):
        return x
    return round(x, digits - 1 - int(np.floor(np.log10(abs(x)))))


def print_PPLS(x, perc=True, digits=3):
    """print.PPLS (EM_W_multi.R:336-354): the per-component variance table of a PPLS fit.
    Returns (rows, text): rows = n x 7 array (LV, ssq(T)/ssq(X), ssq(U)/ssq(Y), sigH^2/ssq(U),
    log LR, #steps, last incr) rounded to ``digits``; ``perc=False`` gives the absolute variances.
    As in R, sigH^2 is added once per component inside the ssq(U) sum."""
    p, q = x["W"].shape[0], x["C"].shape[0]
    sig, B, oo = np.asarray(x["sig"]), np.asarray(x["B"]), x["Other_output"]
    ll = np.asarray(oo["Loglikelihoods"], dtype=np.float64)
    dll = np.concatenate([[0.0], np.diff(ll)])
    pc = 1.0 if perc else 0.0
    rows = []
    for i in range(sig.shape[0]):
        st = float(np.sum(sig[: i + 1, 3] ** 2))
        su = float(np.sum(sig[: i + 1, 3] ** 2 * B[: i + 1] ** 2 + sig[i, 2] ** 2))
        rows.append([i + 1, st / (pc * (st + p * sig[i, 0] ** 2) + (1 - pc)),
                     su / (pc * (su + q * sig[i, 1] ** 2) + (1 - pc)),
                     sig[i, 2] ** 2 / (pc * su + (1 - pc)), dll[i], float(oo["Number_steps"][i]),
                     _signif(float(oo["Last_increment"][i]), 3)])
    rows = np.round(np.array(rows, dtype=np.float64), digits)
    names = ["LV", "ssq(T)/ssq(X)" if perc else "ssq(T)", "ssq(U)/ssq(Y)" if perc else "ssq(U)",
             "sigH^2/ssq(U)" if perc else "sigH^2", "log LR", "#steps", "last incr"]
    text = "  ".join(names) + "\n" + "\n".join(
        "  ".join(f"{v:g}" for v in row) for row in rows)
    return rows, text


def scores_PPLS(fit, X, Y, subset=None, ctx=None):
    """scores.PPLS (EM_W_multi.R:411-420): rbind(X W[, subset], Y C[, subset]) (a vector when one
    component is selected); X W and Y C are computed on the GPU in one pass.  ``fit``: a PPLS list
    (W, C) or a PPLS_simult list (estimates$W, estimates$C)."""
    ctx = _ctx_with(X, Y, ctx)
    est = fit.get("estimates", fit)
    W, C = np.asarray(est["W"]), np.asarray(est["C"])
    cols = list(range(W.shape[1])) if subset is None else [int(s) - 1 for s in np.atleast_1d(subset)]
    T, U = ctx.scores(W[:, cols], C[:, cols])
    if len(cols) == 1:
        return np.concatenate([T[:, 0], U[:, 0]])
    return np.vstack([T, U])


def PPLS_to_o2m(X_true, Y_true, fit_PPLS, ctx=None):
    """PPLS_to_o2m (PPLS_to_o2m.R:28-80): a sequential PPLS fit as an OmicsPLS "o2m" list.  The
    scores Tt = X W, U = Y C come from one device pass (ppls_scores); ssq(X), ssq(Y) from the
    context; ssq(U B_U W'), ssq(Tt B_T C') are evaluated as r x r traces (no n x p product)."""
    ctx = _ctx_with(X_true, Y_true, ctx)
    W = np.asarray(fit_PPLS["W"], dtype=np.float64).reshape(ctx.p, -1)
    C = np.asarray(fit_PPLS["C"], dtype=np.float64).reshape(ctx.q, -1)
    b = np.ravel(np.asarray(fit_PPLS["B"], dtype=np.float64))
    B_T = np.diag(b)                                          # diag(fit_PPLS$B, length(fit_PPLS$B)) (:33)
    B_U = np.linalg.inv(B_T)                                  # solve(B_T) (:34)
    Tt, U = ctx.scores(W, C)                                  # :35-36
    n = Tt.shape[0]
    ssqX, ssqY = ctx.ssq()                                    # :44-45

    def ssq(A):
        A = np.asarray(A, dtype=np.float64)
        return float(np.sum(A * A))

    def ssq_prod(S, M, L):   # ssq(S M L') = tr(M' S'S M L'L)
        return float(np.trace(M.T @ (S.T @ S) @ M @ (L.T @ L)))
    R2Xcorr, R2Ycorr = ssq(Tt) / ssqX, ssq(U) / ssqY          # :47-48
    R2Xhat = ssq_prod(U, B_U, W) / ssqX                       # :51
    R2Yhat = ssq_prod(Tt, B_T, C) / ssqY                      # :52
    z = lambda r, c: np.zeros((r, c))
    model = dict(Tt=Tt, U=U, W_=W, C_=C, P_Yosc_=z(W.shape[0], 1), P_Xosc_=z(C.shape[0], 1),
                 T_Yosc_=z(n, 1), U_Xosc_=z(n, 1), W_Yosc=z(W.shape[0], 1), C_Xosc=z(C.shape[0], 1),
                 B_T_=B_T, B_U=B_U, H_TU=0 * Tt, H_UT=U - Tt @ B_T,
                 R2X=R2Xcorr + 0.0, R2Y=R2Ycorr + 0.0, R2Xcorr=R2Xcorr, R2Ycorr=R2Ycorr, R2Xhat=R2Xhat,
                 R2Yhat=R2Yhat)                               # :60-64 (R2X_YO = R2Y_XO = 0)
    model["flags"] = dict(time=float("nan"), n=W.shape[1], nx=0, ny=0, stripped=True, highd=False, ssqX=ssqX,
                          ssqY=ssqY, varXjoint=np.sum(Tt * Tt, axis=0), varYjoint=np.sum(U * U, axis=0),
                          varXorth=np.zeros(1), varYorth=np.zeros(1))
    model["class"] = ["o2m", "o2m_stripped"]
    return model


def PPLS_simult_to_o2m(X_true, Y_true, fit_PPLS, ctx=None):
    """PPLS_simult_to_o2m (PPLS_to_o2m.R:82-140): the fit as an OmicsPLS "o2m" list.  Host-side
    bookkeeping on the fit's Expectations (mu_T, mu_U from the device Eout) and estimates; the
    only data terms, ssq(X) and ssq(Y), come from the context (computed on the device at load)."""
    ctx = _ctx_with(X_true, Y_true, ctx)
    est, E = fit_PPLS["estimates"], fit_PPLS["Expectations"]
    W, C = np.asarray(est["W"]), np.asarray(est["C"])
    r = W.shape[1]
    B_T = np.asarray(est["B"])
    Tt, U = np.asarray(E["mu_T"]), np.asarray(E["mu_U"])
    p, q = W.shape[0], C.shape[0]
    sT, B = np.asarray(est["sigT"]), np.asarray(est["B"])
    sE, sF, sH = float(est["sigE"]), float(est["sigF"]), float(est["sigH"])

    def ssq(A):
        A = np.asarray(A, dtype=np.float64)
        return float(np.sum(A * A))
    ssqX, ssqY = ctx.ssq()
    R2Xcorr = ssq(sT @ sT) / (ssq(sT @ sT) + p * sE ** 2)
    v = sT @ sT @ B @ B + np.diag(np.full(r, sH ** 2))
    R2Ycorr = ssq(v) / (ssq(v) + q * sF ** 2)
    R2Yhat = ssq(sT @ sT @ B) / (ssq(sT @ sT @ B @ B) + r * sH ** 2 + q * sF ** 2)
    P_Yosc = np.zeros((p, 1))
    P_Xosc = np.zeros((q, 1))
    model = dict(Tt=Tt, U=U, W_=W, C_=C, P_Yosc_=P_Yosc, P_Xosc_=P_Xosc, T_Yosc_=np.zeros((Tt.shape[0], 1)),
                 U_Xosc_=np.zeros((Tt.shape[0], 1)), W_Yosc=np.zeros((p, 1)), C_Xosc=np.zeros((q, 1)),
                 B_T_=B_T, B_U=np.linalg.inv(B_T), H_TU=0 * Tt, H_UT=U - Tt @ B_T,
                 R2X=R2Xcorr + 0, R2Y=R2Ycorr + 0, R2Xcorr=R2Xcorr, R2Ycorr=R2Ycorr, R2Xhat=float("nan"),
                 R2Yhat=R2Yhat)
    model["flags"] = dict(time=float("nan"), n=r, nx=0, ny=0, stripped=True, highd=False, ssqX=ssqX, ssqY=ssqY,
                          varXjoint=np.sum(Tt * Tt, axis=0), varYjoint=np.sum(U * U, axis=0),
                          varXorth=np.zeros(1), varYorth=np.zeros(1))
    model["class"] = ["o2m", "o2m_stripped"]
    return model


def _populations(Ipopu, n):
    """as.factor(Ipopu) -> level counts in level order (table(Ipopu)); R sorts the levels."""
    Ipopu = np.asarray(Ipopu)
    if Ipopu.ndim != 1 or Ipopu.shape[0] != n:
        raise ValueError("nrow(X) == length(Ipopu) is not TRUE")   # stopifnot (:448, :511)
    levels, counts = np.unique(Ipopu, return_counts=True)
    return levels, counts.astype(np.int64)


def _params_list(levels, P):
    return [dict(B_T=float(P[j, 0]), sigX=float(P[j, 1]), sigY=float(P[j, 2]), sigH=float(P[j, 3]),
                 sigT=float(P[j, 4])) for j in range(len(levels))]


def _params_matrix(params):
    return np.array([[float(np.ravel(pp[k])[0]) for k in ("B_T", "sigX", "sigY", "sigH", "sigT")]
                     for pp in params])


def meta_EMstep(X, Y, W, C, Ipopu, params, ctx=None):
    """meta_EMstep (EM_W_multi.R:446-485) on the GPU: one EM step of the multi-population rank-1
    model.  ``params``: one dict per population (B_T, sigX, sigY, sigH, sigT), in level order.
    Returns the reference's list: per population dict(B, sighat, siglathat, Cxt, Cyu), plus
    ``W.`` and ``C.`` (shared loadings, orth of the sign-aligned sums, :481-482)."""
    ctx = _ctx_with(X, Y, ctx)
    levels, counts = _populations(Ipopu, ctx.n_total)
    if len(params) != len(levels):
        raise ValueError(f"{len(params)} parameter sets for {len(levels)} populations")
    Wo, Co, P, cxt, cyu = ctx.meta_emstep(W, C, counts, _params_matrix(params))
    out = [dict(B=P[j, 0], sighat=P[j, 1:3].copy(), siglathat=P[j, 3:5].copy(), Cxt=cxt[:, j].copy(),
                Cyu=cyu[:, j].copy()) for j in range(len(levels))]
    return dict(pops=out, **{"W.": Wo.reshape(-1, 1), "C.": Co.reshape(-1, 1)})


def meta_PPLSi(X, Y, Ipopu, EMsteps=100, atol=1e-4, initialGuess=("equal", "o2m", "random", "custom"),
               customGuess=None, critfunc=None, constraints=None, rng=None, ctx=None):
    """meta_PPLSi (EM_W_multi.R:509-589) on the GPU: a rank-1 PPLS fit with loadings shared across
    populations and per-population scalars.  Returns the reference's list (W, C, params, log) where
    ``log`` is logvalue[1:i+1, ] (rows 2..i+1 of the trace: the per-population log-likelihoods after
    each step; kept 2-D) and, additionally, ``logvalue`` (the full trace incl. the initial row).
    critfunc: None/identity or abs.  constraints: dict with numeric "W" / "C" (the only constraints
    the reference applies, :543-544)."""
    ctx = _ctx_with(X, Y, ctx)
    levels, counts = _populations(Ipopu, ctx.n_total)
    kind = initialGuess if isinstance(initialGuess, str) else initialGuess[0]
    if customGuess is not None:
        kind = "custom"
    if kind == "custom":
        g = customGuess
        init = dict(W=np.ravel(g["W"]), C=np.ravel(g["C"]), B=g["B"], sigE=g["sigE"], sigF=g["sigF"],
                    sigH=g["sigH"], sigT=g["sigT"])
    elif kind == "o2m":
        init = o2m_guess_from_gram(_joint_gram(ctx), ctx.n_total, ctx.p, ctx.q)   # :520-525
    else:
        init = initial_guess(ctx.p, ctx.q, kind, rng if rng is not None else np.random.default_rng())
    if constraints:
        if constraints.get("W") is not None:
            init["W"] = np.ravel(np.asarray(constraints["W"], dtype=np.float64))
        if constraints.get("C") is not None:
            init["C"] = np.ravel(np.asarray(constraints["C"], dtype=np.float64))
    if critfunc is None or critfunc is (lambda x: x) or getattr(critfunc, "__name__", "") == "identity":
        crit_abs = False
    elif critfunc in (abs, np.abs):
        crit_abs = True
    else:
        raise NotImplementedError("critfunc must be the identity (default) or abs")
    W, C, P, lg = ctx.meta_ppls(counts, int(EMsteps), float(atol), init, crit_abs)
    return dict(W=W, C=C, params=_params_list(levels, P), log=lg[1:], logvalue=lg)


def variances_PPLS_simult(fit, data, XorY=("X", "Y"), ctx=None, full=True):
    """variances.PPLS_simult (EM_W_multi.R:830-860) on the GPU: asymptotic standard errors of the
    loadings.  ``fit``: a PPLS_simult list (Expectations, estimates); ``data``: X (XorY = "X") or Y
    (XorY = "Y"), or None to use the context's resident X / Y.  Returns the reference's list: per
    component dict(B_exp, SSt_exp, SSt_star), then varMatrix (list of p x p) and seLoad (p x a);
    full=False skips the p x p B_exp / SSt_exp / SSt_star matrices (B_exp is then its scalar).
    The reference's t(X) %*% diag(Ctt, N) %*% X is Ctt X'X, computed once on MFMA; like the reference
    it uses estimates$sigE for XorY = "Y" as well."""
    if isinstance(XorY, (list, tuple)):
        raise ValueError("the condition has length > 1")   # if(XorY=="X") with the default c("X","Y")
    if XorY not in ("X", "Y"):
        return None                                        # neither branch: W undefined in R
    xory = 0 if XorY == "X" else 1
    E = fit["Expectations"]
    mu = np.asarray(E["mu_T"] if xory == 0 else E["mu_U"])
    Cd = np.diag(np.asarray(E["Ctt"] if xory == 0 else E["Cuu"]))
    sigE = float(np.ravel(fit["estimates"]["sigE"])[0])
    own = None
    if data is not None:
        D = np.asarray(data, dtype=np.float64)
        own = Context(0) if ctx is None else ctx
        dummy = np.zeros((D.shape[0], 1))
        own.set_data(D, dummy) if xory == 0 else own.set_data(dummy, D)
        c = own
    else:
        c = ctx or default_context()
    try:
        W, Bx, V, se, SE, SS = c.variances(mu, Cd, sigE, xory, full)
    finally:
        if own is not None and ctx is None:
            own.close()
    p = W.shape[0]
    comps = [dict(B_exp=(Bx[i] * np.eye(p) if full else float(Bx[i])),
                  SSt_exp=(SE[i] if full else None), SSt_star=(SS[i] if full else None)) for i in range(len(Bx))]
    return dict(components=comps, varMatrix=[V[i] for i in range(len(Bx))], seLoad=se, W=W)


def PPLS_simult(X, Y, a, EMsteps=10, atol=1e-4, type=("SVD", "QR"), init=None, ctx=None, **kw):
    """PPLS_simult (EM_W_multi.R:758-807) on the GPU.

    ``init``: dict(W, C, B, sigE, sigF, sigH, sigT) used as theta0.  Default: the reference's own
    f0 = PPLS(X, Y, a, 20, 1e-4, 'random') (:762-770, retried when it raises, up to three times),
    computed on the device; its draws come from ``rng`` (an R-compatible stream, see
    ``initial_guess``) or numpy (``seed`` keyword).  Returns dict(Expectations, loglik, estimates) like
    the R list of class "PPLS_simult"; warns "Negative increments of likelihood" where the
    reference does (:801).  ``timings`` (keyword, a dict): filled with the wall seconds of the
    initialiser (``init``) and of the loop + Expectations (``loop``) and the initialiser's steps.
    """
    if kw.get("debug"):
        raise NotImplementedError("debug=TRUE is an oracle-only cross-check")
    timings = kw.get("timings")   # optional dict: init / loop seconds and the initialiser's steps
    t0 = time.perf_counter()
    ctx = _ctx_with(X, Y, ctx)
    t = _orth_type(type)
    init_steps = []
    if init is None:
        rng = kw.get("rng")
        rng = rng if rng is not None else np.random.default_rng(kw.get("seed"))
        f0, last = None, None
        for _ in range(3):   # f0 = try(PPLS(...)): retried only when PPLS raises (:762-764)
            try:
                with warnings.catch_warnings():
                    warnings.simplefilter("ignore")
                    f0 = PPLS(None, None, a, 20, 1e-4, "random", rng=rng, ctx=ctx)
                break
            except PplsError as e:
                f0, last = None, e
        if f0 is None:   # R: f0 is a try-error and `f0$W` stops the call (:765)
            raise PplsError(last.code, f"f0 = try(PPLS(X, Y, a, 20, 1e-4, 'random')) failed three times "
                                       f"(EM_W_multi.R:762-765): {last}")
        if len(f0["B"]) < a:
            # R carries the truncated f0 on and fails at W.[, rotLoad] (:773-776)
            raise PplsError(-1, f"subscript out of bounds: PPLS returned {len(f0['B'])} of {a} components")
        init = dict(W=f0["W"], C=f0["C"], B=np.diag(f0["B"]), sigE=f0["sig"][a - 1, 0],
                    sigF=f0["sig"][a - 1, 1], sigH=f0["sig"][a - 1, 2], sigT=np.diag(f0["sig"][:, 3]))
        init_steps = list(f0["Other_output"]["Number_steps"])
    t1 = time.perf_counter()
    th = Theta(init["W"], init["C"], init["B"], init["sigE"], init["sigF"], init["sigH"], init["sigT"])
    if th.r != a:
        raise ValueError(f"init has {th.r} components, a = {a}")
    est, ll, eout, neg = ctx.em_run(th, int(EMsteps), float(atol), t, want_eout=True, want_mu=True)
    if neg:
        warnings.warn("Negative increments of likelihood")
    d = est.as_dict()
    estimates = dict(W=d["W"], C=d["C"], B=d["B"], sigE=d["sigE"], sigF=d["sigF"], sigH=d["sigH"],
                     sigT=d["sigT"])
    out = dict(Expectations=eout.as_dict(), loglik=ll, estimates=estimates)
    out["class"] = "PPLS_simult"
    if timings is not None:
        timings.update(init=t1 - t0, loop=time.perf_counter() - t1, init_steps=init_steps)
    return out
