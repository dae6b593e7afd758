"""Generate the golden fixtures of tests/golden/ from the CPU oracle (oracle/ppls_oracle.py).

The reference (R + Rcpp/RcppEigen + OmicsPLS) cannot run in this image, so the vectors come
from the oracle's line-by-line restatement, which tests/test_oracle.py pins against the
reference's own identity checks and dense formulation.  Run from the repo root:
    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import make_problem  # noqa: E402
from oracle import ppls_oracle as o  # noqa: E402

CASES = [
    # name, n, p, q, r, EMsteps, atol, type, seed
    ("c1_n200_p50_q50_r2", 200, 50, 50, 2, 10, float("-inf"), "SVD", 1),
    ("r1_n150_p30_q20", 150, 30, 20, 1, 10, float("-inf"), "SVD", 2),
    ("r5_n300_p41_q37", 300, 41, 37, 5, 8, float("-inf"), "SVD", 3),
    ("qr_n200_p24_q18_r3", 200, 24, 18, 3, 6, float("-inf"), "QR", 4),
    ("atol_n250_p20_q16_r2", 250, 20, 16, 2, 300, 5e-3, "SVD", 5),
    # stress variant of the simulation study's noise level sigE = sigF = 0.05 (Package/EM_Cpp.R:26-28)
    ("stress_sig005_n300_p40_q30_r3", 300, 40, 30, 3, 12, float("-inf"), "SVD", 6),
]
PROBLEM_KW = {"stress_sig005_n300_p40_q30_r3": dict(sigE=0.05, sigF=0.05, sigH=0.05)}


# sequential initialiser PPLS(X, Y, a, EMsteps, atol, initialGuess) and the PPLS_simult run it seeds
SEQ_CASES = [
    # name, n, p, q, a, EMsteps, atol, initialGuess, seed (data) , init seed ('random')
    ("seq_equal_n200_p30_q25_a3", 200, 30, 25, 3, 20, 1e-4, "equal", 11, None),
    ("seq_random_n240_p36_q20_a2", 240, 36, 20, 2, 20, 1e-4, "random", 12, 99),
    ("seq_equal_atol_n150_p16_q12_a2", 150, 16, 12, 2, 100, 1e-2, "equal", 13, None),
]


def seq_fixtures(here):
    for name, n, p, q, a, steps, atol, kind, seed, iseed in SEQ_CASES:
        X, Y, _ = make_problem(n, p, q, a, seed=seed)
        rng = np.random.default_rng(iseed) if iseed is not None else None
        inits = [o.initial_guess(p, q, kind, rng) for _ in range(a)]
        f = o.ppls(X, Y, a, steps, atol, inits)
        oo = f["Other_output"]
        lv = np.full((a, steps + 1), np.nan)
        for k, v in enumerate(oo["logvalue"]):
            lv[k, :len(v)] = v
        sim = o.ppls_simult(X, Y, a, EMsteps=10, atol=1e-4, theta0=o.simult_theta0_from_ppls(f))
        meta = dict(n=n, p=p, q=q, a=a, EMsteps=steps, atol=atol, initialGuess=kind, seed=seed,
                    init_seed=iseed)
        np.savez_compressed(
            os.path.join(here, name + ".npz"), meta=json.dumps(meta), X=X, Y=Y,
            init_W=np.stack([t["W"] for t in inits], 1), init_C=np.stack([t["C"] for t in inits], 1),
            init_s=np.array([[t["B"], t["sigE"], t["sigF"], t["sigH"], t["sigT"]] for t in inits]),
            W=f["W"], C=f["C"], B=f["B"], sig=f["sig"], logvalue=lv,
            last_increment=np.array(oo["Last_increment"]), number_steps=np.array(oo["Number_steps"]),
            loglikelihoods=np.array(oo["Loglikelihoods"]), simult_loglik=sim["loglik"],
            simult_W=sim["estimates"]["W"], simult_C=sim["estimates"]["C"])
        print(name, "steps", oo["Number_steps"], "logliks", oo["Loglikelihoods"])


# multi-population meta_PPLSi(X, Y, Ipopu, EMsteps, atol, initialGuess): shared W, C, per-population
# scalars (B, t, sigE, sigF) -- populations are contiguous row blocks in level order
META_CASES = [
    # name, pop sizes, p, q, EMsteps, atol, initialGuess, data seed, init seed ('random')
    ("meta_equal_k2_p30_q20", (120, 80), 30, 20, 100, 5e-3, "equal", 21, None),
    ("meta_random_k3_p24_q18", (100, 60, 90), 24, 18, 25, 1e-6, "random", 22, 7),
]


def meta_problem(sizes, p, q, seed):
    rng = np.random.default_rng(seed)
    w = rng.standard_normal(p)
    c = rng.standard_normal(q)
    w, c = w / np.linalg.norm(w), c / np.linalg.norm(c)
    Xs, Ys = [], []
    for j, nj in enumerate(sizes):
        t, b, sE, sF, sH = 1.0 + 0.3 * j, 1.5 - 0.4 * j, 0.5 + 0.1 * j, 0.6 - 0.05 * j, 0.2
        T = t * rng.standard_normal(nj)
        U = b * T + sH * rng.standard_normal(nj)
        Xs.append(np.outer(T, w) + sE * rng.standard_normal((nj, p)))
        Ys.append(np.outer(U, c) + sF * rng.standard_normal((nj, q)))
    return np.vstack(Xs), np.vstack(Ys)


def meta_fixtures(here):
    for name, sizes, p, q, steps, atol, kind, seed, iseed in META_CASES:
        X, Y = meta_problem(sizes, p, q, seed)
        rng = np.random.default_rng(iseed) if iseed is not None else None
        init = o.initial_guess(p, q, kind, rng)
        f = o.meta_pplsi(X, Y, list(sizes), steps, atol, init)
        P = np.array([[pp[k] for k in ("B_T", "sigX", "sigY", "sigH", "sigT")] for pp in f["params"]])
        one = o.meta_emstep(X, Y, init["W"], init["C"], list(sizes),
                            [dict(B_T=init["B"], sigX=init["sigE"], sigY=init["sigF"], sigH=init["sigH"],
                                  sigT=init["sigT"])] * len(sizes))
        meta = dict(sizes=list(sizes), p=p, q=q, EMsteps=steps, atol=atol, initialGuess=kind, seed=seed,
                    init_seed=iseed, steps=int(f["logvalue"].shape[0] - 1))
        np.savez_compressed(
            os.path.join(here, name + ".npz"), meta=json.dumps(meta), X=X, Y=Y, init_W=init["W"],
            init_C=init["C"],
            init_s=np.array([init["B"], init["sigE"], init["sigF"], init["sigH"], init["sigT"]]),
            W=f["W"], C=f["C"], params=P, logvalue=f["logvalue"],
            step1_W=one["W"], step1_C=one["C"],
            step1_params=np.array([[e["B"], *e["sighat"], *e["siglathat"]] for e in one["pops"]]),
            step1_Cxt=np.stack([e["Cxt"] for e in one["pops"]], 1),
            step1_Cyu=np.stack([e["Cyu"] for e in one["pops"]], 1))
        print(name, "steps", meta["steps"], "log", f["logvalue"][-1])


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    if "--meta" in sys.argv:   # only the meta_* fixtures (the others are unchanged)
        meta_fixtures(here)
        return
    only = None
    if "--cases" in sys.argv:   # only these PPLS_simult fixtures, e.g. --cases qr_n200_p24_q18_r3,...
        only = set(sys.argv[sys.argv.index("--cases") + 1].split(","))
    else:
        meta_fixtures(here)
        seq_fixtures(here)
    for name, n, p, q, r, steps, atol, typ, seed in CASES:
        if only is not None and name not in only:
            continue
        X, Y, th0 = make_problem(n, p, q, r, seed=seed, **PROBLEM_KW.get(name, {}))
        res = o.ppls_simult(X, Y, r, EMsteps=steps, atol=atol, type=typ, theta0=th0)
        one = o.ppls_simult(X, Y, r, EMsteps=1, atol=atol, type=typ, theta0=th0)
        two = o.ppls_simult(X, Y, r, EMsteps=2, atol=atol, type=typ, theta0=th0)
        est, E = res["estimates"], res["Expectations"]
        meta = dict(n=n, p=p, q=q, r=r, EMsteps=steps, atol=atol, type=typ, seed=seed,
                    steps_done=int(len(res["loglik"])))
        np.savez_compressed(
            os.path.join(here, name + ".npz"), meta=json.dumps(meta), X=X, Y=Y,
            W0=th0["W"], C0=th0["C"], B0=np.diag(th0["B"]), T0=np.diag(th0["sigT"]),
            sig0=np.array([th0["sigE"], th0["sigF"], th0["sigH"]]),
            loglik=res["loglik"], W=est["W"], C=est["C"], B=np.diag(est["B"]), T=np.diag(est["sigT"]),
            sig=np.array([est["sigE"], est["sigF"], est["sigH"]]),
            W1=one["estimates"]["W"], loglik1=one["loglik"], W2=two["estimates"]["W"], loglik2=two["loglik"],
            mu_T=E["mu_T"], mu_U=E["mu_U"], Ctt=np.diag(E["Ctt"]), Cuu=np.diag(E["Cuu"]),
            Cut=np.diag(E["Cut"]), Cee=E["Cee"][0, 0], Cff=E["Cff"][0, 0], Chh=E["Chh"])
        print(name, "steps", len(res["loglik"]), "loglik", res["loglik"][-1])


if __name__ == "__main__":
    main()
