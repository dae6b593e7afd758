"""bench.py -- EM iterations/s of the PPLS_simult inner loop on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|...] [--no-cpu]
                    [--comm rccl|host] [--oversubscribe] [--xprod-steps K] [--no-call]

One "step" = one EM iteration = sweep over X, Y (E-step sufficient statistics + log-likelihood of
the current theta) + deterministic reduction + [RCCL all-reduce] + finalize (M-step incl. polar
factor).  Workload: BASELINE config C3 (n = 1e6, p = q = 2000, r = 5, fp64) by default; samples
are sharded over ranks (strong scaling: n is fixed).  Data are synthetic (simulC model, Philox
normals) generated on the device before the timed region.  Rank 0 prints ONE JSON line -- or, when
the ranks disagree (theta digests, RCCL's own rank count, a non-finite log-likelihood), nothing on
stdout, the reason on stderr and exit status 3.

Beside the headline: the cross-product form of the same iterations ("xprod"), and the whole
user-facing call PPLS_simult(X, Y, r) with its defaults ("call": the 'random' PPLS(X, Y, r, 20,
1e-4) initialiser, EMsteps = 10, atol = 1e-4, Expectations) under each statistics path, with the
C restatement of the same call timed on a row sample of the host.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    "c3": dict(n=1_000_000, p=2000, q=2000, r=5, name="C3: n=1e6, p=q=2000, r=5, fp64 (headline)"),
    "c2": dict(n=100_000, p=1000, q=1000, r=3, name="C2: n=1e5, p=q=1000, r=3, fp64"),
    "c5": dict(n=500_000, p=10_000, q=500, r=10, storage="f32",
               name="C5: n=5e5, p=1e4, q=500, r=10, fp32 storage / fp64 arithmetic (wide-p omics case)"),
    "c5d": dict(n=500_000, p=10_000, q=500, r=10, name="C5 shape in fp64 storage"),
    # one GPU's share of C5 over 8 GPUs (n = 6.25e4 of 5e5), fp32 storage, no all-reduce
    "c5s": dict(n=62_500, p=10_000, q=500, r=10, storage="f32",
                name="C5 per-GPU shard (n=6.25e4 of 5e5), fp32 storage, no all-reduce"),
    # one GPU's share of C4 (C3 over 8 GPUs): the per-GPU sweep + fixed per-iteration costs, no all-reduce
    "c4s": dict(n=125_000, p=2000, q=2000, r=5, name="C4 per-GPU shard (n=1.25e5 of C3's 1e6), fp64, no all-reduce"),
}
METRIC = "EM iterations/sec + log-lik rel-err vs CPU ref, n=1e6 p=q=2000 r=5"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
READ_CEILING_GBS = 6848.0   # measured read-only ceiling, profiles/r1_read_bw_probe.txt (tools/read_bw_probe.hip)
MALL_REREAD_GBS = 6800.0    # measured re-read of a 128 MB (MALL-resident) buffer, low end of 6.8-7.8 TB/s
                            # (profiles/r3_mall_read_probe.txt, tools/mall_read_probe.hip)
FP64_PEAK_TF = 78.6     # MI355X fp64 vector (= fp64 MFMA) dense peak, TFLOP/s
INT8_PEAK_TOPS = 5000.0  # MI355X int8 MFMA dense peak (2x BF16's 2.5 PF, MI355X_MICROARCH.md:435), TOP/s
CALL_SEED = 20261017    # numpy stream of the 'random' initial guesses of the timed PPLS_simult calls
READBACK = "readback of a committed rocprofv3 PMC summary under profiles/ (not measured in this run)"


class _Markers:
    """roctx ranges around the bench's phases when PPLS_ROCTX=1 (a rocprofv3 --marker-trace run):
    tools/timed_launches.py then splits the kernel trace into the balance calibration, warm-up,
    timed, cross-product and whole-call launches.  Without the variable nothing is loaded."""

    def __init__(self):
        self.lib = None
        if os.environ.get("PPLS_ROCTX") != "1":
            return
        import ctypes
        for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                self.lib = lib
                break
            except (OSError, AttributeError):
                continue

    def push(self, label):
        if self.lib is not None:
            self.lib.roctxRangePushA(f"bench:{label}".encode())

    def pop(self):
        if self.lib is not None:
            self.lib.roctxRangePop()


MARK = _Markers()


def polar(M):
    U, _, Vt = np.linalg.svd(M, full_matrices=False)
    return U @ Vt


def make_truth_and_theta0(p, q, r):
    """Truth: t_k = exp(-0.1(k-1)), b_k = exp(log 1.5 - 0.3(k-1)), sigE = sigF = 0.5,
    sigH = 0.1, W/C = polar(N(0,1)) seeds 1/2; theta0: W0/C0 = polar(N(0,1)) seeds 3/4, B0 = sigT0 = I,
    sigmas 1."""
    from ppls_amd import Theta
    k = np.arange(r)
    W = polar(np.random.default_rng(1).standard_normal((p, r)))
    C = polar(np.random.default_rng(2).standard_normal((q, r)))
    truth = Theta(W, C, np.exp(np.log(1.5) - 0.3 * k), 0.5, 0.5, 0.1, np.exp(-0.1 * k))
    W0 = polar(np.random.default_rng(3).standard_normal((p, r)))
    C0 = polar(np.random.default_rng(4).standard_normal((q, r)))
    th0 = Theta(W0, C0, np.ones(r), 1.0, 1.0, 1.0, np.ones(r))
    return truth, th0


def _profile_json(name):
    try:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def _source(name, js):
    """Where a committed number came from: the file, the source tree the profiled run used (when
    the summary records it) and its own description."""
    return dict(file=f"profiles/{name}", profiled_tree=js.get("profiled_tree"), recorded=js.get("source"),
                kind=READBACK)


def load_traffic(workload_key):
    """(HBM bytes per sweep launch, provenance) from a committed rocprofv3 PMC pass, or (None, None)."""
    name = f"pmc_sweep_{workload_key}.json"
    js = _profile_json(name)
    if not js or js.get("hbm_bytes_per_launch") is None:
        return None, None
    return js["hbm_bytes_per_launch"], _source(name, js)


def load_xprod_traffic(config):
    """(Read bytes per launch of the cross-product tile kernel, provenance) from a committed
    rocprofv3 PMC pass (profiles/pmc_xprod_<config>_dp1.json), or (None, None)."""
    name = f"pmc_xprod_{config}_dp1.json"
    js = _profile_json(name)
    for kname, k in ((js or {}).get("kernels") or {}).items():
        if "pass" in kname or "tile" in kname:
            return k.get("read_bytes_per_launch"), _source(name, js)
    return None, None


def load_timed_profile(config):
    """The committed rocprofv3 kernel trace of this bench command (tools/r6_profiles.sh,
    tools/timed_launches.py): the timed launches' average duration and roofline, split from the
    warm-up and every other phase by roctx ranges -- a readback, or None."""
    name = f"r6{config}_timed_launches.json"
    js = _profile_json(name)
    if not js:
        return None
    t = js["phases"]["timed"]
    return dict(file=f"profiles/{name}", profiled_tree=js.get("profiled_tree"), command=js.get("command"),
                kernel=js.get("kernel"), timed_launches=t["launches"], avg_ms=t["avg_ms"], min_ms=t["min_ms"],
                max_ms=t["max_ms"], frac=t.get("frac"), line_of_that_run=js.get("bench_line"),
                check=js.get("check"), kind=READBACK.replace("PMC summary", "kernel trace"))


def load_compute_counters(workload_key, kernel_sub):
    """Counter-based MFMA / VALU utilisation of a kernel from a committed rocprofv3 PMC pass
    (profiles/pmc_compute_<workload>.json, tools/pmc_compute.sh + pmc_compute_summary.py), or None."""
    name = f"pmc_compute_{workload_key}.json"
    js = _profile_json(name)
    k = ((js or {}).get("kernels") or {}).get(kernel_sub)
    if not k:
        return None
    return dict(mfma_busy=k["mfma_busy"], valu_busy=k["valu_busy"], effective_clock_ghz=k.get("effective_clock_ghz"),
                fp64_valu_tflops=k.get("fp64_valu_tflops"), fp64_mfma_tflops=k.get("fp64_mfma_tflops"),
                source=dict(_source(name, js), kernel=kernel_sub))


def affinity_cores():
    """The CPUs this process may run on (its affinity mask; os.cpu_count() without one)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cgroup_cpus():
    """The cgroup v2 CPU quota in CPUs (cpu.max "quota period"), or None when unlimited / absent."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else max(1, int(int(quota) // int(period)))
    except (OSError, ValueError):
        return None


def usable_cores():
    """All the CPU this process can use: its affinity mask, capped by the cgroup CPU quota.  On the
    GPU box the mask holds 256 CPUs but cpu.max grants 16: 256 OpenMP threads there ran the C3
    baseline at 0.21 it/s against 0.63 it/s on 16 (profiles/r6_bench_c3_first.log, round 6) --
    threads beyond the quota only queue for it."""
    q = cgroup_cpus()
    return min(affinity_cores(), q) if q else affinity_cores()


def host_cores():
    """What "all cores" means on this host: the machine's CPUs (os.cpu_count = nproc without an
    affinity mask), the CPUs this process may run on (its affinity mask), the inherited
    OMP_NUM_THREADS, and the cgroup CPU quota (cpu.max: a quota below the mask caps what more
    threads can buy)."""
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota = f.read().strip()
    except OSError:
        pass
    return dict(nproc=os.cpu_count(), affinity=affinity_cores(), omp_num_threads_env=os.environ.get("OMP_NUM_THREADS"),
                cgroup_cpu_max=quota, usable=usable_cores())


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(ctx, th0, cfg, iters=3, one_core_rows=100_000):
    """Time the C restatement of the reference path (oracle/cpu_ref.c: its pass structure, OpenMP
    over rows) on the host cores, on the SAME rows the GPU holds (full n, >= 3 steady-
    state iterations after one untimed iteration, OpenMP over all the CPU the process can use -- the
    affinity mask capped by the cgroup quota, whatever OMP_NUM_THREADS it inherited; the inherited
    thread count as a second figure when it differs; plus 1 core on a row sample, scaled linearly in
    n), and compare the CPU's log-likelihood trace and loadings with the GPU's first iterations
    from the same theta0."""
    from oracle import cpu_ref
    from oracle.ppls_oracle import canonicalize
    th = th0.as_dict()
    env_threads = cpu_ref.load().cpu_ref_max_threads()   # the runtime default (OMP_NUM_THREADS)
    cores = usable_cores()
    X, Y = ctx.get_data_rows()             # all rows, row-major (what cpu_ref streams)

    def timed(nthreads):   # 1 untimed iteration (faults the pages in, spins up OpenMP), then `iters`
        t0 = time.perf_counter()
        th1, ll1 = cpu_ref.em_steps(X, Y, th, 1, nthreads=nthreads)
        t_first = time.perf_counter() - t0
        t0 = time.perf_counter()
        th_cpu, ll_cpu = cpu_ref.em_steps(X, Y, th1, iters, nthreads=nthreads)
        return th_cpu, np.concatenate([ll1, ll_cpu]), time.perf_counter() - t0, t_first

    th_cpu, ll_all, dt, t_first = timed(cores)
    inherited = None
    if env_threads != cores:
        _, ll_env, dt_env, _ = timed(env_threads)
        inherited = dict(value=iters / dt_env, unit="EM iterations/s", cores=int(env_threads),
                         sample=f"the same {iters} iterations on {env_threads} OpenMP threads (the inherited "
                                f"OMP_NUM_THREADS / runtime default) in {dt_env:.1f} s",
                         loglik_equal_to_all_core_run=bool(np.array_equal(ll_env, ll_all)))
    # the whole affinity mask as OpenMP threads, when the cgroup quota caps the
    # usable CPUs below it: reported beside the value, which stays the faster, quota-sized run
    affinity = None
    aff = affinity_cores()
    if aff != cores:
        _, ll_aff, dt_aff, _ = timed(aff)
        affinity = dict(value=iters / dt_aff, unit="EM iterations/s", cores=int(aff),
                        sample=f"the same {iters} iterations on {aff} OpenMP threads (every CPU of the affinity "
                               f"mask) in {dt_aff:.1f} s, time-sliced onto the cgroup's quota",
                        loglik_equal_to_value_run=bool(np.array_equal(ll_aff, ll_all)))
    # 1 core on the first rows (bounded time), per-row rate scaled to the full n
    ns = int(min(one_core_rows, X.shape[0]))
    Xs, Ys = X[:ns], Y[:ns]
    cpu_ref.em_steps(Xs, Ys, th, 1, nthreads=1)
    t0 = time.perf_counter()
    cpu_ref.em_steps(Xs, Ys, th, iters, nthreads=1)
    dt1 = time.perf_counter() - t0
    del X, Y, Xs, Ys
    # GPU on the same resident rows, same theta0, iters + 1 iterations
    ctx.set_option("xprod", 0)
    est, ll_gpu, _, _ = ctx.em_run(th0, iters + 1, -np.inf, 0, want_eout=False)
    rel = float(np.abs(ll_gpu - ll_all).max() / np.abs(ll_all).max())
    Wc, Cc, _, _ = canonicalize(th_cpu["W"], th_cpu["C"], th_cpu["B"], th_cpu["sigT"])
    werr = float(max(np.abs(est.W - Wc).max(), np.abs(est.C - Cc).max()))
    n = cfg["n"]
    one_core = iters * ns / dt1 / n
    return dict(value=iters / dt, unit="EM iterations/s", cores=int(cores), kind="port", host=host_cores(),
                sample=f"{iters} steady-state EM iterations (after 1 untimed, {t_first:.1f} s) on all n={n} rows "
                       f"in {dt:.1f} s: oracle/cpu_ref.c (reference pass structure), OpenMP {cores} threads "
                       f"(the affinity mask capped by the cgroup CPU quota), -O3 -march=native, {cpu_model()}",
                inherited_threads=inherited, affinity_threads=affinity,
                one_core=dict(value=one_core, unit="EM iterations/s", cores=1,
                              sample=f"{iters} EM iterations on the first {ns} rows in {dt1:.1f} s, 1 thread; "
                                     f"value = rows*iterations/s / n")), rel, werr


def _reduce_max(dist, torch, v):
    if dist is None:
        return v
    tt = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def bench_xprod(ctx, th0, args, barrier, tmax, r, ll_stream, t_stream):
    """The cross-product form of the same iterations (option "xprod", ppls_xprod.hip): S = [X Y]'[X Y]
    formed once (MFMA Gram of the local rows + ONE all-reduce of S), then every iteration reads S
    (8 P^2 bytes) instead of X and Y and needs no collective.  Timed like the headline: barrier +
    synchronize around the formation of S and around args.xprod_steps iterations, max over ranks."""
    barrier()
    ctx.set_option("xprod", 1)
    ctx.xprod_release()
    t0 = time.perf_counter()
    gram_ms, _ = ctx.xprod_prepare()
    barrier()
    t_setup = tmax(time.perf_counter() - t0)
    _, ar_ms, total_ms = ctx.xprod_setup_times()
    info = ctx.xprod_info(r)
    ctx.em_begin(th0)
    ctx.em_iterate(args.warmup)
    barrier()
    t0 = time.perf_counter()
    ctx.em_iterate(args.xprod_steps)   # wall clock: no events between the launches
    barrier()
    dt = tmax(time.perf_counter() - t0)
    est, ll_x = ctx.em_state()
    # the tile kernel's average duration: HIP events around a batch of back-to-back launches for the
    # final theta (an event pair around every ~20-us launch reads ~3 us long; rocprofv3 agrees with
    # the batch figure)
    launches = max(args.xprod_steps, 1)
    kms = ctx.xprod_tile_timing(launches) * launches
    k = min(len(ll_x), len(ll_stream))
    rel = float(np.abs(ll_x[:k] - ll_stream[:k]).max() / np.abs(ll_stream[:k]).max()) if k else None
    t_x = dt / args.xprod_steps
    avg_us = 1e3 * kms / max(launches, 1)
    achieved = info["bytes_per_pass"] / (avg_us * 1e-6) / 1e9 if launches else None
    # useful flops of S: the lower triangle incl. the diagonal over the real columns, n P (P + 1)
    # (P = p + q; the kernel also runs the zero padding of 128-column tiles it cannot skip)
    Pr = float(ctx.p + ctx.q)
    useful = float(ctx.n_local) * Pr * (Pr + 1.0)   # this rank's rows: its kernel's time
    gram_tf = useful / (gram_ms * 1e-3) / 1e12 if gram_ms > 0 else None
    traffic, traffic_src = load_xprod_traffic(args.config)
    gi = ctx.gram_info()
    if gi["int8"]:
        # the int8 CRT form (ppls_ozaki.hip): nmod int8 SYRKs of residue planes; the SYRK kernel's
        # rate against the int8 MFMA peak, and the whole Gram's fp64-equivalent rate (gram_tflops)
        syrk_ms = gi["ms"][1]
        tops = gi["nmod"] * useful / (syrk_ms * 1e-3) / 1e12 if syrk_ms > 0 else None
        gram_roof = dict(bound="mfma", achieved=tops, peak=INT8_PEAK_TOPS, unit="TOP/s",
                         frac=(tops / INT8_PEAK_TOPS) if tops else None,
                         kernel="ppls_oz_syrk_kernel (v_mfma_i32_32x32x32_i8), one plane per modulus",
                         ops_per_launch=gi["nmod"] * useful,
                         ops="useful: nmod n P (P + 1), P = p + q, this rank's rows",
                         fp64_equivalent_tflops=gram_tf, fp64_equivalent_frac_of_fp64_peak=(gram_tf / FP64_PEAK_TF)
                         if gram_tf else None)
        gram_path = dict(path="int8-crt", nmod=gi["nmod"], L=gi["L"],
                         ms=dict(stats_and_residues=gi["ms"][0], syrk=gi["ms"][1], crt=gi["ms"][2], total=gi["ms"][3]))
    else:
        gram_roof = dict(bound="mfma", achieved=gram_tf, peak=FP64_PEAK_TF, unit="TFLOP/s",
                         frac=(gram_tf / FP64_PEAK_TF) if gram_tf else None,
                         flops_per_launch=useful, flops="useful: n P (P + 1), P = p + q, this rank's rows",
                         tile_flops_per_launch=info["gram_flops"],
                         counters=load_compute_counters(f"{args.config}_dp1", "gram_mfma"))
        gram_path = dict(path="fp64-mfma")

    def fit_s(steps):   # a PPLS_simult loop of `steps` iterations (+1 sweep for the last loglik)
        return dict(stream=(steps + 1) * t_stream, xprod=t_setup + (steps + 1) * t_x)

    return est, ll_x, dict(
        what="cross-product form: S = [X Y]'[X Y] formed once on MFMA (+1 all-reduce of S over ranks), then each "
             "iteration reads S instead of X, Y (no per-iteration collective); same iterates, sums reordered",
        setup_s=t_setup, gram_kernel_ms=gram_ms, gram_tflops=gram_tf,
        setup_allreduce_ms=ar_ms, setup_allreduce_bytes=info["bytes_per_pass"] if ar_ms > 0 else 0,
        setup_total_ms_rank0=total_ms, gram=gram_path, gram_roofline=gram_roof,
        steps=args.xprod_steps, ms_per_step=1e3 * t_x, it_per_s=1.0 / t_x,
        roofline=dict(bound="hbm", achieved=achieved, peak=HBM_PEAK_GBS, unit="GB/s",
                      frac=(achieved / HBM_PEAK_GBS) if achieved else None,
                      # S (128 MB at C3) lives in the 256 MiB Infinity Cache between iterations: the
                      # measured re-read rate of such a buffer is the ceiling that applies there
                      measured_mall_reread=MALL_REREAD_GBS,
                      frac_of_mall_reread=(achieved / MALL_REREAD_GBS) if achieved else None,
                      kernel="xprod_tile (+ the Gram B'M in the finalize)",
                      traffic=traffic, traffic_source=traffic_src,
                      avg_kernel_us=avg_us, timing=f"HIP events around {launches} back-to-back launches",
                      bytes_per_launch=info["bytes_per_pass"],
                      rows_per_wave=info["rows_per_wave"]),
        loglik_rel_diff_vs_streaming=rel, loglik_compared=k,
        breakeven_steps=(t_setup / (t_stream - t_x)) if t_stream > t_x else None,
        fit_seconds={str(s): fit_s(s) for s in (10, 100, 1000, 10000)})


def bench_call(ctx, r, barrier, tmax):
    """The whole user-facing PPLS_simult(X, Y, r) (EM_W_multi.R:758-807) with its defaults: the
    initialiser PPLS(X, Y, r, 20, 1e-4, 'random') (:762, :229-279; draws from a fixed numpy stream),
    EMsteps = 10, atol = 1e-4, and the Expectations (mu_T, mu_U of this rank's rows copied to the
    host), through ppls_amd.PPLS_simult on the resident data.  Once per statistics path: stream
    (option xprod 0), xprod (1: S formed inside the call) and auto (-1: the cost model, S formed
    inside the call when it chooses it).  Barrier + synchronize around each call, max over ranks."""
    from ppls_amd import PPLS_simult
    out = {}
    for mode, opt in (("stream", 0), ("xprod", 1), ("auto", -1)):
        ctx.set_option("xprod", opt)
        ctx.xprod_release()   # every call pays for its own S
        tm = {}
        barrier()
        t0 = time.perf_counter()
        fit = PPLS_simult(None, None, r, ctx=ctx, seed=CALL_SEED, timings=tm)
        barrier()
        dt = tmax(time.perf_counter() - t0)
        ll = fit["loglik"]
        out[mode] = dict(seconds=dt, init_seconds=tmax(tm["init"]), loop_seconds=tmax(tm["loop"]),
                         init_steps=[int(v) for v in tm["init_steps"]], em_steps=int(len(ll)),
                         read_S=bool(ctx.xprod_info(r)["ready"]), loglik_last=float(ll[-1]))
        if out[mode]["read_S"]:
            gi = ctx.gram_info()
            out[mode]["gram"] = "int8-crt" if gi["int8"] else "fp64-mfma"
            out[mode]["gram_ms"] = gi["ms"][3] if gi["int8"] else None
        out[f"_{mode}_fit"] = fit
    ctx.set_option("xprod", 0)
    ref = out["stream"]["loglik_last"]
    for mode in ("xprod", "auto"):
        out[mode]["loglik_rel_diff_vs_stream"] = abs(out[mode]["loglik_last"] - ref) / abs(ref)
    return out


def cpu_call_baseline(ctx, r, cfg, device, rows):
    """oracle/cpu_ref.c's restatement of the same PPLS_simult(X, Y, r) call (cpu_ref_ppls_simult:
    the initialiser on explicitly deflated copies, the EM loop, Eout; the same 'random' draws) timed
    on the host cores over the first `rows` rows, its seconds scaled by n / rows (every pass is
    linear in n); and the GPU running the same call on the same rows, for parity."""
    from oracle import cpu_ref
    from ppls_amd import Context, PPLS_simult, initial_guess
    X, Y = ctx.get_data_rows(0, rows)
    rng = np.random.default_rng(CALL_SEED)
    inits = [initial_guess(cfg["p"], cfg["q"], "random", rng) for _ in range(r)]
    cores = usable_cores()
    t0 = time.perf_counter()
    est, ll, cs, secs = cpu_ref.ppls_simult_call(X, Y, r, inits, nthreads=cores)
    dt = time.perf_counter() - t0
    with Context(device) as c2:   # the GPU on the same rows, same draws (streaming statistics)
        c2.set_data(X, Y)
        fit = PPLS_simult(None, None, r, ctx=c2, seed=CALL_SEED)
    gl = fit["loglik"]
    k = min(len(gl), len(ll))
    scale = cfg["n"] / rows
    return dict(value=dt * scale, unit="seconds per PPLS_simult call (scaled to n)", cores=int(cores), kind="port",
                host=host_cores(),
                sample=f"PPLS_simult(X, Y, {r}) with the defaults (PPLS(X, Y, {r}, 20, 1e-4) from the same 'random' "
                       f"draws, EMsteps 10, atol 1e-4, Eout) on the first {rows} of n = {cfg['n']} rows in {dt:.1f} s "
                       f"(init {secs['init']:.1f} s, loop {secs['loop']:.1f} s, Eout {secs['eout']:.2f} s; "
                       f"init steps {list(map(int, cs))}, EM steps {len(ll)}), x {scale:.0f}: oracle/cpu_ref.c, "
                       f"OpenMP {cores} threads, {cpu_model()}",
                sample_seconds=dt,
                em_steps_cpu=int(len(ll)), em_steps_gpu=int(len(gl)),
                loglik_rel_err_gpu_vs_cpu=float(np.abs(gl[:k] - ll[:k]).max() / np.abs(ll[:k]).max()) if k else None,
                W_abs_err_gpu_vs_cpu=float(np.abs(fit["estimates"]["W"] - est["W"]).max()))


_DEVICE = {}


def _rank_entry(rank, world, port, argv):
    """Child rank of spawn_ranks: the launcher's environment, then main() (before any GPU call)."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.argv = argv
    sys.exit(main())


def spawn_ranks(n, oversubscribe=False):
    """`bench.py --gpus N` without torchrun: N fresh rank processes (multiprocessing spawn), one per
    GPU, started before this process touches a GPU; returns the exit status (non-zero if any rank
    failed or fewer than N GPUs are visible).  oversubscribe: several ranks per GPU (rank % GPUs),
    for rehearsing the multi-rank flow on fewer GPUs (only with --comm host: RCCL refuses two ranks
    on one device)."""
    import multiprocessing as mp
    import socket
    import torch
    ndev = torch.cuda.device_count()   # does not initialise the GPU on this image
    if ndev < 1 or (ndev < n and not oversubscribe):
        print(f"error: --gpus {n} but only {ndev} GPU(s) visible", file=sys.stderr)
        return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank_entry, args=(r, n, port, list(sys.argv))) for r in range(n)]
    for p in procs:
        p.start()
    for p in procs:
        p.join()
    bad = [(r, p.exitcode) for r, p in enumerate(procs) if p.exitcode != 0]
    if bad:
        print(f"error: rank(s) failed (rank, exit status): {bad}", file=sys.stderr)
        return max(3 if c == 3 else 1 for _, c in bad)
    return 0


def _digest(arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()[:16]


def _theta_arrays(est, ll):
    return [est.W, est.C, est.B, est.sigT, np.array([est.sigE, est.sigF, est.sigH]), ll]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)   # C3: ~1 s timed, long enough for a GPU-busy sampler
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--sweep", type=int, default=0, help="0 auto, 3 panel")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-iters", type=int, default=3, help="timed CPU-baseline iterations (full n)")
    ap.add_argument("--cpu-call-rows", type=int, default=0,
                    help="rows of the host PPLS_simult-call sample (0: n / 20, at least 5000)")
    ap.add_argument("--timing-every", type=int, default=4,
                    help="bracket every N-th sweep of the timed region with HIP events")
    ap.add_argument("--xprod-steps", type=int, default=2000,
                    help="iterations of the cross-product form timed after the headline (0: skip it)")
    ap.add_argument("--no-call", action="store_true", help="skip the whole-call PPLS_simult timings")
    ap.add_argument("--gram-int8", type=int, default=None, choices=[0, 1],
                    help="the Gram that forms S for the xprod / call sections: 1 the int8-MFMA CRT form "
                         "(ppls_ozaki.hip), 0 the fp64 MFMA Gram (default: the library's default)")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                    help="N>1 statistics all-reduce: RCCL (default) or the host reducer hook over gloo "
                         "(ppls_set_reducer; rehearses the multi-rank bench with several ranks on one GPU)")
    ap.add_argument("--oversubscribe", action="store_true",
                    help="with --comm host: allow more ranks than visible GPUs (rank r on GPU r % count)")
    args = ap.parse_args()
    if args.oversubscribe and args.comm != "host":
        print("error: --oversubscribe needs --comm host (RCCL refuses two ranks on one GPU)", file=sys.stderr)
        return 2

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus, args.oversubscribe)   # no launcher: one child process per GPU (spawn, no exec)
    if world != args.gpus:
        print(f"error: {world} rank(s) (WORLD_SIZE) but --gpus {args.gpus}", file=sys.stderr)
        return 2
    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo: barriers, max-over-ranks, RCCL id exchange
        dist.init_process_group("gloo")

    import torch
    from ppls_amd import Context

    cfg = CONFIGS[args.config]
    n, p, q, r = cfg["n"], cfg["p"], cfg["q"], cfg["r"]
    ndev = max(1, torch.cuda.device_count())   # does not initialise the GPU
    if world > ndev and not args.oversubscribe:
        print(f"error: {world} ranks on {ndev} GPU(s) (use --oversubscribe with --comm host)", file=sys.stderr)
        return 2
    device = local % ndev
    ctx = Context(device)
    _DEVICE[id(ctx)] = device
    if cfg.get("storage") == "f32":
        ctx.set_option("dtype", 1)
    ctx.set_option("sweep", args.sweep)
    if args.gram_int8 is not None:
        ctx.set_option("gram_int8", args.gram_int8)
    if world > 1 and args.comm == "rccl":
        uid = [Context.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(world, rank, uid[0])
    elif world > 1:
        def host_allreduce(buf):   # the library's host staging buffer, summed in place over gloo
            dist.all_reduce(torch.from_numpy(buf))
        ctx.set_reducer(host_allreduce)
    row0, n_local = Context.shard_range(n, world, rank)
    truth, th0 = make_truth_and_theta0(p, q, r)
    ctx.generate_synthetic(n, p, q, truth, seed=20261015, row0=row0, n_local=n_local)

    if torch.cuda.is_available():
        torch.cuda.set_device(device)   # torch.cuda.synchronize() below then waits on this rank's GPU

    def barrier():
        ctx.synchronize()
        if torch.cuda.is_available():
            torch.cuda.synchronize(device)
        if dist is not None:
            dist.barrier()

    def tmax(v):
        return _reduce_max(dist, torch, v)

    MARK.push("em_begin")   # the split sweep's balance calibration launches run here
    ctx.em_begin(th0)
    barrier()
    MARK.pop()
    MARK.push("warmup")
    ctx.em_iterate(args.warmup)
    barrier()
    MARK.pop()
    ctx.set_option("timing", args.timing_every)
    ctx.sweep_timing(reset=True)
    MARK.push("timed")
    t0 = time.perf_counter()
    ctx.em_iterate(args.steps)
    barrier()
    dt = tmax(time.perf_counter() - t0)
    MARK.pop()
    ctx.set_option("timing", 0)
    kern_ms, launches = ctx.sweep_timing(reset=True)
    est, ll = ctx.em_state()
    info = ctx.sweep_info(r)
    rccl_nranks, rccl_rank, ar_ms, ar_calls = ctx.comm_info(reset=True)
    digest_parts = _theta_arrays(est, ll)
    xp = None
    if args.xprod_steps > 0:
        MARK.push("xprod")
        est_x, ll_x, xp = bench_xprod(ctx, th0, args, barrier, tmax, r, ll, dt / args.steps)
        MARK.pop()
        digest_parts += _theta_arrays(est_x, ll_x)
        ctx.set_option("xprod", 0)
    call = None
    if not args.no_call:
        MARK.push("call")
        call = bench_call(ctx, r, barrier, tmax)
        MARK.pop()
        for mode in ("stream", "xprod", "auto"):
            f = call.pop(f"_{mode}_fit")
            e = f["estimates"]
            digest_parts += [e["W"], e["C"], e["B"], e["sigT"], np.array([e["sigE"], e["sigF"], e["sigH"]]), f["loglik"]]
    # every rank's theta and traces (headline, cross-product, calls) hashed: a dp-N run proves its
    # ranks stayed identical, and fails loudly when they did not (PPLS_BENCH_TEST_DIVERGE = a rank:
    # that rank's digest is perturbed -- tests/test_gpu_bench.py checks the failure path)
    if os.environ.get("PPLS_BENCH_TEST_DIVERGE") == str(rank):
        digest_parts.append(np.ones(1))
    digest = _digest(digest_parts)
    digests = [digest]
    # per rank: its sweep kernel's average (HIP events), its statistics all-reduce (RCCL: events
    # around the collective) and the all-reduce of S -- a scaling run shows load balance and
    # collective cost without re-profiling
    mine = dict(sweep_kernel_ms=kern_ms / max(launches, 1) if launches else None,
                allreduce_us=(1e3 * ar_ms / ar_calls) if ar_calls else None,
                xprod_setup_allreduce_ms=xp["setup_allreduce_ms"] if xp else None,
                xprod_gram_kernel_ms=xp["gram_kernel_ms"] if xp else None, rows=n_local)
    ranks = [mine]
    if dist is not None:
        digests = [None] * world
        dist.all_gather_object(digests, digest)
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    backend = "none" if world == 1 else ("rccl" if args.comm == "rccl" else "host reducer over gloo")
    problems = []
    if len(set(digests)) != 1:
        problems.append(f"ranks hold different estimates (theta digests {digests})")
    if backend == "rccl" and rccl_nranks != world:
        problems.append(f"RCCL reports {rccl_nranks} ranks for a world of {world}")
    if not (len(ll) and np.isfinite(ll).all()):
        problems.append("non-finite log-likelihood")
    if problems:
        if rank == 0:
            print("error: " + "; ".join(problems), file=sys.stderr)
        ctx.close()
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return 3

    if rank == 0:
        its = args.steps / dt
        avg_kernel_ms = kern_ms / max(launches, 1)
        achieved = info["bytes_per_sweep"] / (avg_kernel_ms * 1e-3) / 1e9 if launches else None
        wl = f"{args.config}_{'dp%d' % world}"
        stat_doubles = (p + q) * r + 4 * r * r      # [X'mu_T | Y'mu_U | Gram], one all-reduce per iteration
        if world == 1:
            parallelism = "dp1 (single rank, no all-reduce)"
        else:
            parallelism = (f"dp{world} (rows sharded, 1 {'RCCL' if args.comm == 'rccl' else 'host (gloo)'} "
                           f"all-reduce of {stat_doubles} doubles/iteration"
                           f"{'; ranks oversubscribed on ' + str(ndev) + ' GPU(s)' if world > ndev else ''})")
        # compute side: 2r fp64 FMAs per element (r for the dots, r for the rank-1 update), on
        # VALU (no fp64 MFMA shape fits r <= 8 better, and its rate equals the VALU rate)
        flops = 4.0 * (n_local * (p + q)) * r
        tflops = flops / (avg_kernel_ms * 1e-3) / 1e12 if launches else None
        traffic, traffic_src = load_traffic(wl)
        roofline = dict(bound="hbm", achieved=achieved, peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=(achieved / HBM_PEAK_GBS) if achieved else None,
                        traffic=traffic, traffic_source=traffic_src, kernel=ctx.sweep_kernel(r),
                        avg_kernel_ms=avg_kernel_ms, bytes_per_launch=info["bytes_per_sweep"],
                        grid=info["grid"], fp64_valu_tflops=tflops, fp64_valu_peak_tflops=FP64_PEAK_TF,
                        fp64_valu_frac=(tflops / FP64_PEAK_TF) if tflops else None,
                        measured_read_ceiling=READ_CEILING_GBS,
                        frac_of_measured_ceiling=(achieved / READ_CEILING_GBS) if achieved else None,
                        profile=load_timed_profile(args.config) if world == 1 else None)
        # rocprofv3 PMC counters (SQ_VALU_MFMA_BUSY_CYCLES, SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE) of the
        # sweep kernel(s) at this workload, committed under profiles/ (readbacks, see their source)
        if info["variant"] == "panel":
            roofline["counters"] = {k: load_compute_counters(wl, k) for k in ("panel_mfmadots", "panel_acc")}
        else:
            roofline["counters"] = {"sweep_split": load_compute_counters(wl, "sweep_split")}
        if xp is not None:
            # the north star's "MFMA utilisation on the M-step GEMMs": the GEMM on MFMA is the Gram that
            # forms S (every statistic of the M-step is then read off S); the streaming sweep's
            # X'mu_T runs on fp64 VALU (r = 5 fills 5 of an MFMA's 16 columns, gfx950's fp64 MFMA and
            # VALU rates are equal, and the sweep already sits at its HBM read ceiling)
            g = xp["gram_roofline"]
            gemm = ("S = [X Y]'[X Y], the cross-product form of the M-step sums X'mu_T, Y'mu_U and the E-step "
                    "Gram (EM_W_multi.R:689-690, 732-733); variances.PPLS_simult's X'X (:846) runs the same kernel")
            note = "the streaming sweep's X'mu_T / Y'mu_U run on fp64 VALU (counters.sweep_split)"
            if xp["gram"]["path"] == "int8-crt":
                roofline["mfma_gemm"] = dict(
                    gemm=gemm, kernel=g["kernel"], int8_mfma_tops=g["achieved"], peak_tops=INT8_PEAK_TOPS,
                    frac=g["frac"], syrk_ms=xp["gram"]["ms"]["syrk"], kernel_ms=xp["gram_kernel_ms"],
                    nmod=xp["gram"]["nmod"], ops=g["ops"], fp64_equivalent_tflops=g["fp64_equivalent_tflops"],
                    sweep_note=note)
            else:
                roofline["mfma_gemm"] = dict(
                    gemm=gemm, kernel="ppls_gram_mfma_kernel (v_mfma_f64_16x16x4_f64)", fp64_mfma_tflops=g["achieved"],
                    peak_tflops=FP64_PEAK_TF, frac=g["frac"], kernel_ms=xp["gram_kernel_ms"],
                    flops=g["flops"], counters=g["counters"], sweep_note=note)
        out = dict(metric=METRIC, value=its, unit="EM iterations/s", n_gpus=world, steps=args.steps,
                   warmup=args.warmup, ms_per_step=1e3 * dt / args.steps, higher_is_better=True,
                   scaling="strong", vs_baseline=None, dtype="f64",
                   storage=cfg.get("storage", "f64"),
                   data="synthetic (simulC model: X=TW'+sigE E, Y=UC'+sigF F; Philox normals on device)",
                   config=dict(workload=cfg["name"], n=n, p=p, q=q, r=r, parallelism=parallelism),
                   roofline=roofline,
                   # same theta0, warmup + steps iterations for every N: equal across dp1..dp8 to
                   # rounding (the sharded sums are reordered)
                   loglik_last=float(ll[-1]) if len(ll) else None,
                   # nranks/rank as ncclCommCount/ncclCommUserRank report them (RCCL only)
                   comm=dict(backend=backend,
                             nranks_reported=rccl_nranks if backend == "rccl" else None,
                             rank0_reported=rccl_rank if backend == "rccl" else None,
                             allreduce_doubles=stat_doubles,
                             allreduce_us=(1e3 * ar_ms / ar_calls) if ar_calls else None,
                             allreduce_timed_calls=ar_calls),
                   theta_sha16=digest, ranks_bitwise_identical=True)
        out["xprod"] = xp
        if world > 1:
            def spread(key):
                v = [rk[key] for rk in ranks]
                ok = [x for x in v if x is not None]
                return dict(min=min(ok) if ok else None, max=max(ok) if ok else None, per_rank=v)
            out["per_rank"] = {k: spread(k) for k in ("sweep_kernel_ms", "allreduce_us", "xprod_setup_allreduce_ms",
                                                      "xprod_gram_kernel_ms", "rows")}
        if call is not None:
            out["call_seconds"] = {m: call[m]["seconds"] for m in ("stream", "xprod", "auto")}
            out["call"] = dict(what=f"PPLS_simult(X, Y, {r}) with its defaults: PPLS(X, Y, {r}, 20, 1e-4, 'random') "
                                    "initialiser, EMsteps 10, atol 1e-4, Expectations to the host; S formed inside "
                                    "the xprod / auto calls", **call)
        if world == 1 and not args.no_cpu:
            MARK.push("cpu_baseline")
            cb, rel, werr = cpu_baseline(ctx, th0, cfg, args.cpu_iters)
            MARK.pop()
            out["cpu_baseline"] = cb
            out["loglik_rel_err_vs_cpu"] = rel
            out["W_abs_err_vs_cpu"] = werr
            if call is not None:
                rows = args.cpu_call_rows or max(5000, n // 20)
                out["call"]["cpu_ref"] = cpu_call_baseline(ctx, r, cfg, device, min(rows, n))
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
