"""Summarise tools/pmc_compute.sh: per kernel, counter-based MFMA / VALU utilisation and fp64 rates.

    python tools/pmc_compute_summary.py <tag> <workload> <kernel_substring,...> [--trace <stats.csv>]

Definitions (gfx950, 256 CUs x 4 SIMDs; rocprofv3 sums a dispatch's counters over XCDs/SEs):
  cycles      = GRBM_GUI_ACTIVE / 8                (the kernel's duration in GPU cycles, per XCD)
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles)         (= rocprofv3's MfmaUtil)
  valu_busy   = SQ_ACTIVE_INST_VALU / (256 CUs x cycles)                  (= rocprofv3's VALUBusy)
  fp64 flops  = 64 x (2 FMA_F64 + ADD_F64 + MUL_F64) + 512 x MFMA_MOPS_F64
  effective clock = cycles / kernel duration (from --trace, rocprofv3 kernel stats of the same run).
Writes profiles/pmc_compute_<workload>.json.
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))



def profiled_tree():
    """The source tree the profiled run used: PPLS_PROFILED_TREE if set, else this checkout's HEAD
    (+ "-dirty" when it has uncommitted changes) -- the summaries are written right after the
    gpurun call that profiled this same tree."""
    import subprocess
    t = os.environ.get("PPLS_PROFILED_TREE")
    if t:
        return t
    try:
        h = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], cwd=ROOT, capture_output=True, text=True,
                           check=True).stdout.strip()
        dirty = subprocess.run(["git", "status", "--porcelain", "--untracked-files=no"], cwd=ROOT,
                               capture_output=True, text=True).stdout.strip()
        return h + ("-dirty" if dirty else "")
    except (OSError, subprocess.CalledProcessError):
        return None

def load(path, sub, ordinals=None):
    """{counter: average per dispatch} over the dispatches of kernels whose name contains sub (only
    those at the given ordinal positions in dispatch order, when ordinals is given)."""
    acc = defaultdict(lambda: defaultdict(float))
    names = set()
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            names.add(r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0])
    if ordinals is not None:
        acc = {k: {d: v[d] for i, d in enumerate(sorted(v, key=int)) if i in ordinals} for k, v in acc.items()}
    return {k: sum(v.values()) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}, names


def main():
    args = sys.argv[1:]
    traces = []   # kernel-stats CSVs; the first that names a kernel gives its duration
    while "--trace" in args:
        i = args.index("--trace")
        traces.append(args[i + 1])
        del args[i:i + 2]
    ordinals = {}   # kernel substring -> ordinals of its timed launches (tools/timed_launches.py)
    while "--ordinals" in args:
        i = args.index("--ordinals")
        sub, path = args[i + 1].split("=", 1)
        with open(path) as f:
            ordinals[sub] = set(json.load(f)["ordinals"]["timed"])
        del args[i:i + 2]
    tag, workload, subs = args[0], args[1], args[2].split(",")
    base = os.path.join(ROOT, "gpurun_out", f"pmcc_{tag}")
    out = dict(workload=workload, kernels={}, definitions=__doc__.split("Definitions")[1].split("Writes")[0].strip(),
               source=f"tools/pmc_compute.sh {tag} (rocprofv3 --pmc, 2 passes, separate runs)",
               profiled_tree=profiled_tree())
    durations = {}
    for trace in traces:
        for r in csv.DictReader(open(trace)):
            durations.setdefault(r["Name"].replace("(anonymous namespace)::", "").split("(")[0], float(r["AverageNs"]))
    for sub in subs:
        c = {}
        n = {}
        names = set()
        for p in ("p1", "p2"):
            f = os.path.join(base, p, "run_counter_collection.csv")
            vals, cnt, nm = load(f, sub, ordinals.get(sub))
            names |= nm
            for k, v in vals.items():
                if k == "GRBM_GUI_ACTIVE" and k in c:
                    c[k + "_p2"] = v
                    continue
                c[k] = v
                n[k] = cnt[k]
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0
        d = dict(kernel=" / ".join(sorted(names)), dispatches=n.get("GRBM_GUI_ACTIVE"), counters=c,
                 launches_selected="timed launches only" if sub in ordinals else "every launch",
                 cycles_per_xcd=cyc,
                 mfma_busy=c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * cyc),
                 valu_busy=c.get("SQ_ACTIVE_INST_VALU", 0.0) / (256.0 * cyc))
        flops_valu = 64.0 * (2.0 * c.get("SQ_INSTS_VALU_FMA_F64", 0.0) + c.get("SQ_INSTS_VALU_ADD_F64", 0.0)
                             + c.get("SQ_INSTS_VALU_MUL_F64", 0.0))
        flops_mfma = 512.0 * c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)
        d.update(fp64_valu_flops=flops_valu, fp64_mfma_flops=flops_mfma)
        kname = next(iter(names)) if len(names) == 1 else None
        if kname and kname in durations:
            t = durations[kname] * 1e-9
            d.update(duration_ms=t * 1e3, effective_clock_ghz=cyc / t / 1e9,
                     fp64_valu_tflops=flops_valu / t / 1e12, fp64_mfma_tflops=flops_mfma / t / 1e12,
                     fp64_total_frac_of_78_6=(flops_valu + flops_mfma) / t / 78.6e12)
            if cyc / t > 2.4e9:   # a short dispatch: the counter window is longer than the kernel
                c24 = t * 2.4e9
                d.update(effective_clock_ghz=None,
                         note="GRBM_GUI_ACTIVE spans more than the kernel (short dispatch): busy fractions "
                              "against duration x 2.4 GHz given as *_at_2p4ghz (lower bounds on the clock)",
                         mfma_busy_at_2p4ghz=c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * c24),
                         valu_busy_at_2p4ghz=c.get("SQ_ACTIVE_INST_VALU", 0.0) / (256.0 * c24))
        out["kernels"][sub] = d
    path = os.path.join(ROOT, "profiles", f"pmc_compute_{workload}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    for sub, d in out["kernels"].items():
        print(sub, f"mfma_busy {d['mfma_busy']:.3f} valu_busy {d['valu_busy']:.3f}",
              {k: (round(v, 3) if v is not None else None) for k, v in d.items() if k.startswith(("fp64_", "effective", "duration", "valu_busy_at"))})
    print(path)


if __name__ == "__main__":
    main()
