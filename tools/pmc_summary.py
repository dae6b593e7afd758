"""HBM traffic per sweep launch from the rocprofv3 PMC passes written by tools/profile.sh.

    python tools/pmc_summary.py <tag> <workload> <algorithmic_bytes_per_launch> [note] [--kernels a,b]

--out <name>: write profiles/pmc_<name>.json instead (a kernel other than the sweep, e.g. the Gram).
--kernels: substrings of the kernels that make up one sweep (default "sweep"); the per-launch
traffic of each is averaged over its dispatches and the sweep's traffic is their sum (the wide-p
panel sweep is two kernels: panel_mfmadots + panel_acc).

Reads gpurun_out/prof_<tag>/pmc_{FETCH_SIZE,WRITE_SIZE}/run_counter_collection.csv and writes
profiles/pmc_sweep_<workload>.json.  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE counts half the bytes of 16 B/lane streaming reads, so read bytes = 2 x FETCH_SIZE x
1024; WRITE_SIZE (kB) is exact.
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

def load_ordinals(path, phase="timed"):
    """The ordinal positions (among the kernel's dispatches) of one phase's launches, from
    tools/timed_launches.py's summary of the kernel trace of the same command."""
    with open(path) as f:
        return set(json.load(f)["ordinals"][phase])


def keep_ordinals(acc, ordinals):
    """acc {(kernel, dispatch id): value} restricted to the dispatches whose position in dispatch
    order (per kernel name) is in ordinals (None: all)."""
    if ordinals is None:
        return acc
    out = {}
    for name in {k[0] for k in acc}:
        ids = sorted((k for k in acc if k[0] == name), key=lambda k: int(k[1]))
        out.update({k: acc[k] for i, k in enumerate(ids) if i in ordinals})
    return out


def per_launch(path, counter, subs=("sweep",), ordinals=None):
    """Sum over the kernels matching subs of the kernel's average counter value per dispatch
    (only the dispatches at the given ordinal positions, when ordinals is given)."""
    total, names, launches = 0.0, set(), 0
    for sub in subs:
        acc = defaultdict(float)
        for r in csv.DictReader(open(path)):
            if sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
                acc[(r["Kernel_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
        acc = keep_ordinals(acc, ordinals)
        names |= {k[0] for k in acc}
        launches = max(launches, len(acc))
        total += sum(acc.values()) / max(len(acc), 1)
    return names, launches, total


def main():
    args = list(sys.argv[1:])
    subs = ("sweep",)
    out_name = None
    if "--out" in args:   # another kernel than the sweep: profiles/pmc_<name>.json
        i = args.index("--out")
        out_name = args[i + 1]
        del args[i:i + 2]
    if "--kernels" in args:
        i = args.index("--kernels")
        subs = tuple(args[i + 1].split(","))
        del args[i:i + 2]
    ordinals, ord_src = None, None
    if "--ordinals" in args:   # only the timed launches (tools/timed_launches.py of the same command)
        i = args.index("--ordinals")
        ord_src = args[i + 1]
        ordinals = load_ordinals(ord_src)
        del args[i:i + 2]
    tag, workload, alg = args[0], args[1], int(float(args[2]))
    note = args[3] if len(args) > 3 else ""
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    names, n, fetch = per_launch(os.path.join(base, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE",
                                 subs, ordinals)
    _, _, write = per_launch(os.path.join(base, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE", subs,
                             ordinals)
    hbm = 2.0 * fetch * 1024 + write * 1024
    out = dict(workload=workload, kernel=" + ".join(sorted(k.split("(")[0] for k in names)) if names else None,
               launches=n,
               FETCH_SIZE_kB_per_launch=fetch, WRITE_SIZE_kB_per_launch=write,
               correction="gfx950: FETCH_SIZE counts half the bytes of 16 B/lane streaming reads "
                          "(MI355X_MICROARCH.md, HBM): read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE exact",
               hbm_bytes_per_launch=hbm, algorithmic_bytes_per_launch=alg,
               traffic_over_algorithmic=hbm / alg,
               source=f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) -- python3 bench.py; {note}",
               launches_selected=("the timed launches only (ordinals from " + os.path.basename(ord_src) + ")")
               if ord_src else "every launch of the kernel",
               profiled_tree=profiled_tree())
    path = os.path.join(ROOT, "profiles", f"pmc_{out_name}.json" if out_name else f"pmc_sweep_{workload}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, f"{hbm / alg:.4f} x algorithmic")


if __name__ == "__main__":
    main()
