"""Split a rocprofv3 kernel trace of bench.py into its phases and summarise the timed launches.

    python tools/timed_launches.py <trace_dir> --kernel <substring> --bytes <algorithmic B/launch>
                                   --name <out_stem> [--bench-json <bench stdout line file>]

bench.py run under `PPLS_ROCTX=1 rocprofv3 --kernel-trace --marker-trace --stats` pushes one roctx
range per phase: bench:em_begin (the split sweep's 8 balance-calibration launches),
bench:warmup, bench:timed (the K steps of the JSON line), bench:xprod, bench:call, bench:cpu_baseline.
Every kernel dispatch is assigned to the range its start timestamp falls in.

Writes
  profiles/<out_stem>.json            per phase: the kernel's launch count, avg / min / max duration;
                                      the timed average's roofline (bytes / avg / 8 TB/s); the ordinal
                                      positions of the timed launches among all dispatches of the
                                      kernel (tools/pmc_summary.py --ordinals uses them on the PMC
                                      runs of the same command, which dispatch the same sequence);
                                      the bench line's own ms_per_step / frac when --bench-json is given
  profiles/<out_stem>_kernel_stats.csv  rocprofv3-style stats of the timed phase only
"""
import argparse
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
HBM_PEAK = 8.0e12


def _csv(trace_dir, suffix):
    for f in sorted(os.listdir(trace_dir)):
        if f.endswith(suffix):
            return os.path.join(trace_dir, f)
    return None


def marker_ranges(path):
    """[(label, start_ns, end_ns)] of the bench:* roctx ranges (any column holding the label)."""
    out = []
    if not path:
        return out
    for r in csv.DictReader(open(path)):
        label = next((v for v in r.values() if isinstance(v, str) and v.startswith("bench:")), None)
        if label:
            out.append((label.split(":", 1)[1], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--kernel", required=True, help="substring of the dominant kernel's name")
    ap.add_argument("--bytes", type=float, required=True, help="algorithmic bytes per launch")
    ap.add_argument("--name", required=True)
    ap.add_argument("--bench-json", default=None)
    ap.add_argument("--command", default=None)
    ap.add_argument("--out-dir", default=os.path.join(ROOT, "profiles"), help="where the summaries go")
    ap.add_argument("--group", type=int, default=1,
                    help="consecutive matching launches of a phase that form one unit (their durations summed): "
                         "2 for the panel sweep's dots + accumulation per iteration (--kernel panel_)")
    a = ap.parse_args()
    kt = _csv(a.trace_dir, "kernel_trace.csv")
    ranges = marker_ranges(_csv(a.trace_dir, "marker_api_trace.csv"))
    if not kt:
        sys.exit(f"no kernel_trace.csv under {a.trace_dir}")
    if not ranges:
        sys.exit("no bench:* roctx ranges in the marker trace (run with PPLS_ROCTX=1 and --marker-trace)")
    rows = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Dispatch_Id"]))

    def phase(ts):
        for label, s, e in ranges:
            if s <= ts <= e:
                return label
        return "other"

    ordinal = 0
    per = {}          # phase -> [durations of the kernel]
    ords = {}         # phase -> [ordinals of the kernel among its dispatches]
    timed_all = {}    # every kernel of the timed phase: name -> [durations]
    for r in rows:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ph = phase(st)
        if ph == "timed":
            timed_all.setdefault(short(r["Kernel_Name"]), []).append(en - st)
        if a.kernel in r["Kernel_Name"]:
            per.setdefault(ph, []).append(en - st)
            ords.setdefault(ph, []).append(ordinal)
            ordinal += 1
    if "timed" not in per:
        sys.exit(f"no {a.kernel} launch inside bench:timed")
    if a.group > 1:   # one unit = a.group consecutive launches (e.g. one sweep = dots + accumulation)
        per = {ph: [sum(v[i:i + a.group]) for i in range(0, len(v) - a.group + 1, a.group)] for ph, v in per.items()}

    def stats(v):
        return dict(launches=len(v), avg_ms=statistics.fmean(v) / 1e6, min_ms=min(v) / 1e6, max_ms=max(v) / 1e6)

    phases = {ph: stats(v) for ph, v in per.items()}
    t = phases["timed"]
    t["achieved_GBs"] = a.bytes / (t["avg_ms"] * 1e-3) / 1e9
    t["frac"] = t["achieved_GBs"] * 1e9 / HBM_PEAK
    try:
        from pmc_summary import profiled_tree
    except ImportError:   # (the summary's provenance helper; absent in a bare checkout of the tool)
        def profiled_tree():
            return os.environ.get("PPLS_PROFILED_TREE")
    out = dict(kernel=a.kernel, launches_per_unit=a.group, algorithmic_bytes_per_launch=a.bytes, hbm_peak_GBs=HBM_PEAK / 1e9,
               command=a.command, profiled_tree=profiled_tree(), phases=phases,
               ordinals={ph: v for ph, v in ords.items()}, kernel_dispatches_total=ordinal,
               timed_iteration_kernels={k: stats(v) for k, v in timed_all.items()},
               ranges=[dict(label=lb, ms=(e - s) / 1e6) for lb, s, e in ranges])
    if a.bench_json:
        line = next(ln for ln in open(a.bench_json) if ln.startswith("{"))
        b = json.loads(line)
        out["bench_line"] = dict(ms_per_step=b["ms_per_step"], steps=b["steps"], warmup=b["warmup"],
                                 value=b["value"], avg_kernel_ms_hip_events=b["roofline"]["avg_kernel_ms"],
                                 frac=b["roofline"]["frac"])
        out["check"] = dict(
            timed_avg_le_ms_per_step=t["avg_ms"] <= b["ms_per_step"],
            frac_trace_over_line=t["frac"] / b["roofline"]["frac"],
            timed_launches_eq_steps=t["launches"] == b["steps"])
    path = os.path.join(a.out_dir, a.name + ".json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.join(a.out_dir, a.name + "_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Phase"])
        for k, v in sorted(timed_all.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([k, len(v), sum(v), statistics.fmean(v), min(v), max(v), "timed"])
    print(path, {ph: (round(s["avg_ms"], 4), s["launches"]) for ph, s in phases.items()},
          f"timed frac {t['frac']:.4f}", out.get("check"))


if __name__ == "__main__":
    main()
