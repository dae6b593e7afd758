"""Per-iteration timeline from a rocprofv3 kernel trace: average duration of each kernel in the EM
loop and the idle gaps between consecutive kernels.  usage: trace_gaps.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "")[:48]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # keep the EM loop: from the first sweep launch on
    first = next(i for i, r in enumerate(rows) if "sweep" in r["Kernel_Name"] or "panel" in r["Kernel_Name"])
    rows = rows[first:]
    dur = defaultdict(list)
    gap = defaultdict(list)
    prev = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = short(r["Kernel_Name"])
        dur[k].append(e - s)
        if prev is not None:
            gap[(prev[0], k)].append(s - prev[1])
        prev = (k, e)
    print("kernel durations (us): name  calls  mean")
    for k, v in dur.items():
        print(f"  {k:50s} {len(v):5d} {sum(v) / len(v) / 1e3:9.2f}")
    print("gaps between consecutive kernels (us): prev -> next  count  median")
    for (a, b), v in gap.items():
        v = sorted(v)
        print(f"  {a[:30]:30s} -> {b[:30]:30s} {len(v):5d} {v[len(v) // 2] / 1e3:8.2f}")


if __name__ == "__main__":
    main()
