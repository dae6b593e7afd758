"""Kernel timeline of the cross-product iteration from a rocprofv3 --kernel-trace CSV: per kernel
name the average duration, and for a window of consecutive iterations the start/end of every kernel
relative to the first, so gaps and overlaps between the tile / pass / apply / finalize kernels show.

    python tools/xprod_timeline.py <run_kernel_trace.csv> [first_dispatch=-60]
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
first = int(sys.argv[2]) if len(sys.argv) > 2 else -60
keys = ("xprod", "finalize")
ks = [r for r in rows if any(k in r["Kernel_Name"] for k in keys)]
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
tot = defaultdict(list)
for r in ks:
    tot[r["Kernel_Name"].split("(")[0][-60:]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in tot.items():
    print(f"{k:60s} n={len(v):5d} avg {sum(v) / len(v) / 1e3:8.2f} us")
win = ks[first:]
t0 = int(win[0]["Start_Timestamp"])
prev_end = None
for r in win:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    gap = "" if prev_end is None else f" gap {(s - prev_end) / 1e3:7.2f}"
    print(f"{s / 1e3:9.2f} .. {e / 1e3:9.2f} us  ({(e - s) / 1e3:6.2f}){gap}  {r['Kernel_Name'].split('(')[0][-50:]}")
    prev_end = e if prev_end is None else max(prev_end, e)
