"""Where the time of one whole PPLS_simult(X, Y, r) call goes (bench.py's `call` with xprod = 1: S
formed inside the call).  Run under rocprofv3 --kernel-trace --memory-copy-trace; the call is made
3 times with the markers printed between them; tools/call_timeline.py --analyze <dir> then splits the
trace of the last call into kernels, copies and gaps.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d D -o run -- python3 tools/call_timeline.py c3
    python3 tools/call_timeline.py --analyze D
"""
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(cfgname):
    import numpy as np
    from bench import CALL_SEED, CONFIGS, make_truth_and_theta0
    from ppls_amd import Context, PPLS_simult
    cfg = CONFIGS[cfgname]
    ctx = Context(0)
    if cfg.get("storage") == "f32":
        ctx.set_option("dtype", 1)
    truth, _ = make_truth_and_theta0(cfg["p"], cfg["q"], 1)
    ctx.generate_synthetic(cfg["n"], cfg["p"], cfg["q"], truth, seed=20261015)
    ctx.set_option("xprod", 1)
    marks = []
    for rep in range(3):
        ctx.xprod_release()
        ctx.synchronize()
        time.sleep(0.05)   # a gap in the trace between calls
        tm = {}
        t0 = time.perf_counter()
        PPLS_simult(None, None, cfg["r"], ctx=ctx, seed=CALL_SEED, timings=tm)
        ctx.synchronize()
        marks.append(dict(rep=rep, seconds=time.perf_counter() - t0, init=float(np.max(tm["init"])),
                          loop=float(np.max(tm["loop"]))))
    print(json.dumps(dict(config=cfg["name"], calls=marks)), flush=True)
    ctx.close()


def analyze(d):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    mt = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    ev = []
    for f in kt:
        for r in csv.DictReader(open(f)):
            ev.append(("K", r["Kernel_Name"][:70], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for f in mt:
        for r in csv.DictReader(open(f)):
            ev.append(("C", r.get("Direction", "copy"), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    ev.sort(key=lambda e: e[2])
    # calls are separated by >= 40 ms idle gaps; take the last segment
    segs, cur = [], [ev[0]]
    for e in ev[1:]:
        if e[2] - max(x[3] for x in cur[-50:]) > 40e6:
            segs.append(cur)
            cur = []
        cur.append(e)
    segs.append(cur)
    last = segs[-1]
    t0, t1 = last[0][2], max(e[3] for e in last)
    busy = {}
    for e in last:
        k = (e[0], e[1])
        busy.setdefault(k, [0, 0])
        busy[k][0] += 1
        busy[k][1] += e[3] - e[2]
    # union of busy intervals
    iv = sorted((e[2], e[3]) for e in last)
    tot, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    print(f"segments {len(segs)}; last call span {(t1 - t0) / 1e6:.2f} ms, device busy {tot / 1e6:.2f} ms, "
          f"idle {(t1 - t0 - tot) / 1e6:.2f} ms")
    for k, (n, ns) in sorted(busy.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {k[0]} {k[1]:70s} x{n:5d} {ns / 1e6:9.3f} ms")


if __name__ == "__main__":
    if sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run(sys.argv[1])
