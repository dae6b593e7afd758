"""The profile evidence behind the bench line's roofline, checked on the CPU:
tools/timed_launches.py on a synthetic rocprofv3 trace (phases from roctx ranges, --group for the
panel sweep's two kernels per iteration), and the committed round-6 summaries against the bench
line of the run they profiled (timed launches = steps, their average <= ms per step, the trace's
frac within 1 % of the line's, PMC traffic from the same tree)."""
import csv
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

TOOL = os.path.join(ROOT, "tools", "timed_launches.py")


def _write(path, header, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def _trace(d, group):
    """warm-up: 2 iterations, timed: 3, then 1 in another phase; each iteration = `group` kernels of
    the sweep plus one other kernel; durations in ns chosen so the timed average is known."""
    kt, t, did = [], 1000, 0
    phases = [("warmup", 2, 5000), ("timed", 3, 4000), ("call", 1, 3000)]
    ranges = []
    for label, iters, dur in phases:
        start = t
        for _ in range(iters):
            for g in range(group):
                kt.append([did, f"void ppls_panel_k{g}<float, 10>(float const*)", t, t + dur])
                did += 1
                t += dur + 10
            kt.append([did, "ppls_finalize_kernel<10>(double const*)", t, t + 50])
            did += 1
            t += 60
        ranges.append([f"bench:{label}", start - 1, t])
        t += 100
    _write(os.path.join(d, "run_kernel_trace.csv"), ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"], kt)
    _write(os.path.join(d, "run_marker_api_trace.csv"), ["Operation", "Start_Timestamp", "End_Timestamp"], ranges)


@pytest.mark.parametrize("group", [1, 2])
def test_timed_launches_on_synthetic_trace(tmp_path, group):
    d = tmp_path / "trace"
    d.mkdir()
    _trace(str(d), group)
    line = dict(ms_per_step=0.0042 * group + 0.0001, steps=3, warmup=2, value=1.0,
                roofline=dict(avg_kernel_ms=0.004 * group, frac=0.5))
    bj = tmp_path / "line.log"
    bj.write_text("noise\n" + json.dumps(line) + "\n")
    r = subprocess.run([sys.executable, TOOL, str(d), "--kernel", "panel_k", "--bytes", "1e6", "--group", str(group),
                        "--name", "t", "--out-dir", str(tmp_path), "--bench-json", str(bj)],
                       capture_output=True, text=True, env=dict(os.environ, PPLS_PROFILED_TREE="abc1234"))
    assert r.returncode == 0, r.stderr
    js = json.load(open(tmp_path / "t.json"))
    ph = js["phases"]
    assert ph["warmup"]["launches"] == 2 and ph["timed"]["launches"] == 3 and ph["call"]["launches"] == 1
    assert abs(ph["timed"]["avg_ms"] - 0.004 * group) < 1e-12
    assert js["launches_per_unit"] == group and js["profiled_tree"] == "abc1234"
    assert js["check"]["timed_launches_eq_steps"] and js["check"]["timed_avg_le_ms_per_step"]
    assert len(js["ordinals"]["timed"]) == 3 * group   # per dispatch (PMC filtering)
    assert os.path.exists(tmp_path / "t_kernel_stats.csv")


@pytest.mark.parametrize("tag", ["r6c3", "r6c5"])
def test_committed_timed_profile_matches_its_line(tag):
    js = json.load(open(os.path.join(ROOT, "profiles", f"{tag}_timed_launches.json")))
    t, line, chk = js["phases"]["timed"], js["bench_line"], js["check"]
    assert t["launches"] == line["steps"] and chk["timed_launches_eq_steps"]
    assert t["avg_ms"] <= line["ms_per_step"] and chk["timed_avg_le_ms_per_step"]
    assert abs(t["frac"] / line["frac"] - 1) < 0.01
    assert abs(t["achieved_GBs"] * 1e9 / 8e12 - t["frac"]) < 1e-9
    assert js["profiled_tree"]


def test_committed_c3_pmc_from_the_traced_tree():
    tl = json.load(open(os.path.join(ROOT, "profiles", "r6c3_timed_launches.json")))
    for name in ("pmc_sweep_c3_dp1.json", "pmc_compute_c3_dp1.json"):
        pm = json.load(open(os.path.join(ROOT, "profiles", name)))
        assert pm["profiled_tree"] == tl["profiled_tree"], name
    sweep = json.load(open(os.path.join(ROOT, "profiles", "pmc_sweep_c3_dp1.json")))
    assert 1.0 <= sweep["traffic_over_algorithmic"] < 1.01
