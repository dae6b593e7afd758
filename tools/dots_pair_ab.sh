#!/bin/bash
# Panel dots: a wave pair per row tile (column split, default on shards with fewer row tiles than
# wave slots) vs one wave per row tile (option dots_pair = 0 forces it).  Interleaved arms in one
# process; kernel trace gives the dots/acc averages per arm.  usage: tools/dots_pair_ab.sh <config>...
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
for cfg in "$@"; do
  out="$R/gpurun_out/dpair_$cfg"
  rm -rf "$out"
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d "$out" -o run \
    -- python3 "$R/tools/option_ab.py" "$cfg" "" "dots_pair=0" --reps 3 --iters 60 > "$out.log" 2>&1 || exit $?
  grep "ms/iter" "$out.log"
  python3 - "$out/run_kernel_trace.csv" <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# arms alternate: split the dots launches into runs by kernel name (KS template argument)
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "mfmadots" in n or "panel_acc" in n:
        d[n.split("(")[0][5:80]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in d.items():
    v = sorted(v)[: max(1, len(v) * 9 // 10)]
    print(f"  {k:75s} n={len(v):4d} mean(fastest 90%) {sum(v) / len(v) / 1e3:8.1f} us")
PY
done
