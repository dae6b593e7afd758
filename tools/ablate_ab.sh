#!/bin/bash
# Kernel traces of ablation builds (abtest/<v>) beside the product, same box, interleaved:
# usage: tools/ablate_ab.sh <config> <variant> [<variant> ...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cfg="$1"; shift
cd /tmp && export TMPDIR=/tmp
for arm in base "$@" base "$@"; do
  if [ "$arm" = base ]; then T="$R"; else T="$R/abtest/$arm"; fi
  out="$R/gpurun_out/abl_${cfg}_${arm}"
  rm -rf "$out"
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run \
    -- python3 "$T/tools/ablate_run.py" "$cfg" > "$out.log" 2>&1 || exit $?
  echo "$cfg $arm: $(tail -1 "$out.log")"
  python3 - "$out/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0]
    if "panel" in n:
        print(f"    {n[:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:8.2f} us")
PY
  rm -rf "$out"
done
