#!/bin/bash
# Same-box A/B of an experiment build (a copied tree under abtest/<name>, built with PPLS_EXTRA_CFLAGS)
# against the in-tree build: finalize and sweep kernel averages (kernel trace) and ms per EM iteration.
# usage: [VAB_SPEC="xprod=1"] [VAB_ITERS=200] tools/variant_ab.sh <variant dir name> <config> [<config> ...]
set -o pipefail
var="$1"; shift
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
for cfg in "$@"; do
  for arm in base "$var" base "$var"; do
    if [ "$arm" = base ]; then T="$R"; else T="$R/abtest/$arm"; fi
    out="$R/gpurun_out/vab_${cfg}_${arm}"
    rm -rf "$out"
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run \
      -- python3 "$T/tools/option_ab.py" "$cfg" "${VAB_SPEC:-}" --reps 1 --iters "${VAB_ITERS:-200}" > "$out.log" 2>&1 || exit $?
    echo "$cfg $arm: $(grep -E 'ms|it/s' "$out.log" | tail -1)"
    python3 - "$out/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if "finalize" in n or "sweep" in n or "dots" in n or "panel" in n or "xprod" in n:
        print(f"    {n[:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:8.2f} us")
PY
  done
done
