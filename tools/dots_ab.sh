#!/bin/bash
# LDS-free MFMA dots (default) vs the LDS-transposed form (ablate bit 11): kernel-trace durations of
# the dots launches at a panel config.  usage: tools/dots_ab.sh <config>
set -o pipefail
cfg="$1"
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
for ab in 0 2048 0 2048; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/dab2_${cfg}_$ab" -o run \
    -- python3 "$R/tools/panel_variants.py" "$cfg" "$ab" > "$R/gpurun_out/dab2_${cfg}_$ab.log" 2>&1 || exit $?
  grep "it/s" "$R/gpurun_out/dab2_${cfg}_$ab.log" | tail -1
  python3 - "$R/gpurun_out/dab2_${cfg}_$ab/run_kernel_stats.csv" "$ab" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "dots" in r["Name"] or "panel_acc" in r["Name"]:
        print(f"  ablate {sys.argv[2]:>5s} {r['Name'].split('(')[0][5:50]:45s} avg {float(r['AverageNs']) / 1e3:8.1f} us")
PY
done
