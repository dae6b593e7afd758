#!/bin/bash
# What bounds the C5 MFMA dots kernel: kernel-trace durations of the dots launches for experiment
# builds of the library compiled with -DPPLS_DOTS_ABLATE=v (bit 0 no MFMAs, bit 1 no X loads,
# bit 2 no B loads; results invalid), built into abtest/v<v>/ (copies of ppls_amd/ and include/).
# usage: tools/dots_ablate.sh <config> <v> [<v> ...]      (v = 0: the production build)
set -o pipefail
cfg="$1"; shift
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = "0" ]; then pkg="$R"; else pkg="$R/abtest/v$v"; fi
  PPLS_PKG_ROOT="$pkg" timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/dab_${cfg}_$v" -o run -- python3 "$R/tools/panel_variants.py" "$cfg" 0 \
    > "$R/gpurun_out/dab_${cfg}_$v.log" 2>&1 || exit $?
  python3 - "$R/gpurun_out/dab_${cfg}_$v/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
names = {"0": "full", "1": "no MFMA", "2": "no X loads", "4": "no B loads", "3": "no MFMA, no X",
         "5": "no MFMA, no B", "6": "no X, no B (MFMA + LDS)"}
for r in csv.DictReader(open(sys.argv[1])):
    if "mfmadots" in r["Name"]:
        print(f"PPLS_DOTS_ABLATE={sys.argv[2]} ({names.get(sys.argv[2], '?'):24s}) dots avg {float(r['AverageNs']) / 1e3:8.1f} us")
PY
done
