#!/bin/bash
# Where the whole variances.PPLS_simult call spends its time: rocprofv3 kernel trace + stats of
# tools/bench_variances.py (C3).  usage: tools/profile_variances_r3.sh [config]
set -o pipefail
cfg="${1:-c3}"
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pvar_$cfg" -o run \
  -- python3 "$R/tools/bench_variances.py" --config "$cfg" --reps 1 > "$R/gpurun_out/pvar_$cfg.log" 2>&1 || exit $?
python3 - "$R/gpurun_out/pvar_$cfg/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f"{r['Name'][:70]:70s} calls {r['Calls']:>6s} total {float(r['TotalDurationNs']) / 1e6:9.3f} ms avg {float(r['AverageNs']) / 1e3:9.1f} us")
PY
grep "variances_s" "$R/gpurun_out/pvar_$cfg.log" | tail -1
