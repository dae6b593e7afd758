#!/bin/bash
# Is the finalize slowed by cold instruction/data caches after each sweep streams GBs through L2?
# ablate bit 13 launches every finalize twice; the second copy runs with warm caches.  Kernel trace:
# odd and even finalize dispatches averaged separately (tools/finalize_cache_summary.py).
# usage: tools/finalize_cache_probe.sh <config>
set -o pipefail
cfg="$1"
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/fcache_$cfg" -o run \
  -- python3 "$R/tools/option_ab.py" "$cfg" "ablate=8192" --reps 1 --iters 40 > "$R/gpurun_out/fcache_$cfg.log" 2>&1 || exit $?
python3 - "$R/gpurun_out/fcache_$cfg/run_kernel_trace.csv" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
fin = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if "finalize_kernel" in r["Kernel_Name"]]
first, second = fin[0::2], fin[1::2]
print(f"finalize launched twice per iteration ({len(fin)} dispatches): first (after the sweep) "
      f"{sum(first) / len(first) / 1e3:.2f} us, second (warm caches) {sum(second) / len(second) / 1e3:.2f} us")
PY
