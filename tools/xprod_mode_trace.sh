#!/bin/bash
# Kernel traces of the cross-product iteration per xprod_pipe mode (tools/xprod_mode_run.py), then the
# timeline summary (tools/xprod_timeline.py).  usage: tools/xprod_mode_trace.sh <config> <mode> [<mode> ...]
set -o pipefail
cfg="$1"; shift
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
for mode in "$@"; do
  out="$R/gpurun_out/xtl_${cfg}_m$mode"
  rm -rf "$out"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$out" -o run \
    -- python3 "$R/tools/xprod_mode_run.py" "$cfg" "$mode" > "$out.log" 2>&1 || exit $?
  echo "=== $cfg mode $mode"
  python3 "$R/tools/xprod_timeline.py" "$(find "$out" -name '*kernel_trace.csv' | head -1)" -24 || exit $?
done
