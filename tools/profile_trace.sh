#!/bin/bash
# rocprofv3 kernel trace + stats only (no PMC passes) for one bench workload.
# usage: tools/profile_trace.sh <tag> <bench args...>
set -o pipefail
tag="$1"; shift
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag/trace" -o run \
  -- python3 "$R/bench.py" --no-cpu "$@" > "$R/gpurun_out/prof_${tag}_trace.log" 2>&1
