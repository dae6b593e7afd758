#!/bin/bash
# rocprofv3 kernel trace + stats of the cross-product iteration (tools/xprod_probe.py) per workload.
# usage: tools/profile_xprod.sh <tag> <probe args...>
set -o pipefail
tag="$1"; shift
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag" -o run \
  -- python3 "$R/tools/xprod_probe.py" "$@" > "$R/gpurun_out/prof_${tag}.log" 2>&1
