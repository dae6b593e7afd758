#!/bin/bash
# rocprofv3 passes for one bench workload: kernel trace + stats, then one PMC pass per counter
# (never combined with other trace domains).  usage: tools/profile.sh <tag> <bench args...>
set -o pipefail
tag="$1"; shift
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag/trace" -o run \
  -- python3 "$R/bench.py" --no-cpu "$@" > "$R/gpurun_out/prof_${tag}_trace.log" 2>&1 || exit $?
for ctr in FETCH_SIZE WRITE_SIZE; do
  rocprofv3 --pmc "$ctr" --output-format csv -d "$R/gpurun_out/prof_$tag/pmc_$ctr" -o run \
    -- python3 "$R/bench.py" --no-cpu "$@" > "$R/gpurun_out/prof_${tag}_$ctr.log" 2>&1 || exit $?
done
