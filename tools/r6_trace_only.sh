#!/bin/bash
# The kernel-trace step of tools/r6_profiles.sh alone (no PMC passes): the driver's bench command under
# PPLS_ROCTX=1 rocprofv3 --kernel-trace --marker-trace, then tools/timed_launches.py.
# usage: tools/r6_trace_only.sh <tag> <kernel_substr> <bytes> <group> [bench args...]
#   e.g. r6c5 panel_ 21e9 2 --config c5 --steps 20 --warmup 5
set -o pipefail
tag="$1"; kern="$2"; bytes="$3"; group="$4"; shift 4
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r6_profiles"
mkdir -p "$O"
T="$R/gpurun_out/prof_$tag"
cmd=(python3 "$R/bench.py" --gpus 1 "$@")
(cd /tmp && export TMPDIR=/tmp && PPLS_ROCTX=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats \
   --output-format csv -d "$T/trace" -o run -- "${cmd[@]}" > "$O/${tag}_bench_line.log" 2> "$O/${tag}_trace_stderr.log") || exit $?
cd "$R" || exit 1
python3 tools/timed_launches.py "$T/trace" --kernel "$kern" --bytes "$bytes" --group "$group" --name "${tag}_timed_launches" \
  --bench-json "$O/${tag}_bench_line.log" --command "rocprofv3 --kernel-trace --marker-trace --stats -- ${cmd[*]}" || exit $?
cp "$T/trace/run_kernel_stats.csv" "$O/${tag}_all_kernel_stats.csv"
cp "profiles/${tag}_timed_launches.json" "profiles/${tag}_timed_launches_kernel_stats.csv" "$O/"
echo "profiles written to $O"
