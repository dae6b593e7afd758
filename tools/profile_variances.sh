#!/bin/bash
# rocprofv3 passes for variances.PPLS_simult (tools/bench_variances.py): kernel trace + stats of the
# whole call, then PMC passes (each its own run, no other trace domains) on the Gram alone.
# usage: tools/profile_variances.sh <config>
set -o pipefail
cfg="${1:-c3}"
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/prof_var_$cfg"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run \
  -- python3 "$R/tools/bench_variances.py" --config "$cfg" > "$O.trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d "$O/pmc_mfma" -o run -- python3 "$R/tools/bench_variances.py" --config "$cfg" --no-full --reps 1 \
  > "$O.mfma.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run \
  -- python3 "$R/tools/bench_variances.py" --config "$cfg" --no-full --reps 1 > "$O.fetch.log" 2>&1 || exit $?
