#!/bin/bash
# Round-6 profiles of the driver's own bench command, all from ONE tree on ONE box:
#   1. PPLS_ROCTX=1 rocprofv3 --kernel-trace --marker-trace --stats -- python3 bench.py <args>
#      (the JSON line is kept; roctx ranges split the trace into em_begin / warmup / timed / ...)
#   2. rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE, and the two compute-counter passes, each its own
#      run of the same command with --no-cpu (the CPU baseline runs after the timed region, so the
#      timed launches keep their ordinal positions)
#   3. tools/timed_launches.py: the timed launches' average (<= ms_per_step) and roofline against the
#      line's; the PMC summaries restricted to those launches (--ordinals)
# usage: PPLS_PROFILED_TREE=<commit> tools/r6_profiles.sh <tag> <workload> <kernel_substr[,second]> <bytes>
#            <compute kernels> [bench args...]
#   e.g. r6c3 c3_dp1 sweep_split 32e9 sweep_split,gram_mfma,xprod_tile,finalize --steps 20 --warmup 5
set -o pipefail
tag="$1"; wl="$2"; kerns="$3"; bytes="$4"; ckerns="$5"; shift 5
kern="${kerns%%,*}"
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r6_profiles"
mkdir -p "$O"
T="$R/gpurun_out/prof_$tag"
cmd=(python3 "$R/bench.py" --gpus 1 "$@")
(cd /tmp && export TMPDIR=/tmp && PPLS_ROCTX=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats \
   --output-format csv -d "$T/trace" -o run -- "${cmd[@]}" > "$O/${tag}_bench_line.log" 2> "$O/${tag}_trace_stderr.log") || exit $?
for ctr in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc "$ctr" --output-format csv -d "$T/pmc_$ctr" -o run \
     -- "${cmd[@]}" --no-cpu > "$O/${tag}_$ctr.log" 2>&1) || exit $?
done
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU"
P2="GRBM_GUI_ACTIVE SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS"
i=0
for pass in "$P1" "$P2"; do
  i=$((i + 1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $pass --output-format csv \
     -d "$R/gpurun_out/pmcc_$tag/p$i" -o run -- "${cmd[@]}" --no-cpu > "$O/${tag}_pmcc_p$i.log" 2>&1) || exit $?
done
cd "$R" || exit 1
python3 tools/timed_launches.py "$T/trace" --kernel "$kern" --bytes "$bytes" --name "${tag}_timed_launches" \
  --bench-json "$O/${tag}_bench_line.log" --command "rocprofv3 --kernel-trace --marker-trace --stats -- ${cmd[*]}" || exit $?
TL="profiles/${tag}_timed_launches.json"
python3 tools/pmc_summary.py "$tag" "$wl" "$bytes" "round 6, the timed launches of the driver's command" \
  --kernels "$kerns" --ordinals "$TL" || exit $?
ords=()
IFS=, read -ra ks <<< "$kerns"
for k in "${ks[@]}"; do ords+=(--ordinals "$k=$TL"); done
python3 tools/pmc_compute_summary.py "$tag" "$wl" "$ckerns" "${ords[@]}" \
  --trace "profiles/${tag}_timed_launches_kernel_stats.csv" --trace "$T/trace/run_kernel_stats.csv" || exit $?
cp "$T/trace/run_kernel_stats.csv" "$O/${tag}_all_kernel_stats.csv"
cp "$TL" "profiles/${tag}_timed_launches_kernel_stats.csv" "profiles/pmc_sweep_$wl.json" "profiles/pmc_compute_$wl.json" "$O/"
rm -rf "$T/pmc_FETCH_SIZE" "$T/pmc_WRITE_SIZE" "$R/gpurun_out/pmcc_$tag"
echo "profiles written to $O"
