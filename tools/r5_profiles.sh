#!/bin/bash
# Round-5 profiles on the GPU box: rocprofv3 kernel trace + FETCH/WRITE passes and the compute
# counter passes for C3 and C5 (bench.py, short runs; the traces include the MFMA Gram that forms S),
# and a kernel trace of meta_PPLSi at C3 with 4 populations (tools/bench_meta.py); summarised on the
# box into gpurun_out/r5_profiles/ (PPLS_PROFILED_TREE names the tree, the box has no .git); the raw
# CSVs are deleted so the merge back stays small.  usage: PPLS_PROFILED_TREE=<commit> tools/r5_profiles.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O="$R/gpurun_out/r5_profiles"
mkdir -p "$O"
bash tools/profile.sh r5c3 --no-call --steps 50 --xprod-steps 300 || exit $?
bash tools/pmc_compute.sh r5c3 --no-call --steps 50 --xprod-steps 300 || exit $?
bash tools/profile.sh r5c5 --config c5 --no-call --steps 20 --xprod-steps 100 || exit $?
bash tools/pmc_compute.sh r5c5 --config c5 --no-call --steps 20 --xprod-steps 100 || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$R/gpurun_out/prof_r5meta/trace" -o run -- python3 "$R/tools/bench_meta.py" c3 --K 4 --steps 20 \
   > "$R/gpurun_out/prof_r5meta_trace.log" 2>&1) || exit $?
cd "$R" || exit 1
python3 tools/pmc_summary.py r5c3 c3_dp1 32e9 "round 5" || exit $?
python3 tools/pmc_summary.py r5c3 c3_dp1 32e9 "round 5: the MFMA Gram forming S; algorithmic = one read of X, Y" \
  --kernels gram_mfma --out gram_s_c3 || exit $?
python3 tools/pmc_xprod_summary.py r5c3 c3 "round 5" || exit $?
python3 tools/pmc_compute_summary.py r5c3 c3_dp1 sweep_split,gram_mfma,xprod_tile,finalize --trace gpurun_out/prof_r5c3/trace/run_kernel_stats.csv || exit $?
python3 tools/pmc_summary.py r5c5 c5_dp1 21e9 "round 5" --kernels panel_mfmadots,panel_acc || exit $?
python3 tools/pmc_summary.py r5c5 c5_dp1 21e9 "round 5: the MFMA Gram forming S; algorithmic = one read of X, Y" \
  --kernels gram_mfma --out gram_s_c5 || exit $?
python3 tools/pmc_xprod_summary.py r5c5 c5 "round 5" --bytes 924844032 || exit $?
python3 tools/pmc_compute_summary.py r5c5 c5_dp1 panel_mfmadots,panel_acc,gram_mfma,xprod_tile,finalize --trace gpurun_out/prof_r5c5/trace/run_kernel_stats.csv || exit $?
cp profiles/pmc_*_dp1.json profiles/pmc_gram_s_c3.json profiles/pmc_gram_s_c5.json "$O/"
cp gpurun_out/prof_r5c3/trace/run_kernel_stats.csv "$O/r5_c3_kernel_stats.csv"
cp gpurun_out/prof_r5c5/trace/run_kernel_stats.csv "$O/r5_c5_kernel_stats.csv"
cp gpurun_out/prof_r5meta/trace/run_kernel_stats.csv "$O/r5_meta_c3_k4_kernel_stats.csv"
cp gpurun_out/prof_r5meta_trace.log "$O/r5_meta_c3_k4_trace_run.log"
rm -rf gpurun_out/prof_r5c3 gpurun_out/prof_r5c5 gpurun_out/prof_r5meta gpurun_out/pmcc_r5c3 gpurun_out/pmcc_r5c5
