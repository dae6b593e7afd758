#!/bin/bash
# Round-end profiles on the GPU box: rocprofv3 kernel trace + FETCH/WRITE passes and the compute
# counter passes for C3 and C5 (bench.py, short runs), summarised on the box (PPLS_PROFILED_TREE names
# the tree, there is no .git there) into gpurun_out/final_profiles/; the raw CSVs are deleted so the
# merge back stays small.  usage: PPLS_PROFILED_TREE=<commit> tools/final_profiles.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
O="$R/gpurun_out/final_profiles"
mkdir -p "$O"
bash tools/profile.sh r4fc3 --no-call --steps 50 --xprod-steps 300 || exit $?
bash tools/pmc_compute.sh r4fc3 --no-call --steps 50 --xprod-steps 300 || exit $?
bash tools/profile.sh r4fc5 --config c5 --no-call --steps 20 --xprod-steps 100 || exit $?
bash tools/pmc_compute.sh r4fc5 --config c5 --no-call --steps 20 --xprod-steps 100 || exit $?
cd "$R" || exit 1
python3 tools/pmc_summary.py r4fc3 c3_dp1 32e9 "round 4 final" || exit $?
python3 tools/pmc_xprod_summary.py r4fc3 c3 "round 4 final" || exit $?
python3 tools/pmc_compute_summary.py r4fc3 c3_dp1 sweep_split,gram_mfma,xprod_tile,finalize --trace gpurun_out/prof_r4fc3/trace/run_kernel_stats.csv || exit $?
python3 tools/pmc_summary.py r4fc5 c5_dp1 21e9 "round 4 final" --kernels panel_mfmadots,panel_acc || exit $?
python3 tools/pmc_xprod_summary.py r4fc5 c5 "round 4 final" --bytes 924844032 || exit $?
python3 tools/pmc_compute_summary.py r4fc5 c5_dp1 panel_mfmadots,panel_acc,gram_mfma,xprod_tile,finalize --trace gpurun_out/prof_r4fc5/trace/run_kernel_stats.csv || exit $?
cp profiles/pmc_*_dp1.json "$O/"
cp gpurun_out/prof_r4fc3/trace/run_kernel_stats.csv "$O/r4_final_c3_kernel_stats.csv"
cp gpurun_out/prof_r4fc5/trace/run_kernel_stats.csv "$O/r4_final_c5_kernel_stats.csv"
rm -rf gpurun_out/prof_r4fc3 gpurun_out/prof_r4fc5 gpurun_out/pmcc_r4fc3 gpurun_out/pmcc_r4fc5
