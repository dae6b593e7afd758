#!/bin/bash
# Compute-side PMC passes (MFMA / VALU utilisation, fp64 instruction mix) for one bench workload:
# two --pmc passes (8 SQ + GRBM counters each, never combined with trace domains), each its own run.
# usage: tools/pmc_compute.sh <tag> <bench args...>      (summary: tools/pmc_compute_summary.py <tag>)
set -o pipefail
tag="$1"; shift
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU"
P2="GRBM_GUI_ACTIVE SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS"
i=0
for pass in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d "$R/gpurun_out/pmcc_$tag/p$i" -o run \
    -- python3 "$R/bench.py" --no-cpu "$@" > "$R/gpurun_out/pmcc_${tag}_p$i.log" 2>&1 || exit $?
done
