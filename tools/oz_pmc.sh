#!/bin/bash
# PMC passes over the int8 SYRK lab (tools/oz_lab): where the residue SYRK's cycles go, for the
# full kernel (variant 0), compute only (16) and DMA only (64).  One counter set per run.
#   bash tools/oz_pmc.sh   -> gpurun_out/oz_pmc/v<variant>_p<pass>/...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"
for v in 0 16 64; do
  pass=1
  for set in "$P1" "$P2"; do
    out=$R/gpurun_out/oz_pmc/v${v}_p${pass}
    mkdir -p "$out"
    echo "=== variant $v pass $pass: $set"
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$out" -o run -- "$R/tools/oz_lab" 1000000 4000 4 0 $v \
      > "$out/stdout.log" 2>&1
    rc=$?
    echo "rc=$rc"; tail -3 "$out/stdout.log"
    [ $rc -ne 0 ] && exit $rc
    pass=$((pass + 1))
  done
done
exit 0
