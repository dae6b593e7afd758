cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for ab in 0 2; do
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/pmc_split_$ab -o run -- python3 $R/tools/split_pmc_driver.py c4s $ab > $R/gpurun_out/pmc_split_$ab.log 2>&1 || exit 1
done
