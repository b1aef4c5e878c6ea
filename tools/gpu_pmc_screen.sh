# PMC counters of the screen kernel (probe builds), one --pmc pass per run.
set -e
mkdir -p gpurun_out/pmc_screen
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-nosync stats}; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmc_screen/$v -o p -- $R/tools/pbin/probe_$v 131072 > /dev/null 2>&1
done
ls -R $R/gpurun_out/pmc_screen | head
