# PMC passes over index probes (repo root on the GPU box): bash tools/gpu_pmc_scan.sh probe1 [probe2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for B in "$@"; do
  OUT=$R/gpurun_out/pmc_$B; mkdir -p $OUT
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/p1 -o p1 -- $R/tools/pbin/$B 65536 > /dev/null 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM --output-format csv -d $OUT/p2 -o p2 -- $R/tools/pbin/$B 65536 > /dev/null 2>&1 || exit 1
  echo "== $B"
  python3 $R/tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv") --match "scan_kernel\|screen_kernel" 2>&1 | head -40
done
