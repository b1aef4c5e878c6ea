# PMC passes over the in-batch probe (run on the GPU box from the repo root).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/ixpmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="$GRAFT_REPO_ROOT/tools/bin/${1:-ixp_new} 262144 105542 100"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o p1 -- $P > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/p2 -o p2 -- $P > /dev/null 2>&1
echo pmc-ok
