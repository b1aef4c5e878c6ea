#!/bin/bash
# PMC passes for the index probe (run on the GPU box from the repo root).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B=${1:-probeNOINSERT}
NQ=${2:-65536}
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/p1 -o p1 -- $GRAFT_REPO_ROOT/tools/bin/$B $NQ 105542 > /dev/null
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM --output-format csv -d $OUT/p2 -o p2 -- $GRAFT_REPO_ROOT/tools/bin/$B $NQ 105542 > /dev/null
echo pmc-ok
