# PMC passes over tools/gemm_probe.py (GPU box, repo root): bash tools/pmc_gemm.sh fwd x3
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/gemmpmc_$1_$2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="python3 $GRAFT_REPO_ROOT/tools/gemm_probe.py $1 $2"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o t -- $P > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAVES --output-format csv -d $OUT/p1 -o p1 -- $P > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU --output-format csv -d $OUT/p2 -o p2 -- $P > /dev/null 2>&1
echo pmc-ok
