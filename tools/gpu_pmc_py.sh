# PMC passes over a python script; summary for kernels matching $MATCH.
#   MATCH=mlp_wgrad bash tools/gpu_pmc_py.sh tag tools/time_mlp.py [args]
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/pmc_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/p1 -o p1 -- python3 "$R/$@" > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM --output-format csv -d $OUT/p2 -o p2 -- python3 "$R/$@" > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o p3 -- python3 "$R/$@" > /dev/null 2>&1 || exit 1
cd $R && python3 tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv") --match "$MATCH" | head -60
