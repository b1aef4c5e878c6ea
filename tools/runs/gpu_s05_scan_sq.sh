# Round 5: SQ counters of scan_kernel<128> on one 131,072-query chunk of C4
# (tools/index_probe.hip builds in tools/pbin: base = this tree, noins = tau
# +inf (nothing staged), bare = no filter work), two --pmc passes each.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05sq; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
for v in base noins bare; do
  timeout -k 10 60 $GRAFT_REPO_ROOT/tools/pbin/probe_$v 131072 105542 100 > $OUT/$v.txt
  cat $OUT/$v.txt | head -3
  timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $OUT/${v}_p1 -o p -- $GRAFT_REPO_ROOT/tools/pbin/probe_$v 131072 105542 100 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $OUT/${v}_p2 -o p -- $GRAFT_REPO_ROOT/tools/pbin/probe_$v 131072 105542 100 > /dev/null 2>&1
  python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT/${v}_p1/p_counter_collection.csv $OUT/${v}_p2/p_counter_collection.csv --match scan_kernel > $OUT/${v}_sq.txt
  cat $OUT/${v}_sq.txt
  rm -f $OUT/${v}_p1/p_counter_collection.csv $OUT/${v}_p2/p_counter_collection.csv
done
