# Round 4: scan kernel SQ counters for the probe builds (base / no insert / bare MFMA loop), 131072 queries.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04i; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/pbin/probe_stats 131072
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
for v in base noins bare; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v/t -o t -- ./tools/pbin/probe_$v 131072 > $OUT/$v.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $A --output-format csv -d $OUT/$v/a -o a -- ./tools/pbin/probe_$v 131072 >> $OUT/$v.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $B --output-format csv -d $OUT/$v/b -o b -- ./tools/pbin/probe_$v 131072 >> $OUT/$v.log 2>&1
  echo "== $v $(grep nq= $OUT/$v.log | tail -1)"
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$OUT/$v/t/*kernel_stats.csv')[0])):
  if 'scan' in r['Name'] or 'finalize' in r['Name']: print('   ', r['Name'][:45], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
  python3 tools/pmc_summary.py $(find $OUT/$v/a $OUT/$v/b -name '*counter_collection.csv') --match scan_kernel
  rm -f $(find $OUT/$v -name '*counter_collection.csv') $(find $OUT/$v -name '*kernel_trace.csv')
done
