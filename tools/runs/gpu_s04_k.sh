# Round 4: the runner point (2048 queries, k = 1000): list-size target and split count probes, kernel times.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04k; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in r3 r2 r15 r3s64 r2s64; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o t -- ./tools/pbin/probe_$v 2048 105542 1000 > $OUT/$v.log 2>&1
  echo "== $v $(grep nq= $OUT/$v.log | tail -1) | $(grep entries $OUT/$v.log | tail -1)"
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$OUT/$v/*kernel_stats.csv')[0])):
  n=r['Name']
  if any(k in n for k in ('scan','finalize','sample','fallback','prep','tau_min')): print('   ', n[:45], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
  rm -f $OUT/$v/*kernel_trace.csv
done
