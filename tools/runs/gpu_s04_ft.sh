# Round 4: flush period in tiles (TT_SCAN_FLUSH_TILES) at 131k x k=100: scan / finalize /
# fallback time, entries per query and certificate failures (TT_INDEX_STATS).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04ft; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in ft4 ft2 ft8 ft0 ft4; do
  tag=$v
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o t -- ./tools/pbin/probe_$v 131072 105542 100 > $OUT/$tag.log 2>&1
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$OUT/$tag/*kernel_stats.csv')[0])):
  n=r['Name']
  if any(x in n for x in ('scan','finalize','fallback','sample')): print('   ', n[30:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
  rm -f $OUT/$tag/*kernel_trace.csv
done
