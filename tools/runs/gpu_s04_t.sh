# Round 4: in-batch entry before (c2feba1) and after the arithmetic contract,
# same box, interleaved; then per-kernel rocprof stats of each.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04t; mkdir -p $OUT
for r in 1 2; do
  for v in new nomask v1 v2 v3; do echo "$v $(timeout -k 10 60 ./tools/pbin/inb_$v 16384 100)"; done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in new v2 v3; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o t -- ./tools/pbin/inb_$v 16384 100 > /dev/null 2>&1
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$OUT/$v/*kernel_stats.csv')[0])):
  print('$v', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
  rm -f $OUT/$v/*kernel_trace.csv
done
