# Round 4: finalize phase breakdown (probe builds returning after each phase:
# 1 staging, 2 radix select + certificate, 3 cut, 4 rescoring, 5 exact select;
# norescore = every phase, survivors scored by their row number).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04s; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in stop1 stop2 stop3 stop4 stop5 norescore new; do
  for shape in "2048 105542 1000" "131072 105542 100"; do
    tag=$v$(echo $shape | cut -d' ' -f1)
    timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o t -- ./tools/pbin/probe_$v $shape > $OUT/$tag.log 2>&1
    python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$OUT/$tag/*kernel_stats.csv')[0])):
  if 'finalize' in r['Name']: print('$v $shape', r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
    rm -f $OUT/$tag/*kernel_trace.csv
  done
done
