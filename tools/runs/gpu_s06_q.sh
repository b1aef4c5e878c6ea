# Round 6: the index list-size target (screened entries per query,
# TT_INDEX_R_MUL k + TT_INDEX_R_ADD; default 3k + 100) at 2.5k + 75 and
# 2k + 50: 1M x k=100 timing and one chunk's kernel times (the fallback's
# time shows the certificate failures' cost).
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06q; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
for r in 1 2; do
  for v in base r25 r2; do
    if [ $v = base ]; then L=""; else L=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so; fi
    TT_LIB_PATH=$L step timeout -k 10 180 python -u tools/time_index.py 1000000 100 3 > $OUT/ab_${v}_$r.txt 2>&1
    echo "$v $(tail -1 $OUT/ab_${v}_$r.txt)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base r25 r2; do
  if [ $v = base ]; then L=""; else L=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so; fi
  TT_LIB_PATH=$L step timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- python3 tools/time_index.py 131072 100 2 > $OUT/prof_$v.log 2>&1
  f=$(find $OUT/prof_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
  n=r['Name']
  if any(x in n for x in ('scan','sample_kernel<128>','finalize','fallback','tau_')): print('   ', n[:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
  rm -f $OUT/prof_$v/*kernel_trace.csv
done
