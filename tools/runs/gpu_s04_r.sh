# Round 4: finalize reads its list segments as one flat index space (segment
# counts prefixed by one wave) instead of segment by segment; candidate-major
# rescoring dropped (runner point 0.72 vs 0.60 ms).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04r; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py -q -k "bruteforce or c4 or index or shard" --timeout 200 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
TT_FINAL_WAVES=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -q -k "bruteforce or c4" --timeout 200 --timeout-method thread > $OUT/tests_nw4.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests_nw4.log | head -40; exit 1; }
echo "nw4 $(tail -1 $OUT/tests_nw4.log)"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in new new_nw2 new_nw1 prev norescore; do
  for shape in "131072 105542 100" "2048 105542 1000" "2048 105542 100"; do
    tag=$v$(echo $shape | cut -d' ' -f1)_$(echo $shape | cut -d' ' -f3)
    pv=$v; nw=0
    case $v in new_nw2) pv=new; nw=2;; new_nw1) pv=new; nw=1;; esac
    [ $v = new_nw1 ] && [ "$shape" != "2048 105542 1000" ] && continue
    [ $v = new_nw2 ] && [ "$shape" != "2048 105542 1000" ] && continue
    TT_FINAL_WAVES=$nw timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o t -- ./tools/pbin/probe_$pv $shape > $OUT/$tag.log 2>&1
    echo "== $v $shape $(grep nq= $OUT/$tag.log | tail -1)"
    python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$OUT/$tag/*kernel_stats.csv')[0])):
  print('   ', r['Name'][:45], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
    rm -f $OUT/$tag/*kernel_trace.csv
  done
done
timeout -k 10 120 python -u tools/time_index.py 2048 1000 10
timeout -k 10 120 python -u tools/time_index.py 2048 100 10
timeout -k 10 120 python -u tools/time_index.py 1000000 100 3
