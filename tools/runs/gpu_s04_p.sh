# Round 4: finalize selects skip the keys' common top bits; register bitonic ranking for P <= 256.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04p; mkdir -p $OUT
for nw in 0 4; do
  TT_FINAL_WAVES=$nw timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py tests/test_pipeline_gpu.py -q -k "bruteforce or index or c4 or topk or retriever or export or recall" --timeout 300 --timeout-method thread -rf > $OUT/tests_$nw.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests_$nw.log | head -40; exit 1; }
  echo "nw=$nw $(tail -1 $OUT/tests_$nw.log)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for v in new prev; do
  for shape in "131072 105542 100" "2048 105542 1000"; do
    tag=$v$rep$(echo $shape | cut -d' ' -f1)
    timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o t -- ./tools/pbin/probe_$v $shape > $OUT/$tag.log 2>&1
    echo "== $v $shape $(grep nq= $OUT/$tag.log | tail -1)"
    python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$OUT/$tag/*kernel_stats.csv')[0])):
  if 'finalize' in r['Name'] or 'scan' in r['Name']: print('   ', r['Name'][:45], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
    rm -f $OUT/$tag/*kernel_trace.csv
  done
done
done
