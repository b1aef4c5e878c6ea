# Round 4: in-batch passes back to two workgroups per CU (mask_diag in 32-bit lane math, launch bounds);
# finalize selects skip the keys' common top bits, register bitonic for P <= 256.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04q; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py tests/test_pipeline_gpu.py -q -k "inbatch or train_step or loss or bruteforce or index or c4 or topk or retriever or export or recall or graph or global" --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
TT_FINAL_WAVES=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -q -k "bruteforce or c4" --timeout 200 --timeout-method thread > $OUT/tests_nw4.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests_nw4.log | head -40; exit 1; }
echo "nw4 $(tail -1 $OUT/tests_nw4.log)"
TT_INDEX_CM=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -q -k "bruteforce or c4" --timeout 200 --timeout-method thread > $OUT/tests_cm.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests_cm.log | head -40; exit 1; }
echo "cm $(tail -1 $OUT/tests_cm.log)"
bash tools/gpu_step_ab.sh 2 now:: pair:TT_TOWER_PAIR=1: fused:-:--fused-apply
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in new cm prev norescore; do
  for shape in "131072 105542 100" "2048 105542 1000"; do
    tag=$v$(echo $shape | cut -d' ' -f1)
    pv=$v; [ $v = cm ] && pv=new
    TT_INDEX_CM=$([ $v = cm ] && echo 1 || echo 0) timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o t -- ./tools/pbin/probe_$pv $shape > $OUT/$tag.log 2>&1
    echo "== $v $shape $(grep nq= $OUT/$tag.log | tail -1)"
    python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$OUT/$tag/*kernel_stats.csv')[0])):
  if 'finalize' in r['Name'] or 'scan' in r['Name'] or 'cm_' in r['Name']: print('   ', r['Name'][:45], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
    rm -f $OUT/$tag/*kernel_trace.csv
  done
done
bash tools/gpu_trace_step.sh s04q
timeout -k 10 120 python -u tools/time_index.py 2048 1000 10
TT_INDEX_CM=1 timeout -k 10 120 python -u tools/time_index.py 2048 1000 10
timeout -k 10 120 python -u tools/time_index.py 1000000 100 3
