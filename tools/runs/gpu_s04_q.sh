# Round 4: in-batch passes back to two workgroups per CU (mask_diag in 32-bit lane math, launch bounds);
# finalize selects skip the keys' common top bits, register bitonic for P <= 256.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04q; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py tests/test_pipeline_gpu.py -q -k "inbatch or train_step or loss or bruteforce or index or c4 or topk or retriever or export or recall or graph or global" --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
TT_FINAL_WAVES=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -q -k "bruteforce or c4" --timeout 200 --timeout-method thread > $OUT/tests_nw4.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests_nw4.log | head -40; exit 1; }
echo "nw4 $(tail -1 $OUT/tests_nw4.log)"
bash tools/gpu_step_ab.sh 2 now::
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in new prev; do
  for shape in "131072 105542 100" "2048 105542 1000"; do
    tag=$v$(echo $shape | cut -d' ' -f1)
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
bash tools/gpu_trace_step.sh s04q
