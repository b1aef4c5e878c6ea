# Round 6: the bare scan loops (TT_INDEX_NOINSERT: nothing staged) of the
# 32x32x16 and 16x16x32 scans, one 131k-query chunk each under rocprof; then
# the sparse update rework (both columns' loads in one round trip, (P+1)-ary
# join search): sparse / train-step tests and the interleaved step A/B
# against the previous tt_sparse.hip (tools/vlib/sparse_old).
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06k; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 32 16; do
  TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/noins/libtt.so TT_SCAN_SHAPE=$v step timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- python3 tools/time_index.py 131072 100 1 > $OUT/prof_$v.log 2>&1
  f=$(find $OUT/prof_$v -name '*kernel_stats.csv' | head -1)
  echo "== noinsert shape $v"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
  n=r['Name']
  if 'scan' in n: print('   ', n[:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
  rm -f $OUT/prof_$v/*kernel_trace.csv
done
step timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_pipeline_gpu.py -k "sparse or dedup or routed or adagrad or adam or train_step or c5 or sharded or fit or scatter" > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
grep -q " failed\| error" $OUT/tests.log && { grep -E "FAILED|Error" $OUT/tests.log | head -20; exit 1; }
bash tools/gpu_step_ab.sh 4 "new:-:" "old:TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/sparse_old/libtt.so:"
