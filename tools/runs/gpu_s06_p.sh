# Round 6: the index scan with hit SCORES compacted into a per-wave
# (score, id, query) queue (TT_SCAN_COMPACT=1 build, tools/vlib/compact)
# instead of 80-B hit rows — every index test under it, interleaved A/B at
# 1M x k=100, and one chunk's kernel times.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06p; mkdir -p $OUT
VL=$GRAFT_REPO_ROOT/tools/vlib/compact/libtt.so
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
TT_LIB_PATH=$VL step timeout -k 10 400 python -u -m pytest -v --timeout 280 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_model_gpu.py tests/test_distributed_gpu.py tests/test_pipeline_gpu.py \
  -k "bruteforce or index or topk or retriever" > $OUT/tests.log 2>&1
echo "compact: $(tail -1 $OUT/tests.log)"
grep -q " failed\| error" $OUT/tests.log && { grep -E "FAILED|Error" $OUT/tests.log | head -20; exit 1; }
for r in 1 2 3; do
  for v in rows compact; do
    if [ $v = compact ]; then L=$VL; else L=""; fi
    TT_LIB_PATH=$L step timeout -k 10 120 python -u tools/time_index.py 1000000 100 3 > $OUT/ab_${v}_$r.txt 2>&1
    echo "$v $(tail -1 $OUT/ab_${v}_$r.txt)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in rows compact; do
  if [ $v = compact ]; then L=$VL; else L=""; fi
  TT_LIB_PATH=$L step timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- python3 tools/time_index.py 131072 100 2 > $OUT/prof_$v.log 2>&1
  f=$(find $OUT/prof_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
  n=r['Name']
  if any(x in n for x in ('scan','sample_kernel<128>','finalize','fallback')): print('   ', n[:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
  rm -f $OUT/prof_$v/*kernel_trace.csv
done
