# Round 6: the chunked id sort for regions up to 131072 lookups (the merge
# stages 16 chunks at a time) instead of the key build + rocPRIM sort above
# 32768 — the sparse sort-path tests and the C5 / sparse-table tests, then
# the C5 leg and the train step, new vs the previous tt_sparse.hip.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06s; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
step timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_model_gpu.py \
  -k "sparse or c5 or sharded or routed or dedup or scatter" > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
grep -q " failed\| error" $OUT/tests.log && { grep -E "FAILED|Error" $OUT/tests.log | head -30; exit 1; }
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then L=$GRAFT_REPO_ROOT/tools/vlib/sort_old/libtt.so; else L=""; fi
    TT_LIB_PATH=$L step timeout -k 10 200 python -u bench.py --c5-only > $OUT/c5_${v}_$r.json 2> $OUT/c5_${v}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/c5_${v}_$r.json')); c=d.get('c5_sharded_table', d); print('c5 $v $r', round(c['ms_per_step'],4), round(c['roofline']['frac'],3))"
  done
done
bash tools/gpu_step_ab.sh 2 "new:-:" "old:TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/sort_old/libtt.so:"
