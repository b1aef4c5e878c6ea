# Round 4: the scan without the every-4-tiles forced flush (TT_SCAN_FLUSH_TILES=0:
# a wave flushes when 64 rows are staged, and at the end), against the default.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04ft0; mkdir -p $OUT
L0=$GRAFT_REPO_ROOT/tools/pbin/libft0/libtt.so
TT_LIB_PATH=$L0 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py -q -k "bruteforce or index or c4 or recall" --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for v in ft4 ft0; do
    if [ $v = ft0 ]; then export TT_LIB_PATH=$L0; else unset TT_LIB_PATH; fi
    echo "$v $(timeout -k 10 120 python -u tools/time_index.py 1000000 100 3 2>&1 | tail -1)"
    echo "$v $(timeout -k 10 120 python -u tools/time_index.py 2048 1000 10 2>&1 | tail -1)"
  done
done
