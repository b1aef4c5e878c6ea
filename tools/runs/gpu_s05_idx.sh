# Round 5: per-row residual screen bound in the index finalize — bit-exact
# index tests, then interleaved timing vs the round-start library.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05idx; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py \
  tests/test_model_gpu.py -m gpu -v -k "index or bruteforce or topk or c4 or candidate or recall" \
  --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
echo "index tests rc=$rc: $(tail -1 $OUT/t.log)"; grep -n "FAIL" $OUT/t.log | head; [ $rc -ne 0 ] && exit 0
for r in 1 2; do
  for v in new base; do
    L=""; [ $v = base ] && L="TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/r05base/libtt.so"
    for cfg in "262144 100 3" "2048 1000 20"; do
      env $L timeout -k 10 120 python -u tools/time_index.py $cfg > $OUT/$v.$r.$(echo $cfg | tr ' ' _).log 2>&1 || exit 0
      echo "$v r$r [$cfg]: $(tail -1 $OUT/$v.$r.$(echo $cfg | tr ' ' _).log)"
    done
  done
done
exit 0
