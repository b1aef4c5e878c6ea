# Round 5: per-row residual screen bound — bit-exact index tests, then
# interleaved index timing: this tree's libtt (per-row cut + certificate,
# no X pass), the TT_INDEX_ROW_X=1 build (plus the X-tightening pass) and
# the same sources with the round-start tt_index.hip.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05idxab; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py \
  tests/test_model_gpu.py -m gpu -v -k "index or bruteforce or topk or c4 or candidate or recall" \
  --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
echo "index tests rc=$rc: $(tail -1 $OUT/t.log)"; grep -n "FAIL" $OUT/t.log | head; [ $rc -ne 0 ] && exit 0
for r in 1 2; do
  for v in new rowx base; do
    L=""; [ $v != new ] && L="TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/r05$v/libtt.so"
    for cfg in "1048576 100 2" "2048 1000 20"; do
      f=$OUT/$v.$r.$(echo $cfg | tr ' ' _).log
      env $L timeout -k 10 120 python -u tools/time_index.py $cfg > $f 2>&1 || { echo "$v r$r [$cfg] FAILED"; tail -3 $f; exit 0; }
      echo "$v r$r [$cfg]: $(tail -1 $f)"
    done
  done
done
exit 0
