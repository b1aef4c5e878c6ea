# Runner point list target for k >= 512: TT_INDEX_R_MUL_BIG 1.5 (tree) vs
# 1.2 / 1.15 / 1.1 / 1.0 (variant builds rm*): the index tests (incl. the
# runner-point shape, bit-exact) on each variant, then interleaved timings.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05rrm; mkdir -p $OUT
V="rm12 rm115 rm11 rm10"
for v in $V; do
  TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_distributed_gpu.py -m gpu -q -k "index or bruteforce or topk or candidate" --timeout 200 --timeout-method thread > $OUT/t_$v.log 2>&1 && echo "$v tests: $(tail -1 $OUT/t_$v.log)" || { echo "$v tests FAILED"; grep -E "FAIL|Error" $OUT/t_$v.log | head -5; }
done
for r in 1 2 3; do
  for v in new $V; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so
    env TT_LIB_PATH=$L timeout -k 10 120 python -u tools/time_index.py 2048 1000 20 > $OUT/$v.$r.log 2>&1 || { echo "$v FAILED"; tail -3 $OUT/$v.$r.log; exit 1; }
    echo "$v r$r: $(tail -1 $OUT/$v.$r.log)"
  done
done
