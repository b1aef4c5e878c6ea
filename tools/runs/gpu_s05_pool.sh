# Runner point with the pooled rank estimate (tau = J-th largest of all
# splits' bins instead of the least per-split estimate; variant builds p*:
# list target x k + 100 and staging capacity x target) vs the tree: index
# tests (bit-exact, incl. the runner-point shape) per variant, then timings.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05pool; mkdir -p $OUT
V="p13 p12 p15 p13w"
for v in $V; do
  TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_distributed_gpu.py -m gpu -q -k "index or bruteforce or topk or candidate" --timeout 200 --timeout-method thread > $OUT/t_$v.log 2>&1 && echo "$v tests: $(tail -1 $OUT/t_$v.log)" || { echo "$v tests FAILED"; grep -E "FAIL|Error" $OUT/t_$v.log | head -5; }
done
for r in 1 2 3; do
  for v in new $V; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so
    for cfg in "2048 1000 20" "2048 100 20"; do
      env TT_LIB_PATH=$L timeout -k 10 120 python -u tools/time_index.py $cfg > $OUT/$v.$r.log 2>&1 || { echo "$v FAILED"; tail -3 $OUT/$v.$r.log; exit 1; }
      echo "$v r$r [$cfg]: $(tail -1 $OUT/$v.$r.log | cut -c1-62)"
    done
  done
done
