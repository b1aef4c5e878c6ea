# Round 4: mlp_rows with A fetched five stages ahead (the whole block at the
# towers' K <= 320) against HEAD's two stages, same box.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04z; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py -q -k "mlp or tower or train_step or c2 or c3 or dense" --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
for v in new head; do
  if [ $v = head ]; then export TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/pbin/libhead/libtt.so; else unset TT_LIB_PATH; fi
  echo "== $v"; timeout -k 10 120 python -u tools/time_mlp.py 2>&1 | grep "us "
done
unset TT_LIB_PATH
bash tools/gpu_step_ab.sh 3 now:: head:TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/pbin/libhead/libtt.so:
