# Round 4: mlp_rows with 32-row workgroups (TT_MLP_BM=32: 512 workgroups,
# 2-5 waves per SIMD) against 64-row ones, same box.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04bm; mkdir -p $OUT
L32=$GRAFT_REPO_ROOT/tools/pbin/libbm32/libtt.so
TT_LIB_PATH=$L32 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -k "mlp or tower or train_step" --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
for v in bm64 bm32; do
  if [ $v = bm32 ]; then export TT_LIB_PATH=$L32; else unset TT_LIB_PATH; fi
  echo "== $v"; timeout -k 10 120 python -u tools/time_mlp.py 2>&1 | grep "us "
done
unset TT_LIB_PATH
bash tools/gpu_step_ab.sh 3 bm64:: bm32:TT_LIB_PATH=$L32:
