# Round 4: in-batch positives masked half way through region B (after the
# score MFMAs have landed) instead of right after region A.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04u; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py -q -k "inbatch or train_step or loss or global or c2 or c3 or sharded" --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for v in new new2 nomask; do echo "$v $(timeout -k 10 60 ./tools/pbin/inb_$v 16384 100)"; done
done
timeout -k 10 120 python -u tools/time_inbatch.py
bash tools/gpu_step_ab.sh 3 now:: head:TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/pbin/libhead/libtt.so:
