# Round 6: after reverting the block-sum and fused-backward experiments —
# sparse / routed / train-step / MLP tests (join search kept, odd-width fused
# Adagrad fix) and the index tests (zeroing kernel).
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06n; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
step timeout -k 10 700 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py \
  -k "sparse or dedup or routed or adagrad or train_step or c5 or sharded or odd or dense or bruteforce or index" > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
grep -q " failed\| error" $OUT/tests.log && { grep -E "FAILED|Error" $OUT/tests.log | head -30; exit 1; }
bash tools/gpu_step_ab.sh 2 "cur:-:"
