# Round 6: x3 (bf16x3 S and P.V) accuracy, the trained-magnitude test with
# its printed errors, then the capture-guard test.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06e; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
step timeout -k 10 400 python -u -m pytest -v -s --timeout 280 --timeout-method thread \
  tests/test_configs_gpu.py tests/test_kernels_gpu.py -k "x3 or inbatch_grads_vs_fp64 or inbatch_softmax" > $OUT/x3.log 2>&1
grep "score_max\|passed\|failed\|Error" $OUT/x3.log | tail -8
step timeout -k 10 120 python -u -m pytest -v --timeout 100 --timeout-method thread tests/test_model_gpu.py -k capture_guard > $OUT/guard.log 2>&1
tail -5 $OUT/guard.log
