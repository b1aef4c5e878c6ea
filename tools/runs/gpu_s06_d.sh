# Round 6: x3 (fp32-faithful scores) accuracy + the trained-magnitude test,
# odd tower widths, then the suite without the capture-guard test, then that
# test alone (last: a crash there ends the call).  A test failure (rc 1) goes
# on; anything else stops.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06d; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
step timeout -k 10 300 python -u -m pytest -v -s --timeout 280 --timeout-method thread \
  "tests/test_configs_gpu.py::test_c3_inbatch_grads_vs_fp64_after_training" tests/test_kernels_gpu.py -k "x3 or dense_stack or trained" > $OUT/x3.log 2>&1
grep "score_max\|passed\|failed\|Error" $OUT/x3.log | tail -8
step timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "not capture_guard" > $OUT/suite.log 2>&1
tail -3 $OUT/suite.log; grep FAILED $OUT/suite.log | head -20
step timeout -k 10 120 python -u -m pytest -v --timeout 100 --timeout-method thread tests/test_model_gpu.py -k capture_guard > $OUT/guard.log 2>&1
tail -5 $OUT/guard.log
