# Round 6: odd-width diagnostic, trained-magnitude fp64 in-batch gradients
# (with its printed errors), the sharded / capture tests, then the suite.
# A test failure (rc 1) goes on to the next step; anything else stops.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06c; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
step timeout -k 10 120 python -u tools/diag_odd_widths.py > $OUT/odd.log 2>&1; cat $OUT/odd.log | tail -8
step timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread \
  "tests/test_configs_gpu.py::test_c3_inbatch_grads_vs_fp64_after_training" > $OUT/fp64.log 2>&1
grep "score_max\|passed\|failed\|Error" $OUT/fp64.log | tail -5
step timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_model_gpu.py -k "sharded or rccl or graph or capture" > $OUT/model.log 2>&1; tail -3 $OUT/model.log
step timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $OUT/suite.log 2>&1
tail -3 $OUT/suite.log; grep FAILED $OUT/suite.log | head -20
