# Round 5: which single earlier test makes the in-process graphed fit crash.
# One pytest process per (test, fit) pair, the most recent tests first; the
# first crash ends the call.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05seg3; mkdir -p $OUT
FIT=tests/test_pipeline_gpu.py::test_graphed_device_fit_equals_eager_host_fit
i=0
for t in $(tac tools/runs/s05_model_tests.txt); do
  i=$((i+1))
  TT_TEST_IN_CHILD=1 TT_SEGV_BT=$OUT/bt_$i.txt timeout -k 10 200 python -u -m pytest "$t" $FIT -m gpu -x -q \
    --timeout 120 --timeout-method thread > $OUT/run_$i.log 2>&1
  rc=$?
  echo "$i $t rc=$rc: $(tail -1 $OUT/run_$i.log)"
  [ $rc -ne 0 ] && break
done
exit 0
