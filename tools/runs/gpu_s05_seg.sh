# Round 5: which earlier tests make the in-process graphed DeviceDataset fit
# crash (TT_TEST_IN_CHILD=1), with a native backtrace on the crash
# (TT_SEGV_BT).  Subsets first; the first crash ends the call.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05seg2; mkdir -p $OUT
FIT=tests/test_pipeline_gpu.py::test_graphed_device_fit_equals_eager_host_fit
run() {  # name, test ids...
  local name=$1; shift
  TT_TEST_IN_CHILD=1 TT_SEGV_BT=$OUT/bt_$name.txt timeout -k 10 400 python -u -m pytest "$@" -m gpu -x -v \
    --timeout 120 --timeout-method thread > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 $OUT/$name.log)"
  return $rc
}
run model tests/test_model_gpu.py $FIT &&
run kernels tests/test_kernels_gpu.py $FIT &&
run dist tests/test_distributed_gpu.py $FIT &&
run configs tests/test_configs_gpu.py $FIT &&
run full tests
exit 0
