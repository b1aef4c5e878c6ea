# Round 4: does the runner-point-shape index test leave the process in a state
# where a later graphed fit aborts?  One pytest process each, stop at the first failure.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04repro; mkdir -p $OUT
TT_GPU_TEST_RUNNER_SHAPE=1 timeout -k 10 400 python -u -X faulthandler -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -v -k "runner_point_shape or graphed_device_fit" --timeout 300 --timeout-method thread > $OUT/a.log 2>&1 && echo "A ok: $(tail -1 $OUT/a.log)" || { echo "A failed"; grep -E "PASSED|FAILED|Fatal|Error" $OUT/a.log | head; exit 1; }
timeout -k 10 400 python -u -X faulthandler -m pytest tests/test_pipeline_gpu.py -v -k "graphed_device_fit" --timeout 300 --timeout-method thread > $OUT/b.log 2>&1 && echo "B ok: $(tail -1 $OUT/b.log)" || { echo "B failed"; grep -E "PASSED|FAILED|Fatal" $OUT/b.log | head; exit 1; }
