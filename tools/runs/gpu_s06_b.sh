# Round 6: the new / changed GPU tests first (route overflow sentinel, odd
# tower widths, trained-magnitude fp64 in-batch gradients, routed exchanges
# captured over RCCL at world 1), then the whole -m gpu suite.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  "tests/test_configs_gpu.py::test_c3_inbatch_grads_vs_fp64_after_training" \
  tests/test_kernels_gpu.py -k "route or routed or dense_stack or wgrad" > $OUT/new1.log 2>&1 || { tail -50 $OUT/new1.log; exit 1; }
tail -3 $OUT/new1.log; grep "score_max" $OUT/new1.log || true
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_model_gpu.py -k "sharded or rccl or graph" > $OUT/new2.log 2>&1 || { tail -50 $OUT/new2.log; exit 1; }
tail -3 $OUT/new2.log
bash tools/gpu_round.sh r06b tests
