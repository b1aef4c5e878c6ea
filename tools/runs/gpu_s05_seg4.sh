# Round 5: (1) the capturable sharded step's tests; (2) the fit crash with HIP
# error logging on and the live-graph count per test (expected crash: last).
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05seg4; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py tests/test_configs_gpu.py -m gpu -v \
  -k "sharded or rccl or c5 or integration" --timeout 200 --timeout-method thread > $OUT/sharded.log 2>&1; rc=$?
echo "sharded rc=$rc: $(tail -1 $OUT/sharded.log)"
[ $rc -ge 124 ] && exit 0
AMD_LOG_LEVEL=1 TT_SEGV_BT=$OUT/bt.txt timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_pipeline_gpu.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > $OUT/a.log 2>&1; rc=$?
echo "rc=$rc: $(tail -1 $OUT/a.log)"
grep -n "hipGraph\|parallel\|Failed\|error" $OUT/a.log | head -20
grep "live CUDAGraph" $OUT/bt.txt | tail -40
exit 0
