# Round 6: the sharded step's tests with the route buffers no
# longer pinned (the TT_SHARDED_KEEP pin is gone) and the canary / overflow
# word checked after every call (TT_SHARDED_DEBUG=1), graphed, world 1
# (ROUTE_SIDE on and off).
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06f; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
export TT_SHARDED_DEBUG=1
step timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_model_gpu.py tests/test_distributed_gpu.py tests/test_pipeline_gpu.py -k "sharded or rccl or global or c5 or graph or fit" > $OUT/keep0.log 2>&1
tail -3 $OUT/keep0.log; grep -c PASSED $OUT/keep0.log; grep "FAILED\|canary" $OUT/keep0.log | head
TT_SHARDED_ROUTE_SIDE=0 step timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_model_gpu.py -k "sharded or rccl" > $OUT/keep0_noside.log 2>&1
tail -3 $OUT/keep0_noside.log
step timeout -k 10 300 python -u -m pytest -v --timeout 280 --timeout-method thread tests/test_configs_gpu.py -k "c5 or sharded" > $OUT/keep0_c5.log 2>&1
tail -3 $OUT/keep0_c5.log
