# Round 5: world-1 sharded step reading the shard directly (no fetch), the
# fused route with its id loads issued together; sharded / route tests,
# route phase times, the sharded step at 2048 / 16384 and C5.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05r4; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_model_gpu.py \
  tests/test_distributed_gpu.py -m gpu -v -k "sharded or rccl or global or route or routed or c5" --timeout 200 \
  --timeout-method thread > $OUT/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 $OUT/t.log)"; grep -n "FAIL\|Error" $OUT/t.log | head; [ $rc -ne 0 ] && exit 0
TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/r05stamps/libtt.so timeout -k 10 120 python -u tools/time_route.py 2048 > $OUT/st.log 2>&1 || { tail -5 $OUT/st.log; exit 0; }
grep -v amdgpu.ids $OUT/st.log
for r in 1 2; do
for b in 2048 16384; do
timeout -k 10 300 python -u bench.py --train-mode sharded --batch $b --steps 100 --warmup 10 --no-index \
  --no-c5 --pipeline-rows 0 --no-cpu-baseline --no-uniform-gather > $OUT/sh$b$r.json 2> $OUT/sh$b$r.err; rc=$?
echo "sharded $b rc=$rc: $(python3 -c "import json;print(json.load(open('$OUT/sh$b$r.json'))['ms_per_step'])" 2>&1 | tail -1)"
[ $rc -ne 0 ] && exit 0
done
done
exit 0
