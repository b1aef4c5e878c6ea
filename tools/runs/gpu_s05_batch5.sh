# Round 5: block_sum with two waves per block slot (D > 64 tables) — the
# sparse / train-step / sharded parity tests, a step trace, and step-time
# A/B against the HEAD tt_sparse.hip (tools/vlib/sp_base) with tools/gpu_step_ab.sh.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05b5; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py tests/test_model_gpu.py -m gpu -v -k "sparse or adagrad or adam or c2 or c3 or sharded or graphed or train or routed or scatter" --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { grep -E "FAIL|Error" $OUT/t.log | head -20; tail -5 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
bash tools/gpu_trace_step.sh b5 > /dev/null && cat gpurun_out/trace_b5/timeline.txt
bash tools/gpu_step_ab.sh 3 "new:-:--no-c5" "base:TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/sp_base/libtt.so:--no-c5"
