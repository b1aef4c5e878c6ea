# Round 4: mlp_rows column groups (TT_MLP_COLSPLIT): MLP/model tests, step A/B, trace.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04o; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py -q -k "mlp or train_step or graph or paired or dense_early or score_matrix or fused or smoke" --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
bash tools/gpu_step_ab.sh 3 split:TT_MLP_COLSPLIT=1: whole:TT_MLP_COLSPLIT=0:
bash tools/gpu_trace_step.sh s04o
