# Round 4: mlp_wgrad with 64 x 128 output tiles (TT_WGRAD_JB=2: A re-read and
# converted half as often) against 64 x 64, same box.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04jb; mkdir -p $OUT
TT_WGRAD_JB=2 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py -q -k "mlp or wgrad or tower or train_step or c3" --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -q -k "runner_point_shape" --timeout 200 --timeout-method thread 2>&1 | tail -1
for v in 1 2; do echo "== JB=$v"; TT_WGRAD_JB=$v timeout -k 10 120 python -u tools/time_mlp.py 2>&1 | grep "wgrad tt"; done
bash tools/gpu_step_ab.sh 3 jb1:: jb2:TT_WGRAD_JB=2:
