# Round 6: one launch per Dense layer in the towers' backward
# (tt_mlp_backward_layer: weight-gradient partials + the layer below's input
# gradient + the upper layer's sums/Adagrad; TT_FUSED_BWD) — the bit-identity
# tests, then the interleaved step A/B.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06l; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
step timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_kernels_gpu.py \
  -k "fused_backward or dense_stack or mlp_wgrad or fused_dense_wgrad or igrad_first or paired_tower or graph_replay" > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
grep -q " failed\| error" $OUT/tests.log && { grep -E "FAILED|Error|assert" $OUT/tests.log | head -30; exit 1; }
bash tools/gpu_step_ab.sh 4 "fbwd1:TT_FUSED_BWD=1:" "fbwd0:TT_FUSED_BWD=0:"
