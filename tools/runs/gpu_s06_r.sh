# Round 6: a layer's weight-gradient sums inside the next input-gradient
# launch (TT_ROWS_SUM: tt_mlp_wgrad_partials + tt_mlp_rows_sum) — the
# bit-identity tests, then the interleaved step A/B.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06r; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
step timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_kernels_gpu.py \
  -k "rows_sum or odd_hidden or fused_dense_wgrad or igrad_first or dense_early or dense_stack or mlp_wgrad or graph_replay" > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
grep -q " failed\| error" $OUT/tests.log && { grep -E "FAILED|Error" $OUT/tests.log | head -30; exit 1; }
bash tools/gpu_step_ab.sh 4 "rs1:TT_ROWS_SUM=1:" "rs0:TT_ROWS_SUM=0:"
