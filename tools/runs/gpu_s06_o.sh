# Round 6: the early join (TT_EARLY_JOIN: the candidate tower joined at its
# input gradient, the query tower's weight gradients after the embedding
# update) — bit-identity tests, then the interleaved step A/B.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06o; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
step timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_model_gpu.py \
  -k "early_join or odd_hidden or igrad_first or dense_early or fused_dense_wgrad or graph_replay or train_steps_match" > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
grep -q " failed\| error" $OUT/tests.log && { grep -E "FAILED|Error" $OUT/tests.log | head -30; exit 1; }
bash tools/gpu_step_ab.sh 4 "ej1:TT_EARLY_JOIN=1:" "ej0:TT_EARLY_JOIN=0:"
