# Round 5: the fused per-tower apply with its id sorts issued right after the
# gather (TT_FUSED_SORT_EARLY=1) — model parity tests, then an interleaved
# step A/B: default (unfused), fused early sorts, fused early sorts + the
# embedding update at the input gradient (TT_IGRAD_FIRST=1), fused late sorts.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05fab; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -m gpu -v -k "fused or igrad or dense_early or graphed or paired" --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { grep -E "FAIL|Error" $OUT/t.log | head; tail -3 $OUT/t.log; exit 1; }
echo "model tests: $(tail -1 $OUT/t.log)"
bash tools/gpu_step_ab.sh 3 "unfused:-:--no-c5" "fused_early:-:--no-c5 --fused-apply" "fused_early_igf:TT_IGRAD_FIRST=1:--no-c5 --fused-apply" "fused_late:TT_FUSED_SORT_EARLY=0:--no-c5 --fused-apply"
