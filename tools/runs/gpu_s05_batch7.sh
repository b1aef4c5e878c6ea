# Round 5: (1) index scan flush as rounds of one store per lane (TT_SCAN_FLUSH_LOOP)
# — bit-exact index tests, interleaved timing vs the per-register flush
# (tools/vlib/idx_flush16); (2) input-gradient-first tower backward
# (TT_IGRAD_FIRST) and the fused per-tower apply — model / config / pipeline
# parity tests and an interleaved step-time A/B of the four combinations.
set -e
# (index part done: profiles/r05_index_scan_ab.txt)
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05b7; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_pipeline_gpu.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { grep -E "FAIL|Error" $OUT/t.log | head -20; tail -5 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
bash tools/gpu_step_ab.sh 3 "old:TT_IGRAD_FIRST=0:--no-c5" "igf:TT_IGRAD_FIRST=1:--no-c5" "fused_old:TT_IGRAD_FIRST=0:--no-c5 --fused-apply" "fused_igf:TT_IGRAD_FIRST=1:--no-c5 --fused-apply"
