# Round 5: new autograd score-matrix tests + index parity, a step trace, and
# the scan's filter-B placement A/B (idx_early = filter B before the barrier).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05b4; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -m gpu -v -k "score_matrix or call" --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
bash tools/gpu_trace_step.sh b4 > /dev/null && tail -60 gpurun_out/trace_b4/timeline.txt
bash tools/runs/gpu_s05_idx_ab2.sh idxab4 idx_early
