# Round 4: gather — row-assembly form (TT_GATHER_ROWS=1) vs per-segment form and its knobs.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04m; mkdir -p $OUT
for r in 1 0; do
  TT_GATHER_ROWS=$r timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_pipeline_gpu.py -q -k "gather or train_steps or graph or golden or score_matrix" --timeout 200 --timeout-method thread -rf > $OUT/tests_$r.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests_$r.log | head -40; exit 1; }
  echo "rows=$r $(tail -1 $OUT/tests_$r.log)"
done
for rep in 1 2; do
  for v in rows seg g2564 g5122 g2568 g1284; do
    case $v in rows) export TT_GATHER_ROWS=1; unset TT_LIB_PATH;; seg) export TT_GATHER_ROWS=0; unset TT_LIB_PATH;; *) export TT_GATHER_ROWS=0 TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so;; esac
    echo "== $v $(timeout -k 10 120 python -u tools/time_gather.py --uniform 2>/dev/null | tr '\n' ' ')"
  done
done
