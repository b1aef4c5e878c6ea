# Round 4: sharded step with the bucket all_reduce + dense Adagrad inside the
# captured middle and one route-index copy per step, against HEAD's package
# (tools/pbin/wt), world 1, interleaved.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04w; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_model_gpu.py -q -k "sharded or global or capture or c5" --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for B in 2048 16384; do
    for v in new head; do
      root=$GRAFT_REPO_ROOT; [ $v = head ] && root=$GRAFT_REPO_ROOT/tools/pbin/wt
      timeout -k 10 300 python -u $root/bench.py --train-mode sharded --batch $B --steps 100 --warmup 10 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather --no-c5 > $OUT/$v$B.json 2> $OUT/$v$B.err
      python -c "import json; d=json.load(open('$OUT/$v$B.json')); print('$v B=$B', round(d['ms_per_step'],4))"
    done
  done
done
