# Round 5: world-1 ShardedTrainStep — sharded parity tests (loss read from the
# graph's own scalar), then the loss through the single-device entry (default) vs the
# rows + columns entries (TT_WORLD1_FUSED=0) at 2048 and 16384 rows, interleaved.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05w1f; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_model_gpu.py -m gpu -v -k "sharded or world1 or rccl or graph" --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { grep -E "FAIL|Error" $OUT/t.log | head; tail -3 $OUT/t.log; exit 1; }
echo "sharded tests: $(tail -1 $OUT/t.log)"
for r in 1 2 3; do
  for B in 2048 16384; do
    for v in fused split; do
      E=""; [ $v = split ] && E="TT_WORLD1_FUSED=0"
      env $E timeout -k 10 150 python -u bench.py --steps 300 --warmup 30 --batch $B --train-mode sharded --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather --no-c5 > $OUT/$v.$B.$r.json 2> $OUT/$v.$B.$r.err || { tail -5 $OUT/$v.$B.$r.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/$v.$B.$r.json')); print('$v B=$B r$r', round(d['ms_per_step'],4))"
    done
  done
done
