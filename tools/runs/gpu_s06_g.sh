# Round 6: index chunk pipelining (finalize of chunk c beside the scan of
# chunk c + 1) — the bit-identity test, then interleaved A/B at 1M x k=100
# (TT_INDEX_PIPE=0 / 1); the x3 train-step test.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06g; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
step timeout -k 10 300 python -u -m pytest -v --timeout 280 --timeout-method thread \
  tests/test_configs_gpu.py -k "pipelined or x3" > $OUT/tests.log 2>&1
tail -4 $OUT/tests.log
for r in 1 2 3; do
  for v in 0 1; do
    TT_INDEX_PIPE=$v step timeout -k 10 120 python -u tools/time_index.py 1000000 100 3 > $OUT/ab_${v}_$r.txt 2>&1
    echo "pipe=$v $(tail -1 $OUT/ab_${v}_$r.txt)"
  done
done
