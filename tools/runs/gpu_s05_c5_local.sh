# ShardedTables.fetch_local / apply_local (world 1: by id, no route) — the
# local-vs-routed bit-identity test and the C5 tests — then the C5 leg local
# (default) vs routed on one stream (serial), interleaved.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05c5l; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "c5 or local or sharded" > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
echo "tests: $(tail -1 $OUT/t.log)"
for r in 1 2 3; do
  for v in local serial; do
    TT_C5_ORDER=$v timeout -k 10 150 python -u bench.py --c5-only --steps 50 --warmup 5 > $OUT/$v.$r.json 2> $OUT/$v.$r.err || { tail -5 $OUT/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v.$r.json'))['c5_sharded_table']; print('$v', $r, round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
  done
done
