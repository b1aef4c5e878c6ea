# World-1 route slots laid out by the head / write passes (default) vs the
# route_pad launch (TT_ROUTE_W1_SLOTS=0): route tests, then the C5 leg and the
# world-1 sharded step interleaved.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05rw1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_distributed_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "route or sharded or world1" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
echo "tests: $(tail -1 $OUT/t.log)"
for r in 1 2 3; do
  for v in w1 pad; do
    E=""; [ $v = pad ] && E="TT_ROUTE_W1_SLOTS=0"
    env $E timeout -k 10 150 python -u bench.py --c5-only --steps 50 --warmup 5 > $OUT/c5.$v.$r.json 2> $OUT/c5.$v.$r.err || { tail -3 $OUT/c5.$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c5.$v.$r.json'))['c5_sharded_table']; print('c5 $v', $r, round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
    env $E timeout -k 10 150 python -u bench.py --steps 300 --warmup 30 --batch 16384 --train-mode sharded --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather --no-c5 > $OUT/sh.$v.$r.json 2> $OUT/sh.$v.$r.err || { tail -3 $OUT/sh.$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/sh.$v.$r.json')); print('sharded16384 $v', $r, round(d['ms_per_step'],4))"
  done
done
