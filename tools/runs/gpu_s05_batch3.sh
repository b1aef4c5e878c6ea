# Round 5 batch 3: tt_route_fixed (one-workgroup route), tt_sparse_routed
# (sums / updates keyed by the route's own sort), tt_dense_adagrad_many:
# parity tests, the sharded step at 2048 / 16384 rows and the C5 leg, timed
# and profiled.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05b3; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_model_gpu.py \
  tests/test_distributed_gpu.py -m gpu -v -k "routed or route or sharded or adagrad or c5_100m or back_to_back or sparse" \
  --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 $OUT/t.log)"; grep -n "FAIL\|Error" $OUT/t.log | head; [ $rc -ne 0 ] && exit 0
for b in 2048 16384; do
timeout -k 10 300 python -u bench.py --train-mode sharded --batch $b --steps 100 --warmup 10 --no-index \
  --no-c5 --pipeline-rows 0 --no-cpu-baseline --no-uniform-gather > $OUT/sh$b.json 2> $OUT/sh$b.err; rc=$?
echo "sharded $b rc=$rc: $(python3 -c "import json;print(json.load(open('$OUT/sh$b.json'))['ms_per_step'])" 2>&1 | tail -1)"
[ $rc -ne 0 ] && exit 0
done
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --c5-only --steps 50 > $OUT/c5_$i.json 2> $OUT/c5_$i.err; rc=$?
echo "c5 $i rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/c5_$i.json'))['c5_sharded_table'];print(d['ms_per_step'], d['roofline']['frac'])" 2>&1 | tail -1)"
[ $rc -ne 0 ] && exit 0
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o c5 -- python3 bench.py --c5-only \
  --steps 20 > $OUT/c5p.json 2> $OUT/c5p.err; rc=$?
echo "prof c5 rc=$rc"; [ $rc -ne 0 ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_sh -o sh -- python3 bench.py \
  --train-mode sharded --batch 2048 --steps 50 --warmup 5 --no-index --no-c5 --pipeline-rows 0 --no-cpu-baseline \
  --no-uniform-gather > $OUT/shp.json 2> $OUT/shp.err; rc=$?
echo "prof sharded rc=$rc"
exit 0
