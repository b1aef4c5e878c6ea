# Round 5: route sort onesweep vs merge (TT_ROUTE_SORT) on the C5 leg and the
# sharded step; route parity under onesweep; the sharded step after the
# world-1 bucket skip.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05r3; mkdir -p $OUT
TT_ROUTE_SORT=onesweep timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -v -k "route or routed" \
  --timeout 120 --timeout-method thread > $OUT/t1.log 2>&1; rc=$?
echo "route tests (onesweep) rc=$rc: $(tail -1 $OUT/t1.log)"; [ $rc -ne 0 ] && exit 0
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py tests/test_model_gpu.py tests/test_distributed_gpu.py -m gpu -v \
  -k "sharded or rccl or global" --timeout 200 --timeout-method thread > $OUT/t2.log 2>&1; rc=$?
echo "sharded tests rc=$rc: $(tail -1 $OUT/t2.log)"; grep -n "FAIL\|Error" $OUT/t2.log | head; [ $rc -ne 0 ] && exit 0
for r in 1 2; do
for v in merge onesweep; do
TT_ROUTE_SORT=$v timeout -k 10 300 python3 -u bench.py --c5-only --steps 50 > $OUT/c5_$v$r.json 2> $OUT/c5_$v$r.err; rc=$?
echo "c5 $v $r rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/c5_$v$r.json'))['c5_sharded_table'];print(d['ms_per_step'], d['roofline']['frac'])" 2>&1 | tail -1)"
[ $rc -ne 0 ] && exit 0
done
for b in 2048 16384; do
TT_ROUTE_SORT=merge timeout -k 10 300 python -u bench.py --train-mode sharded --batch $b --steps 100 --warmup 10 --no-index \
  --no-c5 --pipeline-rows 0 --no-cpu-baseline --no-uniform-gather > $OUT/sh$b$r.json 2> $OUT/sh$b$r.err; rc=$?
echo "sharded $b rc=$rc: $(python3 -c "import json;print(json.load(open('$OUT/sh$b$r.json'))['ms_per_step'])" 2>&1 | tail -1)"
[ $rc -ne 0 ] && exit 0
done
done
exit 0
