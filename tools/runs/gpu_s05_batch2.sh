# Round 5 batch 2: (a) the sharded step with the route counts zeroed by a
# kernel and NOT kept alive; (b) route / sharded / back-to-back replay tests;
# (c) index per-row bound: bit-exact tests + A/B vs the round-start library;
# (d) kernel profiles of the sharded step and the C5 leg.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05b2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
TT_SHARDED_KEEP=0 timeout -k 10 300 python -u bench.py --train-mode sharded --batch 2048 --steps 100 --warmup 10 --no-index \
  --no-c5 --pipeline-rows 0 --no-cpu-baseline --no-uniform-gather > $OUT/nk$i.json 2> $OUT/nk$i.err; rc=$?
echo "no-keep kernel-zeroed $i rc=$rc: $(grep -m1 'overflowed' $OUT/nk$i.err) $(python3 -c "import json;print(json.load(open('$OUT/nk$i.json'))['ms_per_step'])" 2>/dev/null)"
[ $rc -ge 124 ] && exit 0
done
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_model_gpu.py -m gpu -v \
  -k "route or sharded or back_to_back or rccl or adagrad_rows or c5_100m" --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 $OUT/t.log)"; grep -n "FAIL" $OUT/t.log | head; [ $rc -ge 124 ] && exit 0
bash tools/runs/gpu_s05_idx.sh
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_sh -o sh -- python3 bench.py --train-mode sharded --batch 2048 \
  --steps 50 --warmup 5 --no-index --no-c5 --pipeline-rows 0 --no-cpu-baseline --no-uniform-gather > $OUT/sh.json 2> $OUT/sh.err; rc=$?
echo "prof sharded rc=$rc"; [ $rc -ne 0 ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o c5 -- python3 bench.py --c5-only --steps 20 > $OUT/c5.json 2> $OUT/c5.err; rc=$?
echo "prof c5 rc=$rc: $(head -c 400 $OUT/c5.json)"
exit 0
