# Round 5: kernel breakdown of the captured sharded step (world 1, 2,048 rows)
# and of the C5 leg; the new route / C3-scale sharded tests first.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05psh; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -m gpu -v -k "route or sharded_step" \
  --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 $OUT/t.log)"; grep -n "FAIL\|Error" $OUT/t.log | head; [ $rc -ge 124 ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_sh -o sh -- python3 bench.py --train-mode sharded --batch 2048 \
  --steps 50 --warmup 5 --no-index --no-c5 --pipeline-rows 0 --no-cpu-baseline --no-uniform-gather > $OUT/sh.json 2> $OUT/sh.err; rc=$?
echo "prof sharded rc=$rc"; [ $rc -ne 0 ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o c5 -- python3 bench.py --c5-only --steps 20 > $OUT/c5.json 2> $OUT/c5.err; rc=$?
echo "prof c5 rc=$rc: $(cat $OUT/c5.json | head -c 300)"
find $OUT -name "*kernel_stats.csv" | head
exit 0
