# Round 6: kernel times of the reworked sparse update (block_sum / join) vs
# the previous tt_sparse.hip under rocprof on the train leg; the fused
# Dense-layer backward tests (fixed) and its interleaved step A/B.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06m; mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi; return 0; }
step timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_kernels_gpu.py \
  -k "fused_backward or dense_stack or mlp_wgrad or fused_dense_wgrad or igrad_first or paired_tower or graph_replay" > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
grep -q " failed\| error" $OUT/tests.log && { grep -E "FAILED|Error" $OUT/tests.log | head -30; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in new old fbwd; do
  case $v in
    new) envs="" ;;
    old) envs="TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/sparse_old/libtt.so" ;;
    fbwd) envs="TT_FUSED_BWD=1" ;;
  esac
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- python3 bench.py --steps 200 --warmup 20 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather > $OUT/prof_$v.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "prof $v rc=$rc"; tail -5 $OUT/prof_$v.log; exit 1; fi
  f=$(find $OUT/prof_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v $(grep -o '"ms_per_step": [0-9.]*' $OUT/prof_$v.log)"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
  n=r['Name']
  if any(x in n for x in ('block_sum','join_kernel','chunk_','mlp_','inbatch_pass_kernel<128, 0, false','combine')): print('   ', n[:70], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
"
  rm -f $OUT/prof_$v/*kernel_trace.csv
done
bash tools/gpu_step_ab.sh 4 "fbwd1:TT_FUSED_BWD=1:" "fbwd0:TT_FUSED_BWD=0:"
