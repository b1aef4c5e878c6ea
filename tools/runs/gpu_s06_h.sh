# Round 6: the embedding update's join as a work list (block_sum lists the
# blocks where a continuing segment starts; a 128-workgroup join walks the
# list) — sparse / routed / train-step tests, then interleaved step A/B
# (TT_JOIN_LIST=0 / 1) and the C5 leg.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06h; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py -k "sparse or dedup or routed or adagrad or train_step or c5 or sharded" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/gpu_step_ab.sh 3 "list:TT_JOIN_LIST=1:" "perblock:TT_JOIN_LIST=0:"
for v in 1 0; do
  TT_JOIN_LIST=$v timeout -k 10 200 python -u bench.py --c5-only > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { tail -20 $OUT/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5_$v.json')); c=d.get('c5_sharded_table', d); print('c5 list=$v', round(c['ms_per_step'],4), round(c['roofline']['frac'],3))"
done
