# Round 5: the captured sharded step (fixed-capacity routing) and the C5 leg.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05sh; mkdir -p $OUT
COMMON="--no-index --pipeline-rows 0 --no-cpu-baseline --no-uniform-gather"
for B in 2048 16384; do
  TT_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --train-mode sharded --batch $B --steps 100 --warmup 10 $COMMON --no-c5 \
    > $OUT/sh_$B.json 2> $OUT/sh_$B.err; rc=$?
  echo "sharded B=$B rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/sh_$B.json'));print(d['ms_per_step'])" 2>/dev/null) $(grep 'host ms' $OUT/sh_$B.err)"
  [ $rc -ne 0 ] && exit 0
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 $COMMON > $OUT/c5.json 2> $OUT/c5.err; rc=$?
echo "c5 rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/c5.json'));c=d['c5_sharded_table'];print(c['ms_per_step'], c['roofline']['frac'], c['all_to_all_share'])" 2>/dev/null)"
[ $rc -ne 0 ] && exit 0
TT_BENCH_REHEARSE=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --index-queries 65536 --pipeline-rows 0 > $OUT/reh2.json 2> $OUT/reh2.err; rc=$?
echo "rehearse-2 rc=$rc: $(head -c 600 $OUT/reh2.json)"
exit 0
