# Round 5: the sharded step's overflow word without per-step syncs: canaries
# around it and the running max of the owner counts inside the graph.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05dbg2; mkdir -p $OUT
for i in 1 2; do
TT_SHARDED_DEBUG=2 timeout -k 10 300 python -u bench.py --train-mode sharded --batch 2048 --steps 100 --warmup 10 --no-index \
  --no-c5 --pipeline-rows 0 --no-cpu-baseline --no-uniform-gather > $OUT/g$i.json 2> $OUT/g$i.err; rc=$?
echo "global $i rc=$rc: $(grep -m2 'debug\|overflowed' $OUT/g$i.err)"
done
exit 0
