# Round 5: (1) do back-to-back replays of one graph overlap?  (2) the sharded
# step without the route's counts kept alive (TT_SHARDED_KEEP=0), twice.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05ovl; mkdir -p $OUT
timeout -k 10 120 python -u tools/graph_replay_overlap_probe.py > $OUT/probe.log 2>&1; rc=$?
echo "probe rc=$rc:"; cat $OUT/probe.log | grep fork
for i in 1 2; do
TT_SHARDED_KEEP=0 timeout -k 10 300 python -u bench.py --train-mode sharded --batch 2048 --steps 100 --warmup 10 --no-index \
  --no-c5 --pipeline-rows 0 --no-cpu-baseline --no-uniform-gather > $OUT/nk$i.json 2> $OUT/nk$i.err; rc=$?
echo "no-keep $i rc=$rc: $(grep -m1 'overflowed' $OUT/nk$i.err)"
done
exit 0
