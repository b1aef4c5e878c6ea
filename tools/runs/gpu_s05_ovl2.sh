OUT=$GRAFT_REPO_ROOT/gpurun_out/s05ovl2; mkdir -p $OUT
timeout -k 10 120 python -u tools/graph_replay_overlap_probe.py > $OUT/probe.log 2>&1; rc=$?
echo "probe rc=$rc:"; grep -v "^$" $OUT/probe.log | tail -6
exit 0
