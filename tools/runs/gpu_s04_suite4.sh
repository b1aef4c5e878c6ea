# Round 4: the full -m gpu suite with the runner-point-shape index test back in.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04suite4; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/suite.log 2>&1
echo "rc=$?: $(tail -1 $OUT/suite.log)"
grep -n "runner_point_shape\|Fatal" $OUT/suite.log | head
exit 0
