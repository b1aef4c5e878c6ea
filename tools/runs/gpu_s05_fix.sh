# Round 5: (1) the full -m gpu suite exactly as the driver runs it (graphed
# fits in-process); (2) the standalone RCCL-graph-lifetime reproduction, the
# fixed order then the old order (a crash there ends the call: last step).
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05fix2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/suite.log 2>&1; rc=$?
echo "suite rc=$rc: $(tail -1 $OUT/suite.log)"; [ $rc -ne 0 ] && exit 0
timeout -k 10 120 python -u tools/repro_rccl_graph_after_pg.py --order fixed > $OUT/repro_fixed.log 2>&1; rc=$?
echo "repro fixed rc=$rc: $(tail -1 $OUT/repro_fixed.log)"; [ $rc -ne 0 ] && exit 0
timeout -k 10 120 python -u tools/repro_rccl_graph_after_pg.py --order old > $OUT/repro_old.log 2>&1; rc=$?
echo "repro old rc=$rc: $(tail -2 $OUT/repro_old.log | tr '\n' ' ')"
exit 0
